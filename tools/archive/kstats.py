#!/usr/bin/env python3
"""Register/LDS/scratch usage and static VALU count per kernel from the
device assembly (make -C con-gen_amd asm)."""
import glob
import os
import re
import sys

d = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(__file__), "..", "con-gen_amd", "build")
for f in sorted(glob.glob(os.path.join(d, "*.s"))):
    txt = open(f).read()
    for m in re.finditer(r"\n(_Z\w+):[^\n]*\n(.*?)s_endpgm", txt, re.S):
        name, body = m.group(1), m.group(2)
        valu = len(re.findall(r"^\s+v_", body, re.M))
        i = txt.find(".name:           " + name)
        meta = None
        if i >= 0:
            k = txt.rfind("\n  - ", 0, i)
            j = txt.find("\n  - ", i)
            meta = txt[k:j if j > 0 else len(txt)]
        md = meta or ""
        g = lambda k: (re.search(r"\." + k + r":\s+(\d+)", md) or [None, "?"])[1]
        if "probe" in name:
            continue
        print(f"{name[:60]:60s} vgpr {g('vgpr_count'):>4} sgpr {g('sgpr_count'):>4} "
              f"lds {g('group_segment_fixed_size'):>6} scratch {g('private_segment_fixed_size'):>4} valu {valu}")
