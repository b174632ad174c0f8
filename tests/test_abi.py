"""The C-ABI library loads and exports every symbol include/cgck.h declares.
No compute calls here (no GPU in the build container)."""
import ctypes
import os
import re

import pytest

import cgck

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, "include", "cgck.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"^\s*typedef[^;]*;", "", src, flags=re.M)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*\b([a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(n for n in names if n not in ("sizeof",)))


def test_header_declares_expected_set():
    assert set(declared_functions()) == set(cgck.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = cgck.load()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.cgck_abi_version() == 2


def test_drop_in_prototypes_match_reference():
    """in_cksum/udp_cksum keep subr.h:373-374's prototypes."""
    ref = open("/root/reference/subr.h").read() if os.path.exists("/root/reference/subr.h") else None
    hdr = open(os.path.join(ROOT, "include", "cgck.h")).read()
    assert "uint16_t in_cksum(void *data, int len);" in hdr
    assert "uint16_t udp_cksum(struct ip *ip, int len);" in hdr
    if ref is not None:
        assert "uint16_t in_cksum(void *, int);" in ref
        assert "uint16_t udp_cksum(struct ip *, int);" in ref


def test_rss_drop_in_prototypes_match_reference():
    """toeplitz_hash/rss_hash4 keep subr.h:370-371's prototypes (u_char is
    unsigned char, be32_t/be16_t are uint32_t/uint16_t, subr.h:183-184)."""
    hdr = open(os.path.join(ROOT, "include", "cgck.h")).read()
    assert ("uint32_t toeplitz_hash(const unsigned char *data, int cnt, const unsigned char *key, "
            "int key_size);") in hdr
    assert "uint32_t rss_hash4(uint32_t laddr, uint32_t faddr, uint16_t lport, uint16_t fport," in hdr
    if os.path.exists("/root/reference/subr.h"):
        ref = open("/root/reference/subr.h").read()
        assert "uint32_t toeplitz_hash(const u_char *, int, const u_char *, int);" in ref
        assert "uint32_t rss_hash4(be32_t, be32_t, be16_t, be16_t, u_char *, int);" in ref


def test_dst_layout():
    assert cgck.DST_DTYPE.itemsize == 16
    assert ctypes.sizeof(cgck.DstParams) == 40   # 16 + 2 + 1 + 1, pad, pointer, int, pad


def test_desc_layout():
    assert cgck.DESC_DTYPE.itemsize == 12
    assert cgck.DESC_DTYPE.fields["l3_off"][1] == 8
    assert cgck.DESC_DTYPE.fields["ip_len"][1] == 10


def test_no_device_fails_loudly():
    """Without a GPU the engine refuses (no silent CPU path)."""
    if cgck.device_count() > 0:
        pytest.skip("a device is visible")
    with pytest.raises(cgck.CgckError, match="no HIP device"):
        cgck.Engine(0)


def test_imix_bytes():
    L = cgck.load()
    assert L.cgck_imix_bytes(12) == 4252
    assert L.cgck_imix_bytes(1) == 64
    assert L.cgck_imix_bytes(7) == 2908
    assert L.cgck_imix_bytes(16 * 12) == 16 * 4252


def test_library_has_gfx950_code_object():
    so = cgck.LIB_PATH
    data = open(so, "rb").read()
    assert b"gfx950" in data
