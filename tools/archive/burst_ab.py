#!/usr/bin/env python3
"""Side-by-side of tools/txburst logs (one per configuration): for each
packet length and burst, the registered RX window through the launch path
and through the burst server, per log.

    python tools/burst_ab.py A.log B.log ...
"""
import json
import sys


def load(path):
    rows = {}
    for line in open(path):
        if line.startswith("{"):
            r = json.loads(line)
            rows[(r["mode"], r["pkt_len"], r["burst"])] = r["us_median"]
    return rows


def main():
    logs = [(p, load(p)) for p in sys.argv[1:]]
    modes = ("rx_window_registered", "rx_window_registered_server", "rx_verify_registered_server",
             "rx_window_server")
    keys = sorted({(k[1], k[2]) for _, rows in logs for k in rows if k[0] in modes})
    print("len  burst  " + "  ".join(f"{p.split('/')[-1]}:{m.replace('rx_', '').replace('registered', 'reg')}"
                                     for p, _ in logs for m in modes))
    for ln, b in keys:
        cells = []
        for _, rows in logs:
            for m in modes:
                v = rows.get((m, ln, b))
                cells.append(f"{v:8.2f}" if v is not None else "       -")
        print(f"{ln:4d} {b:6d}  " + "  ".join(cells))
    for p, rows in logs:
        ic = rows.get(("in_cksum_server", 20, 1))
        print(f"{p}: in_cksum_server {ic}")


if __name__ == "__main__":
    main()
