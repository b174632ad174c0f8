"""The pipelined-window table of DESIGN.md §5.3 / INTEGRATION.md §3 from a
tools/txburst log: per frame size and burst, the worker thread's
microseconds per burst with one burst in flight (RX window, TX fill with its
calls / post / wait split) beside the same binary's reference loop.

usage: python tools/burst_table.py profiles/r04/burst/<log> [bursts]
"""
import json
import sys


def load(path):
    rows = {}
    with open(path) as f:
        for line in f:
            try:
                d = json.loads(line)
            except ValueError:
                continue
            if "pkt_len" in d and "burst" in d:
                rows.setdefault(d["mode"], {})[(d["pkt_len"], d["burst"])] = d
    return rows


def main():
    rows = load(sys.argv[1])
    bursts = [int(b) for b in sys.argv[2].split(",")] if len(sys.argv) > 2 else [32, 256, 2048]
    rx, rr = rows["rx_window_pipelined_registered_server"], rows["rx_reference_loop"]
    tx, tr = rows["tx_fill_pipelined_registered_server"], rows["tx_reference_loop"]
    print("| frames | burst | RX window, pipelined | RX reference loop "
          "| TX fill, pipelined (calls / post / wait); p10-p90 | TX reference loop |")
    print("|---|---|---|---|---|---|")
    for ln in (64, 576, 1500):
        for b in bursts:
            x, t = rx[(ln, b)], tx[(ln, b)]
            split = ""
            if "us_calls" in t:
                split = f" ({t['us_calls']:.2f} / {t['us_post']:.2f} / {t['us_wait']:.2f})"
            spread = f"; {t['us_p10']:.1f}-{t['us_p90']:.1f}" if "us_p10" in t else ""
            print(f"| {ln} B | {b} | {x['us_median']:.2f} | {rr[(ln, b)]['us_median']:.2f} "
                  f"| {t['us_median']:.2f}{split}{spread} | {tr[(ln, b)]['us_median']:.2f} |")


if __name__ == "__main__":
    main()
