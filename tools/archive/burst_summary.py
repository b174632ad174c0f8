"""Table of tools/txburst rows (us per burst) beside the reference CPU loop
(bench.cpu_burst JSON): python3 tools/burst_summary.py txburst.log cpu_burst.json"""
import json
import sys

rows = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
cb = {}
if len(sys.argv) > 2:
    cpu = json.load(open(sys.argv[2]))
    cb = {(r["pkt_len"], r["burst"]): r["us_per_burst"] for r in cpu["rows"]}
modes = ["rx_verify_registered", "rx_verify_registered_server", "rx_window_registered",
         "rx_window_registered_server", "tx_fill_registered", "tx_fill_registered_server"]
by = {}
for r in rows:
    if "burst" in r and r.get("mode") in modes:
        by.setdefault((r["pkt_len"], r["burst"]), {})[r["mode"]] = r
print("%5s %5s %9s %9s %9s %9s %9s %9s %9s %8s" % ("len", "burst", "verify", "verify_s", "window", "window_s",
                                                 "calls_s", "tx", "tx_s", "cpu"))
for k in sorted(by):
    g = by[k]
    f = lambda m: "%9.2f" % g[m]["us_median"] if m in g else "%9s" % "-"
    calls = g.get("rx_window_registered_server", {}).get("us_calls")
    print("%5d %5d %s %s %s %s %9s %s %s %8.2f" % (k[0], k[1], f(modes[0]), f(modes[1]), f(modes[2]), f(modes[3]),
                                                    "%.2f" % calls if calls is not None else "-", f(modes[4]),
                                                    f(modes[5]), cb.get(k, float("nan"))))
for r in rows:
    if "burst" not in r or r.get("mode", "").startswith("in_cksum"):
        print(r)
