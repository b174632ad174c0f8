"""Table of tools/txloop rows: per (mix, stack budget) and burst, the worker's
us per burst processed for each form (its checksum-path time over the bursts
it processed: the coalesced form opens several bursts in some iterations and
none in others), the waits and the latencies.

    python3 tools/loop_table.py gpurun_out/r5b/txloop.log
"""
import json
import sys

rows = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
loop = [r for r in rows if r["mode"] == "loop"]
cells = sorted({(r["mix"], r["stack_ns_per_frame"], r["stack_us_fixed"]) for r in loop})
forms = ("reference", "pipelined", "coalesced", "sync")
for c in cells:
    print("%s, stack work %s" % (c[0], "%g us a burst" % c[2] if c[2] else "%g ns a frame" % c[1]))
    print("%6s %9s %9s %9s %9s | %7s %7s | %8s %8s %8s | %s" % ("burst", "ref", "pipe", "coal", "sync", "p_wait",
                                                                "c_wait", "p_lat", "c_lat", "s_lat", "exact"))
    for b in sorted({r["burst"] for r in loop}):
        g = {r["form"]: r for r in loop if (r["mix"], r["stack_ns_per_frame"], r["stack_us_fixed"]) == c
             and r["burst"] == b}
        print("%6d %9.3f %9.3f %9.3f %9.3f | %7.2f %7.2f | %8.2f %8.2f %8.2f | %s" % (
            b, *(g[f]["us_per_burst"] for f in forms), g["pipelined"]["us_wait"], g["coalesced"]["us_wait"],
            g["pipelined"]["us_latency"], g["coalesced"]["us_latency"], g["sync"]["us_latency"],
            all(x["exact"] for x in g.values())))
    print()
print("lone burst (drain rule), post to window end:",
      {r["burst"]: r["us_latency"] for r in rows if r["mode"] == "lone"})
