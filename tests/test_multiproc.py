"""N > 1 path of bench.py on the CPU (gloo, world size 2): the batch split
has no data-path collective; ranks own disjoint contiguous packet ranges with
their own generator seeds, and timing is the max over ranks behind barriers
(SURVEY §8(e))."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    d = bench.Dist()
    plan = bench.shard_plan(d.rank, d.world, 1000)
    d.barrier()
    m = d.max(float(rank + 1) * 0.5)   # per-rank "elapsed": max must win
    q.put((rank, plan, m))
    d.close()


def test_two_rank_shard_plan_and_max():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, p0, m0), (r1, p1, m1) = res
    assert (p0["first"], p0["n"]) == (0, 1000) and (p1["first"], p1["n"]) == (1000, 1000)
    assert p0["seed"] != p1["seed"]                      # independent shards
    assert m0 == m1 == 1.0                               # max over ranks


def _worker4(rank, world, port, q):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                       "RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    d = bench.Dist()
    plan = bench.shard_plan(d.rank, d.world, 4096)
    tot = d.sum(rank + 1)                   # per-rank parity counts are summed
    devs = d.gather({"rank": rank, "device": rank})
    q.put((rank, plan, tot, devs))
    d.close()


def test_four_rank_plan_covers_batch_disjointly():
    """configs[4] at 4 ranks: the shards tile [0, 4n) exactly once, each rank
    has its own seed, the checker's totals are summed and every rank's device
    id is gathered (the line records them)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker4, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=120) for _ in procs), key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    covered = []
    for rank, plan, tot, devs in res:
        covered.extend(range(plan["first"], plan["first"] + plan["n"]))
        assert tot == 1 + 2 + 3 + 4
        assert [d["device"] for d in devs] == [0, 1, 2, 3]
    assert sorted(covered) == list(range(4 * 4096))
    assert len({plan["seed"] for _, plan, _, _ in res}) == 4


def test_device_for_refuses_oversubscription():
    assert [bench.device_for(r, 8, 8) for r in range(8)] == list(range(8))
    with pytest.raises(SystemExit, match="WORLD_SIZE 2 > 1 visible GPUs"):
        bench.device_for(1, 2, 1)
    assert bench.device_for(1, 2, 1, allow_shared=True) == 0
    with pytest.raises(SystemExit, match="no GPU visible"):
        bench.device_for(0, 1, 0)


def test_burst_summary_is_compact():
    modes = [m for _, m in bench.BURST_MODES + bench.BURST_REF]
    rows = [{"mode": m, "pkt_len": ln, "burst": b, "us_median": 1.0 + i}
            for i, m in enumerate(modes) for ln in bench.BURST_LENS for b in bench.BURSTS]
    cpu = {"rows": [{"pkt_len": ln, "burst": b, "us_per_burst": 2.0} for ln in bench.BURST_LENS for b in bench.BURSTS]}
    s = bench.burst_summary(rows, cpu)
    assert len(s) <= 10
    for r in s:
        assert len(r) == len(bench.BURST_COLS) and r[-1] == 2.0
        assert r[2:-1] == [1.0 + i for i in range(len(modes))]   # each column its own routing, no minimum


def test_burst_crossover():
    """The crossover is the first burst of the final winning run, per
    routing: a GPU win at a small burst followed by a loss does not count,
    and one routing's win is not credited to another."""
    B = bench.BURSTS
    gpu = {64: [9.0] * len(B), 576: [1.0] + [9.0] * (len(B) - 3) + [1.0, 1.0], 1500: [1.0] * len(B)}
    rows = [{"mode": "rx_window_registered", "pkt_len": ln, "burst": b, "us_median": gpu[ln][i]}
            for ln in gpu for i, b in enumerate(B)]
    rows += [{"mode": "rx_window_registered_server", "pkt_len": 64, "burst": B[-1], "us_median": 1.0}]
    cpu = {"rows": [{"pkt_len": ln, "burst": b, "us_per_burst": 2.0} for ln in gpu for b in B]}
    x = bench.burst_crossover(rows, cpu)
    assert x["64"]["rx_window_launch"] is None
    assert x["64"]["rx_window_server"] == B[-1]   # the server row wins at the largest burst only
    assert x["576"]["rx_window_launch"] == B[-2]
    assert x["1500"]["rx_window_launch"] == B[0]
    assert x["1500"]["tx_fill_pipelined"] is None    # no TX rows measured
    assert bench.burst_crossover({"error": "x"}, cpu) is None


def test_single_rank_is_noop():
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    d = bench.Dist()
    assert d.world == 1 and d.max(3.0) == 3.0
    d.barrier()
    d.close()


def test_cpu_burst_leg_runs():
    """bench.py's CPU burst baseline (oracle as the timed reference loop, one
    pinned core) produces a row per packet length and burst size."""
    r = bench.cpu_burst()
    assert r["cores"] == 1 and r["kind"] in ("reference", "port")
    assert {(x["pkt_len"], x["burst"]) for x in r["rows"]} == {(ln, b) for ln in bench.BURST_LENS for b in bench.BURSTS}
    assert all(x["us_per_burst"] > 0 for x in r["rows"])


def test_launch_decision():
    """--gpus 1 (or no flag) stays in-process; --gpus N > 1 without a launcher
    spawns N ranks; under a launcher --gpus must equal WORLD_SIZE."""
    assert bench.launch_decision(None, {}) == ("inprocess", 1)
    assert bench.launch_decision(1, {}) == ("inprocess", 1)
    assert bench.launch_decision(2, {}) == ("spawn", 2)
    assert bench.launch_decision(8, {}) == ("spawn", 8)
    assert bench.launch_decision(8, {"WORLD_SIZE": "8"}) == ("inprocess", 8)
    assert bench.launch_decision(None, {"WORLD_SIZE": "4"}) == ("inprocess", 4)
    with pytest.raises(SystemExit, match="--gpus 8 but WORLD_SIZE 2"):
        bench.launch_decision(8, {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit, match="--gpus 2 but WORLD_SIZE 1"):
        bench.launch_decision(2, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.launch_decision(0, {})


def test_child_command_is_torchrun_on_loopback():
    cmd = bench.child_command(4, ["--gpus", "4", "--steps", "3"], 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-5].endswith("bench.py") and cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def test_spawn_relays_rank0_line(monkeypatch, capsys):
    """spawn_ranks runs the child, passes the one JSON line to stdout and
    everything else to stderr, and returns the child's exit code."""
    import sys
    line = '{"metric": "m", "value": 1.0, "n_gpus": 2}'
    prog = f"print('noise'); print({line!r}); print('more')"
    monkeypatch.setattr(bench, "child_command", lambda n, argv, port: [sys.executable, "-c", prog])
    assert bench.spawn_ranks(2, []) == 0
    out, err = capsys.readouterr()
    assert out.strip() == line and "noise" in err and "more" in err
    monkeypatch.setattr(bench, "child_command", lambda n, argv, port: [sys.executable, "-c", "raise SystemExit(3)"])
    assert bench.spawn_ranks(2, []) == 3
    monkeypatch.setattr(bench, "child_command", lambda n, argv, port: [sys.executable, "-c", "print('x')"])
    assert bench.spawn_ranks(2, []) == 1        # rc 0 but no result line


def test_gpus_2_starts_two_ranks_on_cpu():
    """End to end without a GPU: `bench.py --gpus 2` starts torch.distributed.run
    with two ranks, each rank runs in-process (WORLD_SIZE 2, so no second
    spawn) and stops at the device check; the failure is the child's."""
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["HIP_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--nproc-per-node=2" in r.stderr and "torch.distributed.run" in r.stderr
    assert r.stderr.count("bench.py: launching") == 1                # the ranks did not re-spawn
    assert "no GPU visible" in r.stderr
    assert r.stdout == ""


def test_loop_summary_empty_cell_is_no_win():
    """a txloop cell that processed no burst prints null
    figures and exact false (tools/txloop.c); the summary lists it, marks the
    leg inexact, and never counts it as beating the reference."""
    rows = []
    for b in (64, 256, 2048):
        for f in bench.LOOP_FORMS:
            v = {"reference": 10.0, "pipelined": 8.0, "coalesced": 7.0, "sync": 12.0}[f] * b / 64
            r = {"mode": "loop", "form": f, "mix": "rx+reply", "pkt_len": 64, "burst": b,
                 "stack_ns_per_frame": 0, "stack_us_fixed": 0, "iters": 100, "bursts": 100,
                 "max_iter_us": 20.0, "us_per_burst": v, "us_worker": v, "us_latency": 30.0, "exact": True}
            if f == "coalesced" and b == 256:   # the driver's r5 cell: nothing recorded
                r.update(bursts=0, us_per_burst=None, us_worker=None, us_latency=None, exact=False, iters=0)
            rows.append(r)
    s = bench.loop_summary(rows)
    key = "rx+reply@0ns/frame"
    assert s["crossover"][key]["coalesced"] == 2048        # the empty 256 cell breaks the run of wins
    assert s["crossover"][key]["pipelined"] == 64
    assert s["exact"] is False and len(s["empty_cells"]) == 1 and "/coalesced/256" in s["empty_cells"][0]
    row256 = [r for r in s["rows"][key] if r[0] == 256][0]
    assert row256[1 + bench.LOOP_FORMS.index("coalesced")] is None
