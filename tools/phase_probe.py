"""Where a short kernel-engine call's time goes (run-hbv3's
456131 B x 10 calls carried ~21 us of fixed cost each).  A loopback pair (two
ranks on GPU 0, one host thread each, a threading barrier before every call
as the reference's MPI_Barrier, mpi_perf.c:499) runs `calls` calls of each
shape; per call and side, mpx_last_phases splits the wall time into host
preparation, launch -> kernel start, the wait for the peer's receives, the
kernel and completion -> return.  Medians over the calls.

    MPX_SYNC=query|event python tools/phase_probe.py [calls] [armed]

armed: every call is armed (mpx_xfer_arm) before the barrier and started
after it, so its launch is outside the timed call.
"""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

CALLS = int(sys.argv[1]) if len(sys.argv) > 1 else 40
ARMED = "armed" in sys.argv[2:]
SHAPES = [("unidir", mpx.MODE_UNIDIR, 456131, 10), ("unidir", mpx.MODE_UNIDIR, 4 << 20, 10),
          ("pingpong", mpx.MODE_PINGPONG, 8, 10), ("unidir", mpx.MODE_UNIDIR, 4 << 20, 500)]
CAP = 4 << 20

with mpx.Context(2, "kernel") as c:
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
        c.fill(tx, CAP, mpx.FILL_SPLITMIX, r + 11)
        c.attach(r, 0, tx, rx, CAP)
        bufs.append((tx, rx))
    bar = threading.Barrier(2)
    for name, mode, n, iters in SHAPES:
        rows = {0: [], 1: []}
        errs = []

        def side(r):
            try:
                for k in range(CALLS + 2):
                    if ARMED:
                        c.arm(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n)
                    bar.wait()
                    t = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n)
                    if k >= 2:
                        rows[r].append(dict(c.phases(r), device_s=t.device_s))
            except Exception as e:  # noqa: BLE001
                errs.append(f"rank {r}: {e}")
                bar.abort()
        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        rec = dict(sync=os.environ.get("MPX_SYNC", "query"), armed=ARMED, shape=name, bytes=n, iters=iters, calls=CALLS)
        if errs:
            rec["error"] = errs[:2]
        else:
            walls = [max(a["wall_s"], b["wall_s"]) for a, b in zip(rows[0], rows[1])]
            rec["pair_wall_us_median"] = round(statistics.median(walls) * 1e6, 2)
            for r, label in ((0, "g1"), (1, "g0")):
                rec[label] = {k: round(statistics.median(x[k] for x in rows[r]) * 1e6, 2) for k in rows[r][0]
                              if k not in ("armed", "resident")}
                rec[label]["resident_fraction"] = sum(x["resident"] for x in rows[r]) / len(rows[r])
            if mode == mpx.MODE_UNIDIR:
                rec["GBps"] = round(n * iters / statistics.median(walls) / 1e9, 2)
        print(json.dumps(rec), flush=True)
