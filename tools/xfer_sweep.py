"""Loopback sweep of the transfer engines: two ranks on GPU 0 (one host
thread each), every mode, sizes 1 B .. 64 MiB.  One JSON line per point:
per-iteration time and GB/s by the reference's byte count (mpi_perf.c:538).
Env: ENGINES=kernel,sdma  MODES=0,1,2  MAXLOG=26."""
import json
import os
import statistics
import sys
import threading

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402

engines = os.environ.get("ENGINES", "kernel,sdma").split(",")
modes = [int(m) for m in os.environ.get("MODES", "0,1,2").split(",")]
maxlog = int(os.environ.get("MAXLOG", "26"))
sizes = [1, 8] + [1 << k for k in range(6, maxlog + 1, 2)]
cap = max(sizes)
for eng in engines:
    c = mpx.Context(2, eng)
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, cap), c.alloc(0, cap)
        c.fill(tx, cap, mpx.FILL_BYTE, 98 - r)
        c.attach(r, 0, tx, rx, cap)
        bufs.append((tx, rx))
    for mode in modes:
        for n in sizes:
            iters = max(20, min(20000, int(2e9 / max(n, 1) / 50)))
            if eng == "sdma":
                iters = min(iters, 2000)
            ts = []
            for rep in range(4):
                out = {}

                def side(r):
                    out[r] = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n, timeout_ms=5000)

                th = [threading.Thread(target=side, args=(r,)) for r in (0, 1)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                if rep:
                    ts.append(max(out[0].wall_s, out[1].wall_s))
            t = statistics.median(ts)
            factor = 1 if mode == 2 else 2
            print(json.dumps(dict(engine=eng, mode=mode, bytes=n, iters=iters, us_per_iter=round(t / iters * 1e6, 3),
                                  GBps=round(n * iters * factor / t / 1e9, 3), protocol=out[0].protocol,
                                  nwg=out[0].nwg, mailbox=os.environ.get("MPX_MAILBOX", "auto"))), flush=True)
    c.close()
