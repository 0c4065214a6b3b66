"""One process of the LL poll A/B (tools/gpu_ll_poll_ab.sh): a loopback pair
on GPU 0, 8 B and 1 KiB ping-pong and 8 B unidir, 20000 iterations, median
of 5 runs; MPX_LL_FLAGS is set by the caller (read once per process)."""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

ITERS = 20000
with mpx.Context(2, "kernel") as c:
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, 4096), c.alloc(0, 4096)
        c.fill(tx, 4096, mpx.FILL_BYTE, ord("b") if r == 0 else ord("a"))
        c.attach(r, 0, tx, rx, 4096)
        bufs.append((tx, rx))
    res = {}
    for name, mode, n in (("pingpong_8", mpx.MODE_PINGPONG, 8), ("pingpong_1024", mpx.MODE_PINGPONG, 1024),
                          ("unidir_8", mpx.MODE_UNIDIR, 8)):
        t = []
        for _ in range(6):
            out = {}

            def side(r):
                out[r] = c.xfer(mode, 1 - r, r, 1 - r, ITERS, bufs[r][0], bufs[r][1], n)

            th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            t.append(max(out[0].device_s, out[1].device_s) / ITERS * 1e6)
        res[name] = round(statistics.median(t[1:]), 4)
    print(json.dumps(dict(ll_flags=os.environ.get("MPX_LL_FLAGS", "0"), us_per_iter=res)), flush=True)
