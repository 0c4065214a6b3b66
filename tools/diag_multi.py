"""Diagnostic: N concurrent loopback pairs on GPU 0; prints per-pair outcome."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402

npairs = int(sys.argv[1])
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for rep in range(reps):
    c = mpx.Context(2 * npairs, "kernel")
    bufs = []
    for r in range(2 * npairs):
        tx, rx = c.alloc(0, 1 << 16), c.alloc(0, 1 << 16)
        c.fill(tx, 1 << 16, mpx.FILL_BYTE, 98)
        c.attach(r, 0, tx, rx, 1 << 16)
        bufs.append((tx, rx))
    for n in (8, 65536):
        out, errs = {}, {}

        def side(r):
            peer = r + npairs if r < npairs else r - npairs
            try:
                out[r] = c.xfer(0, 1 if r < npairs else 0, r, peer, 20, bufs[r][0], bufs[r][1], n, timeout_ms=1000)
            except mpx.MpxError as e:
                errs[r] = str(e).split("(")[-2][:60]

        th = [threading.Thread(target=side, args=(r,)) for r in range(2 * npairs)]
        t0 = time.time()
        for t in th:
            t.start()
        for t in th:
            t.join()
        print(f"rep{rep} npairs={npairs} n={n} failed_ranks={sorted(errs)} {time.time()-t0:.2f}s", flush=True)
        if errs:
            break
    c.close()
