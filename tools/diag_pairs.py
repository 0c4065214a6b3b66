"""Diagnostic: loopback ping-pong / unidir on GPU 0 under each mailbox kind.
Prints one line per case: ok or the error.  Used to find the cause of the
pair-test timeouts (run under gpurun, one process per kind)."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402


def run(c, bufs, mode, n, iters, tmo=1500):
    out, errs = {}, {}

    def side(r):
        try:
            out[r] = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n, timeout_ms=tmo)
        except mpx.MpxError as e:
            errs[r] = str(e)[:160]

    th = [threading.Thread(target=side, args=(r,)) for r in (1, 0)] if os.environ.get("REV") else \
         [threading.Thread(target=side, args=(r,)) for r in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return out, errs


def main():
    engine = os.environ.get("ENGINE", "kernel")
    with mpx.Context(2, engine) as c:
        bufs = []
        for r in range(2):
            tx, rx = c.alloc(0, 1 << 20), c.alloc(0, 1 << 20)
            c.fill(tx, 1 << 20, mpx.FILL_BYTE, 98 - r)
            c.attach(r, 0, tx, rx, 1 << 20)
            bufs.append((tx, rx))
        for mode in (0, 2, 1):
            for n in (0, 8, 4096, 65541, 1 << 20):
                t0 = time.time()
                out, errs = run(c, bufs, mode, n, 20)
                print(f"kind={os.environ.get('MPX_MAILBOX','auto')} mode={mode} n={n} "
                      f"{'OK' if not errs else 'FAIL ' + repr(errs)} {time.time()-t0:.3f}s", flush=True)
                if errs:
                    return


main()
