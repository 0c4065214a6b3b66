"""Diagnostic 2: which test condition breaks loopback pairs: check mode,
extra live contexts/streams, or many contexts created before."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402


def pair_case(label, engine="kernel", check=False, extra_ctx=0, modes=(0, 2), sizes=(0, 8, 65541)):
    extras = [mpx.Context(8, "kernel") for _ in range(extra_ctx)]
    for e in extras:  # give each extra context a live utility stream
        b = e.alloc(0, 64)
        e.fill(b, 64, mpx.FILL_BYTE, 1)
    c = mpx.Context(2, engine)
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, 1 << 20), c.alloc(0, 1 << 20)
        c.fill(tx, 1 << 20, mpx.FILL_BYTE, 98 - r)
        c.attach(r, 0, tx, rx, 1 << 20)
        bufs.append((tx, rx))
    for mode in modes:
        for n in sizes:
            exp = {r: (c.checksum(bufs[1 - r][0], n), c.checksum(bufs[1 - r][0], 1)) for r in (0, 1)}
            out, errs = {}, {}

            def side(r):
                try:
                    out[r] = c.xfer(mode, 1 - r, r, 1 - r, 7, bufs[r][0], bufs[r][1], n, check_payload=check,
                                    expect=exp[r][0], expect_ack=exp[r][1], timeout_ms=1500)
                except mpx.MpxError as e:
                    errs[r] = str(e)[:200]

            th = [threading.Thread(target=side, args=(r,)) for r in (0, 1)]
            t0 = time.time()
            for t in th:
                t.start()
            for t in th:
                t.join()
            print(f"{label} mode={mode} n={n} {'OK' if not errs else 'FAIL ' + repr(errs)} {time.time()-t0:.3f}s",
                  flush=True)
    c.close()
    for e in extras:
        e.close()


case = sys.argv[1]
if case == "check":
    pair_case("check", check=True)
elif case == "extra":
    pair_case("extra1", extra_ctx=1)
elif case == "extra3":
    pair_case("extra3", extra_ctx=3)
elif case == "seq":
    for i in range(4):
        pair_case(f"seq{i}", check=True)
