"""A/B of the one-workgroup waits' polling (MPX_POLL_STAGGER at build time:
0 = one polling wave, else four staggered waves): a loopback pair (two ranks
on GPU 0, one thread each) — 8 B LL ping-pong half round trip, unidir 32 KiB
and 456131 B per-iteration time (the receiver's flag wait), run-hbv3's
456131 B x 10 armed call wall.  Run once per libmpx variant copied into
place; prints one JSON line.

    python tools/poll_stagger_ab.py <label>
"""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

CAP = 1 << 20
out = {"variant": sys.argv[1]}
with mpx.Context(2, "kernel") as c:
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
        c.fill(tx, CAP, mpx.FILL_SPLITMIX, r + 3)
        c.attach(r, 0, tx, rx, CAP)
        bufs.append((tx, rx))
    bar = threading.Barrier(2)

    def pair(mode, n, iters, calls, armed=False):
        walls = {0: [], 1: []}

        def side(r):
            for _ in range(calls):
                if armed:
                    c.arm(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n)
                bar.wait()
                walls[r].append(c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n).wall_s)
        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        return statistics.median(max(a, b) for a, b in zip(walls[0], walls[1]))

    pair(mpx.MODE_PINGPONG, 8, 1000, 2)
    out["pingpong_8B_half_rtt_us"] = round(pair(mpx.MODE_PINGPONG, 8, 100000, 3) / 200000 * 1e6, 4)
    out["pingpong_512B_half_rtt_us"] = round(pair(mpx.MODE_PINGPONG, 512, 50000, 3) / 100000 * 1e6, 4)
    out["unidir_32KiB_us_per_iter"] = round(pair(mpx.MODE_UNIDIR, 32768, 20000, 3) / 20000 * 1e6, 4)
    out["unidir_456131_us_per_iter"] = round(pair(mpx.MODE_UNIDIR, 456131, 5000, 3) / 5000 * 1e6, 4)
    out["hbv3_call_wall_us"] = round(pair(mpx.MODE_UNIDIR, 456131, 10, 40, armed=True) * 1e6, 2)
print(json.dumps(out), flush=True)
