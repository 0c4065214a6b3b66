"""A/B of BASELINE config 2's copy at every size 2^0 .. 2^30: one k_copy
launch per copy (MPX_COPY_STEPS_MAX=0) against all copies of the call in one
k_copy_steps launch with a grid barrier per step.  Both in one process,
interleaved per size, best of 5 batches of `iters` copies each; output of
each size checked.  One JSON line per (size, path): us per copy and the rate
counted as HBM traffic (2B per copy) — sizes up to the 4 MB L2 per XCD / the
256 MB Infinity Cache are served from cache, not HBM.

    python tools/copy_steps_ab.py [iters]   -> stdout JSON lines
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
top = 1 << 30
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 11)
    for k in range(0, 31):
        n = 1 << k
        it = iters if n < (256 << 20) else 3
        res = {}
        for _ in range(2):   # interleave the two paths twice
            for path, cap in (("launch", "0"), ("steps", str(top))):
                os.environ["MPX_COPY_STEPS_MAX"] = cap
                c.copy(0, b, a, n, 2)
                best = None
                for _ in range(5):
                    t = c.copy(0, b, a, n, it)
                    per = t.device_s / it
                    best = per if best is None or per < best[0] else best
                    best = (min(best[0], per), t.protocol, t.launches, t.nwg) if isinstance(best, tuple) else \
                        (per, t.protocol, t.launches, t.nwg)
                prev = res.get(path)
                if prev is None or best[0] < prev[0]:
                    res[path] = best
        assert c.checksum(b, n) == c.checksum(a, n), n
        for path, (per, proto, launches, grid) in res.items():
            print(json.dumps(dict(bytes=n, path=path, iters=it, us_per_copy=round(per * 1e6, 3),
                                  hbm_GBps=round(2 * n / per / 1e9, 1), protocol=mpx.PROTOCOLS.get(proto, proto),
                                  launches=launches, grid=grid)), flush=True)
