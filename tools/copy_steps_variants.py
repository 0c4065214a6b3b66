"""k_copy_steps variants (MPX_COPY_STEPS="grid_cap:xcd:drain") at the sizes
where dispatch dominates, against one k_copy launch per copy; one process,
interleaved, best of 5 batches of 20 copies.  JSON lines on stdout."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

VARIANTS = ["launch"] + [f"{g}:{x}:{d}" for g in (64, 256, 1024) for x in (0, 1) for d in (0, 1)]
top = 64 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 5)
    for n in [1 << k for k in (0, 12, 16, 18, 20, 21, 22, 23, 24, 25, 26)]:
        best = {}
        for _ in range(2):
            for v in VARIANTS:
                if v == "launch":
                    os.environ["MPX_COPY_STEPS_MAX"] = "0"
                else:
                    os.environ["MPX_COPY_STEPS_MAX"] = str(top)
                    os.environ["MPX_COPY_STEPS"] = v
                c.copy(0, b, a, n, 2)
                for _ in range(5):
                    t = c.copy(0, b, a, n, 20)
                    per = t.device_s / 20
                    if v not in best or per < best[v][0]:
                        best[v] = (per, t.nwg)
        assert c.checksum(b, n) == c.checksum(a, n), n
        for v, (per, grid) in best.items():
            print(json.dumps(dict(bytes=n, variant=v, grid=grid, us_per_copy=round(per * 1e6, 3),
                                  GBps_2B=round(2 * n / per / 1e9, 1))), flush=True)
