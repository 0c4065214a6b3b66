"""k_copy_steps at config 2's mid sizes (4-128 MiB), where a launch per copy
still pays a kernel boundary per copy: one k_copy launch per copy against
all copies in one k_copy_steps launch (MPX_COPY_STEPS="cap:xcd:drain:upl",
per-XCD barrier counters).  One process, interleaved, best of 5 calls of 10
copies, two passes.  JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

VARIANTS = ["launch"] + [f"{g}:1:0:{u}" for g in (256, 512, 1024) for u in (2, 8)]
top = 128 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 5)
    for n in [1 << k for k in (21, 22, 23, 24, 25, 26, 27)]:
        best = {}
        for _ in range(2):
            for v in VARIANTS:
                os.environ.pop("MPX_COPY_STEPS", None)
                if v == "launch":
                    os.environ["MPX_COPY_STEPS_MAX"] = "0"
                else:
                    os.environ["MPX_COPY_STEPS_MAX"] = str(top)
                    os.environ["MPX_COPY_STEPS"] = v
                c.copy(0, b, a, n, 2)
                for _ in range(5):
                    t = c.copy(0, b, a, n, 10)
                    per = t.device_s / 10
                    if v not in best or per < best[v][0]:
                        best[v] = (per, t.nwg)
            assert c.checksum(b, n) == c.checksum(a, n), n
        for v, (per, grid) in best.items():
            print(json.dumps(dict(bytes=n, variant=v, grid=grid, us_per_copy=round(per * 1e6, 3),
                                  GBps_2B=round(2 * n / per / 1e9, 1))), flush=True)
