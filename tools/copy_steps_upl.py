"""k_copy_steps with batched loads: grid cap x units-per-lane per step
(MPX_COPY_STEPS="cap:xcd:drain:upl"), against one k_copy launch per copy, at
the sizes config 2's sweep runs as one launch.  One process, interleaved,
best of 5 calls of 10 copies (the bench sweep's shape).  JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

VARIANTS = ["launch", "default"] + [f"{g}:{int(g > 64)}:0:{u}" for g in (64, 128, 256, 512) for u in (1, 2, 4, 8)]
top = 8 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 5)
    for n in [1 << k for k in (0, 12, 16, 17, 18, 19, 20, 21, 22, 23)]:
        best = {}
        for _ in range(2):
            for v in VARIANTS:
                os.environ.pop("MPX_COPY_STEPS", None)
                if v == "launch":
                    os.environ["MPX_COPY_STEPS_MAX"] = "0"
                else:
                    os.environ["MPX_COPY_STEPS_MAX"] = str(top)
                    if v != "default":
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
