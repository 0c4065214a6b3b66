"""k_copy_steps with few workgroups (grid cap 8 / 16 / 32 / 64): fewer arrivals
per grid barrier against more units per lane, at 64 KiB - 1 MiB
(MPX_COPY_STEPS="cap:0:0:1", units per lane then n/16/(cap*256)).  One
process, interleaved, best of 5 calls of 10 copies, two passes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

VARIANTS = ["default", "8:0:0:1", "16:0:0:1", "32:0:0:1", "64:0:0:1"]
top = 1 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 5)
    for n in [1 << k for k in (16, 17, 18, 19, 20)]:
        best = {}
        for _ in range(2):
            for v in VARIANTS:
                os.environ.pop("MPX_COPY_STEPS", None)
                if v != "default":
                    os.environ["MPX_COPY_STEPS"] = v
                c.copy(0, b, a, n, 2)
                for _ in range(5):
                    t = c.copy(0, b, a, n, 10)
                    per = t.device_s / 10
                    if v not in best or per < best[v][0]:
                        best[v] = (per, t.nwg)
            assert c.checksum(b, n) == c.checksum(a, n), n
        print(json.dumps(dict(bytes=n, **{v: dict(us=round(p * 1e6, 3), grid=g) for v, (p, g) in best.items()})),
              flush=True)
