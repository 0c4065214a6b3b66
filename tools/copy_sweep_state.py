"""Diagnostic: k_copy_steps shapes at 1-2 MiB after bench.py's full config 2
sweep (1 B - 1 GiB), the state in which bench's own sweep read 3.4-3.9 us
for 2 MiB where a fresh process reads 2.35 (tools/copy_sweep_order.py).
Variants interleaved, 3 rounds, best of 5 calls of 10 copies.  JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402
import bench  # noqa: E402

G = 1 << 30
VARIANTS = ["launch", "64:0:0:8:256:1", "64:0:0:8:256:0", "64:0:0:2:1024:1", "128:0:0:1:1024:1",
            "64:0:1:8:256:1", "32:0:0:4:1024:1"]
with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 5)

    def measure(label):
        for n in (1 << 20, 2 << 20):
            best = {}
            for _ in range(3):
                for v in VARIANTS:
                    os.environ["MPX_COPY_STEPS_MAX"] = "0" if v == "launch" else str(4 << 20)
                    os.environ["MPX_COPY_STEPS"] = "" if v == "launch" else v
                    c.copy(0, dst, src, n, 2)
                    per = min(c.copy(0, dst, src, n, 10).device_s / 10 for _ in range(5))
                    best[v] = min(best.get(v, 9), per)
            print(json.dumps(dict(state=label, bytes=n, us_per_copy={k: round(v * 1e6, 3) for k, v in best.items()})),
                  flush=True)

    measure("fresh")
    bench.copy_sweep(mpx, c, src, dst, G)
    measure("after bench.copy_sweep to 1 GiB")
    c.copy(0, dst, src, G, 30)
    measure("after 30 more 1 GiB copies")
