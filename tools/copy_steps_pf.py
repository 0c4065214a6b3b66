"""k_copy_steps with and without prefetch (the loads of copy s+1 issued before
the barrier that ends copy s), against a launch per copy, 4 KiB - 16 MiB.
MPX_COPY_STEPS="cap:xcd:drain:upl:pf" (the pf field and its kernel variant were removed after this A/B); one process, interleaved, best of 5
calls of 10 copies, two passes, output checked.  JSON lines.

    python tools/copy_steps_pf.py > gpurun_out/copy_steps_pf.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402


def upl_default(n: int) -> int:   # launch_copy_steps' rule
    return 1 if n <= 128 << 10 else 4 if n <= 512 << 10 else 8


def variants(n: int) -> list[str]:
    u = upl_default(n)
    v = ["launch", f"64:0:0:{u}:0", f"64:0:0:{u}:1"]
    if n > 1 << 20:
        v += ["128:0:0:8:1", "256:0:0:8:1", "256:1:0:8:1", "512:1:0:8:1"]
    return v


top = 16 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 7)
    for n in [4096, 65536, 262144, 524288, 1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20]:
        best = {}
        for _ in range(2):
            for v in variants(n):
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
                assert c.checksum(b, n) == c.checksum(a, n), (n, v)
                c.fill(b, n, mpx.FILL_BYTE, 0)
        for v, (per, grid) in best.items():
            print(json.dumps(dict(bytes=n, variant=v, grid=grid, us_per_copy=round(per * 1e6, 3),
                                  GBps_2B=round(2 * n / per / 1e9, 1))), flush=True)
