"""Diagnostic: config 2's sweep (bench.copy_sweep) at 1-4 MiB as bench.py runs
it, with and without the 1 GiB headline copies first, beside the interleaved
A/B's shape (copy_steps_wgsize.py mid).  Prints one JSON line per case."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402
import bench  # noqa: E402

if os.environ.get("WITH_TORCH"):     # bench.py's process: torch on the device first
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
    print(json.dumps(dict(case="torch initialised")), flush=True)

G = 1 << 30
with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 5)

    def sweep_at(sizes, label):
        out = {}
        for b in sizes:
            c.copy(0, dst, src, b, 2)
            best = min(c.copy(0, dst, src, b, 10).device_s / 10 for _ in range(5))
            out[str(b)] = round(best * 1e6, 3)
        print(json.dumps(dict(case=label, us_per_copy=out)), flush=True)

    mids = [1 << 20, 2 << 20, 4 << 20]
    sweep_at(mids, "cold: 1, 2, 4 MiB")
    sweep_at([2 << 20] * 3, "2 MiB three times")
    full = bench.copy_sweep(mpx, c, src, dst, 8 << 20)
    print(json.dumps(dict(case="bench.copy_sweep to 8 MiB", us_per_copy={k: v["us"] for k, v in full.items()
                                                                        if int(k) >= (1 << 20)})), flush=True)
    full = bench.copy_sweep(mpx, c, src, dst, G)
    print(json.dumps(dict(case="bench.copy_sweep to 1 GiB", us_per_copy={k: v["us"] for k, v in full.items()
                                                                        if (1 << 20) <= int(k) <= (8 << 20)})), flush=True)
    for _ in range(3):
        c.copy(0, dst, src, G, 10)
    sweep_at(mids, "after 30 x 1 GiB copies")
    sweep_at([2 << 20] * 3, "2 MiB three times")
