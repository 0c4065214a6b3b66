"""k_copy (a launch per copy) with 256-lane workgroups (default) against the
same one-unit-per-lane shape with 512 / 1024 lanes (MPX_COPY_WIDE: the knob
and its kernel were removed after this A/B — no size gained beyond noise,
16-64 MiB lost 12-50 %), at config
2's sizes above the one-launch switch, up to 1 GiB (the headline).  One
process, interleaved, best of 5 calls (10 copies; 3 from 256 MiB), three
passes, output checked.  JSON lines.

    python tools/copy_wide.py > gpurun_out/copy_wide.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

G = 1 << 30
VARIANTS = ["256", "512", "1024"]
with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 5)
    for n in [2 << 20, 4 << 20, 8 << 20, 16 << 20, 64 << 20, 256 << 20, G]:
        copies = 10 if n < (256 << 20) else 3
        best = {}
        for _ in range(3):
            for v in VARIANTS:
                if v == "256":
                    os.environ.pop("MPX_COPY_WIDE", None)
                else:
                    os.environ["MPX_COPY_WIDE"] = f"{G}:{v}"
                c.copy(0, dst, src, n, 2)
                for _ in range(5):
                    per = c.copy(0, dst, src, n, copies).device_s / copies
                    best[v] = min(best.get(v, 9.0), per)
                assert c.checksum(dst, n) == c.checksum(src, n), (n, v)
        for v, per in best.items():
            print(json.dumps(dict(bytes=n, threads=int(v), us_per_copy=round(per * 1e6, 3),
                                  hbm_GBps=round(2 * n / per / 1e9, 1))), flush=True)
