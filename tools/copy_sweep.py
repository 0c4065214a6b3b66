"""Tuning sweep of the HBM copy kernel variants (MPX_COPY_VARIANT); each
variant runs in its own process (the launcher reads the env once).
Prints one JSON line per variant: 1 GiB copy, HBM GB/s = 2B / avg launch."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "one":
    sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
    import mpx
    n = int(sys.argv[2])
    with mpx.Context(1) as c:
        a, b = c.alloc(0, n), c.alloc(0, n)
        c.fill(a, n, mpx.FILL_SPLITMIX, 7)
        c.copy(0, b, a, n, 3)
        best = 0
        for _ in range(5):
            t = c.copy(0, b, a, n, 10)
            best = max(best, 2 * n * t.launches / t.device_s / 1e9)
        assert c.checksum(a, n) == c.checksum(b, n)
        print(json.dumps({"variant": os.environ.get("MPX_COPY_VARIANT", "default"), "bytes": n,
                          "us_per_launch": round(2 * n / best / 1e3, 3), "hbm_GBps": round(best, 1),
                          "grid": t.nwg}), flush=True)
    sys.exit(0)

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
variants = []
if os.environ.get("SWEEP") == "refine":
    for u in (2, 4, 8):
        for bpc in (128, 256, 512, 1024):
            variants.append(f"{u}:1:1:1:{bpc}")
    for u in (2, 4):
        for bpc in (256, 512):
            variants.append(f"{u}:1:1:0:{bpc}")
elif os.environ.get("SWEEP") == "sizes":
    variants = [os.environ.get("MPX_COPY_VARIANT", "16:1:1:1:16")]
else:
    for u in (4, 8, 16):
        for ldnt in (0, 1):
            for stnt in (0, 1):
                for contig in (0, 1):
                    for bpc in (4, 8, 16):
                        variants.append(f"{u}:{ldnt}:{stnt}:{contig}:{bpc}")
sizes = [n]
if os.environ.get("SWEEP") == "sizes":
    sizes = [1 << k for k in range(12, 31, 2)]
if os.environ.get("SWEEP") == "cfg2":       # BASELINE config 2: 1 B .. 1 GiB, default variant
    variants = [None]
    sizes = [1 << k for k in range(0, 31)]
for v in variants:
    for size in sizes:
        env = dict(os.environ)
        if v:
            env["MPX_COPY_VARIANT"] = v
        else:
            env.pop("MPX_COPY_VARIANT", None)
        p = subprocess.run([sys.executable, __file__, "one", str(size)], env=env, capture_output=True, text=True,
                           timeout=120)
        print(p.stdout.strip() or json.dumps({"variant": v, "error": p.stderr[-300:]}), flush=True)
