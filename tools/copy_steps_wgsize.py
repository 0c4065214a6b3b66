"""k_copy_steps workgroup size: one wide workgroup (512 / 1024 lanes, no grid
barrier: __syncthreads ends a step) against the default grid of 256-lane
workgroups with a one-counter grid barrier, at config 2's sizes that run as one
launch (MPX_COPY_STEPS="cap:xcd:drain:upl:threads").  One process,
interleaved, best of 5 calls of 10 copies (the bench sweep's shape), two
passes, output checked.  JSON lines.

    python tools/copy_steps_wgsize.py > gpurun_out/copy_steps_wgsize.jsonl
    python tools/copy_steps_wgsize.py confirm    # the chosen default vs the old rule, 3 passes
    python tools/copy_steps_wgsize.py mid        # 1-4 MiB: one launch (widths) vs a launch per copy
    python tools/copy_steps_wgsize.py onexcd     # every working workgroup on XCD 0 (6th field)
    python tools/copy_steps_wgsize.py hier       # 256 KiB - 1 MiB: per-XCD arrival counters (2nd field)

"old" is the earlier default: 256-lane workgroups, grid <= 64, sized for 1
unit per lane up to 128 KiB, 4 at 256-512 KiB and 8 above.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

MODE = sys.argv[1] if len(sys.argv) > 1 else ""
CONFIRM = MODE == "confirm"
MID = MODE == "mid"
ONEXCD = MODE == "onexcd"
HIER = MODE == "hier"
VARIANTS = (["default", "64:1:0:1:1024:0", "64:1:0:2:1024:0", "64:1:0:4:256:0", "64:1:0:1:512:0"] if HIER else
            ["default", "prev", "64:0:0:1:1024:1", "64:0:0:1:512:1"] if ONEXCD else
            ["default", "old", "64:0:0:2:1024", "64:0:0:1:512"] if CONFIRM else
            ["launch", "default", "64:0:0:8:256", "64:0:0:4:512", "64:0:0:2:1024"] if MID else
            ["default", "1:0:0:8:256", "1:0:0:8:512", "1:0:0:8:1024", "1:0:0:16:1024", "1:0:0:32:1024",
             "16:0:0:8:1024", "64:0:0:1:1024", "64:0:0:4:1024", "64:0:0:8:512"])
top = (4 << 20) if MID else (2 << 20)
with mpx.Context(1) as c:
    # AB_ALLOC=bytes: allocate larger buffers (bench.py copies the first B
    # bytes of 1 GiB ones) while copying the same sizes
    alloc = max(top, int(os.environ.get("AB_ALLOC", "0")))
    a, b = c.alloc(0, alloc), c.alloc(0, alloc)
    c.fill(a, alloc, mpx.FILL_SPLITMIX, 5)
    os.environ["MPX_COPY_STEPS_MAX"] = str(top)
    sizes = ([1, 64, 1024] if CONFIRM else []) + [1 << k for k in range(12, 22)] + [(64 << 10) + 13]
    if MID:
        sizes = [32 << 10, 1 << 20, 3 << 19, 2 << 20, 3 << 20, 4 << 20]
    if HIER:
        sizes = [256 << 10, 512 << 10, 768 << 10, 1 << 20]
    for n in sizes:
        best = {}
        for _ in range(3 if CONFIRM or MID or ONEXCD or HIER else 2):
            for v in VARIANTS:
                os.environ.pop("MPX_COPY_STEPS", None)
                os.environ["MPX_COPY_STEPS_MAX"] = "0" if v == "launch" else str(top)
                if v == "prev":      # the default before the one-XCD rule: 1024 lanes, 1 unit, all XCDs
                    os.environ["MPX_COPY_STEPS"] = "64:0:0:1:1024:0" if n <= (1 << 20) else "64:0:0:8:256:0"
                elif v == "old":
                    upl = 1 if n <= (128 << 10) else 4 if n <= (512 << 10) else 8
                    os.environ["MPX_COPY_STEPS"] = f"64:0:0:{upl}:256"
                elif v != "default":
                    os.environ["MPX_COPY_STEPS"] = v
                c.fill(b, n, mpx.FILL_BYTE, 0)
                c.copy(0, b, a, n, 2)
                assert c.checksum(b, n) == c.checksum(a, n), (n, v)
                for _ in range(5):
                    t = c.copy(0, b, a, n, 10)
                    per = t.device_s / 10
                    if v not in best or per < best[v][0]:
                        best[v] = (per, t.nwg)
        for v, (per, grid) in best.items():
            print(json.dumps(dict(bytes=n, variant=v, grid=grid, us_per_copy=round(per * 1e6, 3),
                                  GBps_2B=round(2 * n / per / 1e9, 1))), flush=True)
