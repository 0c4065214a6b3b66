"""Diagnostic: bench.py's config 2 sweep (bench.copy_sweep) right after the
headline's load (23 x 10 copies of 1 GiB), again 2 s later, then with the
pipe off (k_copy_steps / a launch per copy) — does the one-launch forms'
slowdown inside bench.py depend on the time since the 1 GiB copies?  JSON
lines: the 256 KiB - 8 MiB rows of each sweep."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402
import bench  # noqa: E402

G = 1 << 30


def rows(sw):
    return {k: (v["us"], v["path"]) for k, v in sw.items() if (256 << 10) <= int(k) <= (8 << 20)}


with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 9)
    t0 = time.time()
    for _ in range(23):
        c.copy(0, dst, src, G, 10)
    print(json.dumps(dict(state="right after the headline load", sweep=rows(bench.copy_sweep(mpx, c, src, dst, 8 << 20)))),
          flush=True)
    time.sleep(2)
    print(json.dumps(dict(state="2 s later", sweep=rows(bench.copy_sweep(mpx, c, src, dst, 8 << 20)))), flush=True)
    os.environ["MPX_COPY_PIPE_MAX"] = "0"
    print(json.dumps(dict(state="pipe off", sweep=rows(bench.copy_sweep(mpx, c, src, dst, 8 << 20)))), flush=True)
    os.environ.pop("MPX_COPY_PIPE_MAX")
    for _ in range(23):
        c.copy(0, dst, src, G, 10)
    print(json.dumps(dict(state="right after the headline load again", sweep=rows(bench.copy_sweep(mpx, c, src, dst, 8 << 20)))),
          flush=True)
