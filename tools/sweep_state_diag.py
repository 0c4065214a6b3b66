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


def one_mib_arms(c, src, dst):
    """`onemib`: which form 1 MiB should take inside bench.py — after the
    headline's load, three interleaved rounds of the sweep to 4 MiB with 1 MiB
    as the one-counter pipe (default), as k_copy_steps (MPX_COPY_PIPE_MIN =
    1 MiB) and as the two-level pipe (MPX_COPY_PIPE_HIER=1)."""
    arms = (("pipe_one_counter", {}), ("steps", {"MPX_COPY_PIPE_MIN": str(1 << 20)}),
            ("pipe_two_level", {"MPX_COPY_PIPE_HIER": "1"}))
    for _ in range(23):
        c.copy(0, dst, src, G, 10)
    for rnd in range(3):
        for name, env in arms:
            os.environ.update(env)
            sw = rows(bench.copy_sweep(mpx, c, src, dst, 4 << 20))
            for k in env:
                os.environ.pop(k)
            print(json.dumps(dict(state=f"after the headline load, round {rnd}", arm=name, sweep=sw)), flush=True)


if len(sys.argv) > 2 and sys.argv[2] == "torch":
    # bench.py's process state: torch initialised on the device first
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()

with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    if len(sys.argv) > 1 and sys.argv[1] == "onemib":
        c.fill(src, G, mpx.FILL_SPLITMIX, 9)
        one_mib_arms(c, src, dst)
        sys.exit(0)
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
