"""Diagnostic: k_copy_pipe per-copy time at 1-16 MiB in a fresh process and
right after 1 GiB copies (the state bench.py's sweep runs in), per units
per lane and barrier form (MPX_COPY_PIPE_UPL, MPX_COPY_PIPE_HIER), against a
launch per copy.  JSON lines."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

G = 1 << 30
BIG = {"MPX_COPY_PIPE_MAX": str(32 << 20)}
ARMS = {"pipe": BIG, "hier_u2": dict(BIG, MPX_COPY_PIPE_HIER="1", MPX_COPY_PIPE_UPL="2"),
        "hier_u4": dict(BIG, MPX_COPY_PIPE_HIER="1", MPX_COPY_PIPE_UPL="4"),
        "hier_u8": dict(BIG, MPX_COPY_PIPE_HIER="1", MPX_COPY_PIPE_UPL="8"),
        "hier_u16": dict(BIG, MPX_COPY_PIPE_HIER="1", MPX_COPY_PIPE_UPL="16"),
        "launch": {"MPX_COPY_PIPE_MAX": "0", "MPX_COPY_STEPS_MAX": "0"}}
KEYS = ("MPX_COPY_PIPE_UPL", "MPX_COPY_PIPE_HIER", "MPX_COPY_PIPE_MAX", "MPX_COPY_STEPS_MAX")


def best(c, src, dst, n, copies=10):
    c.copy(0, dst, src, n, 2)
    out = []
    for _ in range(5):
        t = c.copy(0, dst, src, n, copies)
        out.append(t.device_s / copies * 1e6)
    return dict(best=round(min(out), 3), median=round(sorted(out)[2], 3), path=mpx.PROTOCOLS[t.protocol], grid=t.nwg)


with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 3)
    for state in ("fresh", "after 30 x 1 GiB"):
        if state != "fresh":
            for k in KEYS:
                os.environ.pop(k, None)
            for _ in range(3):
                c.copy(0, dst, src, G, 10)
        for n in (1 << 20, 2 << 20, 4 << 20, 8 << 20, 16 << 20):
            for arm, env in ARMS.items():
                for k in KEYS:
                    os.environ.pop(k, None)
                os.environ.update(env)
                print(json.dumps(dict(state=state, bytes=n, arm=arm, **best(c, src, dst, n))), flush=True)
