"""k_copy_steps load policy at config 2's small sizes: nontemporal loads
(default) against default-policy loads that can stay in the XCD's L2 across
the copies of one call (MPX_COPY_STEPS 5th field), with the default grid
rule.  One process, interleaved, best of 5 calls of 10 copies, two passes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402


def rule(n):   # launch_copy_steps' defaults
    return 1 if n <= (128 << 10) else 4 if n <= (512 << 10) else 8


top = 1 << 20
with mpx.Context(1) as c:
    a, b = c.alloc(0, top), c.alloc(0, top)
    c.fill(a, top, mpx.FILL_SPLITMIX, 5)
    for n in [1 << k for k in (0, 4, 8, 12, 13, 14, 16, 17, 18, 19, 20)]:
        best = {}
        for _ in range(2):
            for ld in (1, 0):
                os.environ["MPX_COPY_STEPS"] = f"64:0:0:{rule(n)}:{ld}"
                c.copy(0, b, a, n, 2)
                for _ in range(5):
                    t = c.copy(0, b, a, n, 10)
                    per = t.device_s / 10
                    if ld not in best or per < best[ld]:
                        best[ld] = per
            assert c.checksum(b, n) == c.checksum(a, n), n
        print(json.dumps(dict(bytes=n, nt_loads_us=round(best[1] * 1e6, 3), plain_loads_us=round(best[0] * 1e6, 3))),
              flush=True)
