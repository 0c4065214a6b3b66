"""k_copy_steps load policy: nontemporal loads against default-policy loads
(MPX_COPY_STEPS 6th field: the knob and its kernel variant were removed after
this A/B found no difference), each with the default grid rule for the size,
in two cache states:

  fresh  — right after the buffers were filled (src resident in L2 / MALL);
  after  — after a run of 1 GiB copies (bench.py's state when its sweep
           starts: the headline's streaming copies have evicted src).

The question: whether nontemporal loads, if they did not allocate on a miss,
would make every repeated copy of an evicted small src pay HBM latency.  They
do not: both policies read the same in both states.
One process, interleaved, best of 5 calls of 10 copies, output checked.
JSON lines.

    python tools/copy_steps_ldpolicy.py > gpurun_out/copy_steps_ldpolicy.jsonl
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

G = 1 << 30


def spec(n: int, ldnt: int) -> str:
    return f"64:0:0:1:1024:{ldnt}" if n <= (1 << 20) else f"64:0:0:8:256:{ldnt}"


SIZES = [4 << 10, 16 << 10, 64 << 10, 256 << 10, 1 << 20, 3 << 19, 2 << 20]
with mpx.Context(1) as c:
    src, dst = c.alloc(0, G), c.alloc(0, G)
    c.fill(src, G, mpx.FILL_SPLITMIX, 5)
    os.environ["MPX_COPY_STEPS_MAX"] = str(2 << 20)
    for state in ("fresh", "after"):
        if state == "after":
            c.copy(0, dst, src, G, 30)
        for n in SIZES:
            best = {}
            for _ in range(2):
                for ldnt in (1, 0):
                    if state == "after":
                        c.copy(0, dst, src, G, 3)    # evict again before each variant
                    os.environ["MPX_COPY_STEPS"] = spec(n, ldnt)
                    c.copy(0, dst, src, n, 2)
                    for _ in range(5):
                        per = c.copy(0, dst, src, n, 10).device_s / 10
                        if ldnt not in best or per < best[ldnt]:
                            best[ldnt] = per
            assert c.checksum(dst, n) == c.checksum(src, n), n
            for ldnt, per in best.items():
                print(json.dumps(dict(state=state, bytes=n, loads="nontemporal" if ldnt else "default",
                                      us_per_copy=round(per * 1e6, 3))), flush=True)
