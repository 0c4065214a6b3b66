"""Workload for rocprofv3 --pmc passes: the bench's 1 GiB HBM copy, 5 launches."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
with mpx.Context(1) as c:
    a, b = c.alloc(0, n), c.alloc(0, n)
    c.fill(a, n, mpx.FILL_SPLITMIX, 7)
    t = c.copy(0, b, a, n, 5)
    print(f"copy {n} B x5: {t.device_s / 5 * 1e6:.1f} us/launch")
