"""A rank paired with itself on the SDMA engine (the non-blocking loop as
MPI's self-send): its payload copies are hipMemcpyDeviceToDeviceNoCU, i.e.
copy-engine (SDMA) transfers even on one GPU — profiled by
tools/gpu.sh prof_sdma with --memory-copy-trace.  Every payload of the first
call is checked; prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

N = 4 << 20
with mpx.Context(1, "sdma") as c:
    tx, rx = c.alloc(0, N), c.alloc(0, N)
    c.fill(tx, N, mpx.FILL_SPLITMIX, 7)
    c.attach(0, 0, tx, rx, N)
    want = c.checksum(tx, N)
    t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, 64, tx, rx, N, check_payload=True, expect=want, timeout_ms=10000)
    assert t.check_iters == 64 and t.check_failures == 0
    t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, 512, tx, rx, N, timeout_ms=10000)
    assert c.checksum(rx, N) == want
    print(json.dumps(dict(bytes=N, iters=512, us_per_iter=round(t.device_s / 512 * 1e6, 3),
                          GBps=round(N * 512 / t.device_s / 1e9, 2))), flush=True)
