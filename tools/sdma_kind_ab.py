"""One process of the SDMA-engine copy-kind A/B (tools/gpu_sdma_kind_ab.sh):
a loopback pair on GPU 0 on the SDMA engine, unidir 4 MiB x 200 and 64 KiB x
1000, ping-pong 8 B x 2000, -x 1 4 MiB x 256, every payload of a first pass
checked, then timed without check (graph-replayed); MPX_SDMA_KIND set by the
caller."""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

CAP = 4 << 20
with mpx.Context(2, "sdma") as c:
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
        c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, r, 0, 0))
        c.attach(r, 0, tx, rx, CAP)
        bufs.append((tx, rx))
    res = {}
    for name, mode, n, iters in (("unidir_4MiB", mpx.MODE_UNIDIR, CAP, 200), ("unidir_64KiB", mpx.MODE_UNIDIR, 65536, 1000),
                                 ("pingpong_8B", mpx.MODE_PINGPONG, 8, 2000), ("nb_4MiB", mpx.MODE_NONBLOCKING, CAP, 256)):
        exp = [(c.checksum(bufs[1 - r][0], n), c.checksum(bufs[1 - r][0], 1)) for r in range(2)]
        t = []
        for rep in range(4):
            out, errs = {}, []
            check = rep == 0

            def side(r):
                try:
                    out[r] = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n, check_payload=check,
                                    expect=exp[r][0], expect_ack=exp[r][1], timeout_ms=10000)
                except Exception as e:  # noqa: BLE001
                    errs.append(str(e))

            th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errs, errs
            if check:
                assert all(out[r].check_failures == 0 and out[r].check_iters == iters for r in range(2)), name
            else:
                t.append(max(out[0].device_s, out[1].device_s) / iters * 1e6)
        us = statistics.median(t)
        res[name] = dict(us_per_iter=round(us, 3), GBps=round(n / us / 1e3, 2))
    print(json.dumps(dict(kind=os.environ.get("MPX_SDMA_KIND", "auto"), results=res)), flush=True)
