"""LL vs bulk between two ranks of ONE GPU (a loopback pair, threads of one
process) at 1-8 KiB: every message LL (MPX_LL_MAX=8192) against every
message bulk (MPX_LL_MAX=0), ping-pong and unidirectional, interleaved,
three rounds, median of 5 runs of 5000 iterations each, with every payload of
one extra run per case checked.  libmpx reads MPX_LL_MAX per call.  The
question: where the one-GPU LL threshold (ll_max_bytes(same_device)) should
sit now that the LL path holds its payload in registers and polls with 16-B
loads.  JSON lines.

    python tools/ll_threshold_ab.py > gpurun_out/ll_threshold_ab.jsonl
"""
import json
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
import mpx  # noqa: E402

ITERS = 5000
CAP = 8192
SIZES = (1024, 2048, 3072, 4096, 6144, 8192)
with mpx.Context(2, "kernel") as c:
    bufs = []
    for r in range(2):
        tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
        c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, r, 1 - r, 0))
        c.attach(r, 0, tx, rx, CAP)
        bufs.append((tx, rx))

    def pair(mode, n, iters, check=False):
        out, errs = {}, []

        def side(r):
            try:
                kw = {}
                if check:
                    peer_tx = bufs[1 - r][0]
                    kw = dict(check_payload=True, expect=c.checksum(peer_tx, n), expect_ack=c.checksum(peer_tx, 1))
                out[r] = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n, timeout_ms=10000, **kw)
            except Exception as e:  # noqa: BLE001
                errs.append(e)

        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]
        return max(out[0].device_s, out[1].device_s) / iters * 1e6, out[0].protocol

    best = {}
    for _ in range(3):
        for name, mode in (("pingpong", mpx.MODE_PINGPONG), ("unidir", mpx.MODE_UNIDIR)):
            for n in SIZES:
                for proto, v in (("ll", "8192"), ("bulk", "0")):
                    os.environ["MPX_LL_MAX"] = v
                    pair(mode, n, 50, check=True)          # every payload checked once per case
                    t = statistics.median(pair(mode, n, ITERS)[0] for _ in range(5))
                    key = (name, n, proto)
                    best.setdefault(key, []).append(t)
    for (name, n, proto), ts in sorted(best.items()):
        print(json.dumps(dict(mode=name, bytes=n, proto=proto, us_per_iter=round(statistics.median(ts), 3),
                              runs=[round(x, 3) for x in ts])), flush=True)
