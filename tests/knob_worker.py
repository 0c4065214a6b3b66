"""GPU worker for tests/test_gpu_engine.py::test_env_knob_variants: runs the
loopback pair (two ranks on GPU 0) through every mode and both engines with
every payload checked, under whatever MPX_* knobs its environment sets (libmpx
reads them once per process, hence a process of its own).  "kernel-pull" is
the kernel engine in pull mode (MPX_XFER_PULL), whose non-blocking receives
publish on the MPX_NB_PUBLISH schedule too; "sdma-pull" the SDMA engine's.  Prints "ok" or raises."""
import os
import sys
import threading

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-perf_amd"))
import mpx  # noqa: E402

CAP = (1 << 20) + 9
STAGE = os.environ.get("WORKER_NOSTAGE") != "1"   # the call flag MPX_XFER_NOSTAGE (bulk pushes read tx from HBM)
for engine in ("kernel", "sdma", "kernel-pull", "sdma-pull"):
    pull = engine.endswith("-pull")
    with mpx.Context(2, engine[:-len("-pull")] if pull else engine) as c:
        bufs = []
        for r in range(2):
            tx, rx = c.alloc(0, CAP), c.alloc(0, CAP)
            c.fill(tx, CAP, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, r, 0, 0))
            c.attach(r, 0, tx, rx, CAP)
            bufs.append((tx, rx))
        for mode in (mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING, mpx.MODE_UNIDIR):
            for n, iters, check in [(8, 300, False), (4100, 7, True), (70001, 5, True), (CAP, 3, True),
                                    (65541, 519, False), (4100, 300, True)]:
                exp = {r: (c.checksum(bufs[1 - r][0], n), c.checksum(bufs[1 - r][0], 1)) for r in (0, 1)}
                errs = []

                def side(r):
                    try:
                        t = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], n, check_payload=check,
                                   expect=exp[r][0], expect_ack=exp[r][1], timeout_ms=10000, pull=pull, stage=STAGE)
                        assert t.check_failures == 0
                    except Exception as e:  # noqa: BLE001
                        errs.append(f"{engine} mode {mode} n {n} rank {r}: {e}")

                th = [threading.Thread(target=side, args=(r,)) for r in (0, 1)]
                for t in th:
                    t.start()
                for t in th:
                    t.join()
                assert not errs, errs
                for r in (0, 1):
                    m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                    assert c.checksum(bufs[r][1], m) == c.checksum(bufs[1 - r][0], m), (engine, mode, n, r)
print("ok")
