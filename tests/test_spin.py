"""The node-local spin barrier (mpxb_spin_*, host/mpx_boot.h; mpx/spin.py)
that stands in front of every timed loop: no rank leaves barrier k before
every rank has entered it, in one process (threads) and across processes
(POSIX shared memory), and a missing rank ends in a timeout, not a hang.
CPU only."""
import multiprocessing as mp
import os
import threading
import uuid

import pytest

from mpx import spin

ROUNDS = 2000


def test_threads_never_pass_early():
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    n = 4
    bars = [spin.SpinBarrier(name, n, True)] + [spin.SpinBarrier(name, n, False) for _ in range(n - 1)]
    spin.unlink(name)
    arrived = [0] * n
    bad = []

    def rank(r):
        for k in range(ROUNDS):
            arrived[r] = k + 1
            bars[r].wait(30)
            # everyone has entered barrier k, so every count is >= k + 1
            if min(arrived) < k + 1:
                bad.append((r, k, list(arrived)))
            bars[r].wait(30)          # nobody enters k + 1 before all checked k

    th = [threading.Thread(target=rank, args=(r,)) for r in range(n)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for b in bars:
        b.close()
    assert not bad, bad[:3]


def _proc(name, n, r, q):
    b = spin.SpinBarrier(name, n, False)
    total = 0
    for k in range(ROUNDS // 4):
        b.wait(30)
        total += 1
    b.close()
    q.put((r, total))


def test_processes_share_one_barrier():
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    n = 3
    root = spin.SpinBarrier(name, n, True)
    q = mp.get_context("fork").Queue()
    ps = [mp.get_context("fork").Process(target=_proc, args=(name, n, r, q)) for r in (1, 2)]
    for p in ps:
        p.start()
    for _ in range(ROUNDS // 4):
        root.wait(30)
    for p in ps:
        p.join(60)
    got = sorted(q.get(timeout=5) for _ in ps)
    root.close()
    spin.unlink(name)
    assert got == [(1, ROUNDS // 4), (2, ROUNDS // 4)] and all(p.exitcode == 0 for p in ps)


def test_a_missing_rank_times_out():
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    b = spin.SpinBarrier(name, 2, True)
    spin.unlink(name)
    with pytest.raises(TimeoutError, match="timed out"):
        b.wait(0.2)
    b.close()


def test_rank_count_must_match():
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    b = spin.SpinBarrier(name, 4, True)
    try:
        with pytest.raises(OSError, match="made for 4 ranks, not 3"):
            spin.SpinBarrier(name, 3, False)
    finally:
        b.close()
        spin.unlink(name)
    assert not os.path.exists("/dev/shm" + name)


def test_wait_then_calls_through_after_every_rank_arrived():
    """mpxb_spin_wait_xfer: the call starts only once the barrier opens and
    its return code comes back.  The callee is a C function of the right
    shape (mpx_xfer_ex with a NULL context: it returns MPX_ERR_INVALID
    without touching a GPU)."""
    import ctypes as C

    import mpx
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    bars = [spin.SpinBarrier(name, 2, True), spin.SpinBarrier(name, 2, False)]
    spin.unlink(name)
    fn = C.cast(mpx.lib().mpx_xfer_ex, C.c_void_p)
    o, t = mpx.XferOpts(), mpx.Timing()
    got = []

    def rank(r):
        got.append(bars[r].wait_then(fn, None, mpx.MODE_UNIDIR, r, r, 1 - r, 1, None, None, 8, C.byref(o),
                                     C.byref(t), timeout_s=30))

    th = threading.Thread(target=rank, args=(1,))
    th.start()
    th.join(0.3)
    assert th.is_alive() and not got        # rank 1 waits: rank 0 has not arrived
    rank(0)
    th.join(30)
    assert got == [mpx.ERR_INVALID, mpx.ERR_INVALID]
    for b in bars:
        b.close()


def test_wait_then_times_out_without_calling():
    import ctypes as C

    import mpx
    name = f"/mpxbar-test-{uuid.uuid4().hex[:12]}"
    b = spin.SpinBarrier(name, 2, True)
    spin.unlink(name)
    o, t = mpx.XferOpts(), mpx.Timing()
    with pytest.raises(TimeoutError):
        b.wait_then(C.cast(mpx.lib().mpx_xfer_ex, C.c_void_p), None, mpx.MODE_UNIDIR, 0, 0, 1, 1, None, None, 8,
                    C.byref(o), C.byref(t), timeout_s=0.2)
    b.close()
