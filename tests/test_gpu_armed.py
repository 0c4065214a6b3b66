"""Armed transfers (mpx_xfer_arm / mpx_xfer_disarm, include/mpx.h): the
kernel is launched before the hosts' barrier and started by a host-memory
word after it, MPI's persistent-request split (MPI_Send_init ... MPI_Start).
An armed call must move and account exactly what the same call unarmed does
— every payload checked against the peer's tx, the receive count and digest
the reference's loop completes — and a call that is armed but never started
must leave no trace on the link (its call number is taken back, so the
receive-posted handshake of later calls still lines up)."""
import threading

import pytest

import mpx
from pairs import Pairs

pytestmark = pytest.mark.gpu

MODES = [mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING, mpx.MODE_UNIDIR]
# LL sizes (<= 2 KiB within one GPU), bulk, ragged, the non-blocking window
CASES = [(8, 40), (1000, 7), (2049, 5), (65536 + 13, 9), ((1 << 20) + 3, 3), (4096, 300)]


@pytest.mark.parametrize("pull", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_armed_calls_match_unarmed(mode, pull):
    """Alternating armed and unarmed calls on one link, every payload
    checked: same check results, receive counts and digests, and rx ends
    holding the peer's tx."""
    P = Pairs("kernel", 1, (1 << 20) + 64, fill="seeded")
    try:
        for n, iters in CASES:
            res = {}
            for armed in (True, False, True):
                out, errs = P.run(mode, n, iters, pull=pull, armed=armed)
                assert not errs, (n, iters, armed, errs)
                for r in (0, 1):
                    assert out[r].check_failures == 0 and out[r].check_iters == iters
                    assert P.c.phases(r)["armed"] == (1 if armed else 0)
                    if not armed:
                        assert P.c.phases(r)["resident"] == 0
                res.setdefault("sig", (out[0].recv_done, out[0].recv_digest, out[1].recv_done, out[1].recv_digest))
                assert (out[0].recv_done, out[0].recv_digest, out[1].recv_done, out[1].recv_digest) == res["sig"]
                for r in (0, 1):
                    m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                    assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m)
    finally:
        P.close()


def test_armed_phases_exclude_the_launch():
    """An armed call's phases: host_prep 0, launch_to_start is the go word's
    trip (no kernel launch), kernel_s within the wall time."""
    P = Pairs("kernel", 1, 1 << 20)
    try:
        for _ in range(3):
            out, errs = P.run(mpx.MODE_UNIDIR, 456131, 10, check=False, armed=True)
            assert not errs, errs
        for r in (0, 1):
            ph = P.c.phases(r)
            assert ph["armed"] == 1 and ph["host_prep_s"] == 0
            # two small grids on one GPU: both fully running before the start
            assert ph["resident"] == 1
            assert 0 < ph["kernel_s"] <= ph["wall_s"]
            assert out[r].device_s == pytest.approx(ph["kernel_s"])
    finally:
        P.close()


def test_mismatched_start_fails_and_leaves_the_call_armed():
    P = Pairs("kernel", 1, 1 << 16)
    try:
        c = P.c
        tx0, rx0 = P.bufs[0]
        c.arm(mpx.MODE_UNIDIR, 1, 0, 1, 5, tx0, rx0, 4096)
        with pytest.raises(mpx.MpxError) as e:
            c.xfer(mpx.MODE_UNIDIR, 1, 0, 1, 6, tx0, rx0, 4096)      # other iteration count
        assert e.value.status == mpx.ERR_STATE and "armed for another call" in str(e.value)
        with pytest.raises(mpx.MpxError) as e:
            c.arm(mpx.MODE_UNIDIR, 1, 0, 1, 5, tx0, rx0, 4096)       # one armed call per rank
        assert e.value.status == mpx.ERR_STATE
        c.disarm(0)
        out, errs = P.run(mpx.MODE_UNIDIR, 4096, 5)
        assert not errs, errs
    finally:
        P.close()


@pytest.mark.parametrize("mode", MODES)
def test_disarmed_calls_leave_the_link_in_step(mode):
    """Both sides arm, neither starts, both disarm — twice; one side arms
    and disarms alone; then unarmed and armed calls still pass every check
    (call numbers, sequence numbers and scratch words untouched)."""
    P = Pairs("kernel", 1, 1 << 20, fill="seeded")
    try:
        c = P.c
        for _ in range(2):
            for r in (0, 1):
                c.arm(mode, P.group(r), r, P.peer(r), 9, P.bufs[r][0], P.bufs[r][1], 70000)
            for r in (0, 1):
                c.disarm(r)
        c.arm(mode, 1, 0, 1, 3, P.bufs[0][0], P.bufs[0][1], 100)
        c.disarm(0)
        for armed in (False, True, False):
            out, errs = P.run(mode, 70000, 9, armed=armed)
            assert not errs, (armed, errs)
            assert all(out[r].check_failures == 0 for r in (0, 1))
    finally:
        P.close()


@pytest.mark.parametrize("mode", MODES)
def test_failed_launch_gives_its_call_number_back(mode, monkeypatch):
    """A call whose launch fails after prepare_call took its numbers
    (MPX_TEST fail_launch=0: rank 0's kernel is never enqueued), armed and
    unarmed, then normal calls on the same link: they must pass every check.
    Without the rollback, rank 0 posts a call number one higher than rank 1
    ever sends and every later call times out."""
    P = Pairs("kernel", 1, 1 << 20, fill="seeded")
    try:
        c = P.c
        monkeypatch.setenv("MPX_TEST", "fail_launch=0")
        with pytest.raises(mpx.MpxError) as e:
            c.arm(mode, P.group(0), 0, 1, 9, P.bufs[0][0], P.bufs[0][1], 70000)
        assert "fail_launch" in str(e.value)
        with pytest.raises(mpx.MpxError) as e:
            c.xfer(mode, P.group(0), 0, 1, 9, P.bufs[0][0], P.bufs[0][1], 70000)
        assert "fail_launch" in str(e.value)
        monkeypatch.setenv("MPX_TEST", "")
        for armed in (False, True, False):
            out, errs = P.run(mode, 70000, 9, armed=armed)
            assert not errs, (armed, errs)
            assert all(out[r].check_failures == 0 and out[r].check_iters == 9 for r in (0, 1))
    finally:
        P.close()


def test_finalize_cancels_an_armed_call():
    """mpx_finalize with armed ranks: the kernels are cancelled and the
    context closes; a new context on the same GPU then works."""
    P = Pairs("kernel", 1, 1 << 16)
    c = P.c
    for r in (0, 1):
        c.arm(mpx.MODE_PINGPONG, P.group(r), r, P.peer(r), 4, P.bufs[r][0], P.bufs[r][1], 512)
    P.close()
    Q = Pairs("kernel", 1, 1 << 16)
    try:
        out, errs = Q.run(mpx.MODE_PINGPONG, 512, 4, armed=True)
        assert not errs, errs
    finally:
        Q.close()


def test_arm_is_a_no_op_on_the_stream_engines():
    P = Pairs("sdma", 1, 1 << 16)
    try:
        out, errs = P.run(mpx.MODE_UNIDIR, 4096, 5, armed=True)
        assert not errs, errs
        assert all(out[r].check_failures == 0 for r in (0, 1))
    finally:
        P.close()
