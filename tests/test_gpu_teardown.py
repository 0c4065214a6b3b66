"""Stream teardown mid-process (round 5, DESIGN.md §5 "Exit").

Rounds 2-4 could not destroy CU-masked rank streams while the process ran:
the destroy raced HIP's completion handler of the stream's last command,
whose release then ran the queue's destruction on the HSA events thread,
which deadlocked on itself (profiles/r05_exit_stall_symbolized.txt).
callback_fence now waits for that handler (event_thread_barrier), so
mpx_shutdown can destroy the pooled rank streams between contexts, every
time, and the next context creates fresh ones.  Each case runs in a child
process under a time limit: a stall ends the child, not the suite."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))

CYCLES = """
import sys, threading
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {here!r})
import mpx
from pairs import Pairs
for k in range({n}):
    P = Pairs({engine!r}, {npairs}, 1 << 16, fill="seeded")
    try:
        out, errs = P.run(mpx.MODE_PINGPONG, 4096, 3)
        assert not errs, errs
        assert all(o.check_failures == 0 for o in out.values())
    finally:
        P.close()
    mpx.shutdown()   # every rank stream destroyed; the next cycle creates new ones
print("cycles done", {n}, flush=True)
"""


@pytest.mark.parametrize("engine,npairs", [("kernel", 1), ("kernel", 2), ("sdma", 1)])
def test_rank_streams_destroyed_and_recreated_every_cycle(engine, npairs):
    """30 cycles of: a context with 2 x npairs ranks on GPU 0, a checked
    ping-pong on every pair, finalize, mpx_shutdown (the rank streams are
    destroyed), in ONE process; then the process exits normally."""
    code = CYCLES.format(pkg=os.path.join(os.path.dirname(HERE), "mpi-perf_amd"), here=HERE, n=30, engine=engine,
                         npairs=npairs)
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=100,
                       env=dict(os.environ))
    assert r.returncode == 0 and "cycles done 30" in r.stdout, (r.returncode, r.stdout[-400:], r.stderr[-800:])


@pytest.mark.parametrize("nbytes,iters", [(1 << 20, 4), (64 << 20, 2), (4096, 1)])
def test_failed_copy_leaks_no_event_and_the_next_copy_works(monkeypatch, nbytes, iters):
    """MPX_TEST=fail_copy: mpx_copy fails after both of its events were
    created and the start one recorded (an early return through HIPCK's
    path).  The events are owned by RAII holders: the
    process's live-event count is the same after the failure, and a normal
    copy in the same context then succeeds and copies (every copy form:
    pipe, a launch per copy, one launch)."""
    import mpx
    c = mpx.Context(1, "kernel")
    try:
        src, dst = c.alloc(0, nbytes), c.alloc(0, nbytes)
        c.fill(src, nbytes, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, 5, 0, 0))
        c.fill(dst, nbytes, mpx.FILL_BYTE, 0)
        before = mpx.live_events()
        for _ in range(3):
            monkeypatch.setenv("MPX_TEST", "fail_copy")
            with pytest.raises(mpx.MpxError, match="fail_copy"):
                c.copy(0, dst, src, nbytes, iters)
            monkeypatch.setenv("MPX_TEST", "")
            assert mpx.live_events() == before
        t = c.copy(0, dst, src, nbytes, iters)
        assert t.launches >= 1 and mpx.live_events() == before
        assert c.checksum(dst, nbytes) == c.checksum(src, nbytes)
    finally:
        monkeypatch.setenv("MPX_TEST", "")
        c.close()
    assert mpx.live_events() == before   # the context attached no rank: it held no event of its own


SHUTDOWN_TWICE = """
import sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {here!r})
import mpx
from pairs import Pairs
P = Pairs("kernel", 1, 1 << 16, fill="seeded")
try:
    out, errs = P.run(mpx.MODE_UNIDIR, 4096, 3)
    assert not errs and all(o.check_failures == 0 for o in out.values()), errs
finally:
    P.close()
mpx.shutdown()
mpx.shutdown()          # nothing pooled: a no-op, not a second destroy of the same streams
P = Pairs("kernel", 1, 1 << 16, fill="seeded")   # fresh rank streams
try:
    out, errs = P.run(mpx.MODE_PINGPONG, 4096, 3)
    assert not errs and all(o.check_failures == 0 for o in out.values()), errs
    try:
        mpx.shutdown()  # a context is alive: refused, nothing destroyed
        raise SystemExit("shutdown with a live context was not refused")
    except mpx.MpxError as e:
        assert e.status == mpx.ERR_STATE, e
    out, errs = P.run(mpx.MODE_PINGPONG, 4096, 3)
    assert not errs, errs
finally:
    P.close()
mpx.shutdown()
print("shutdown ok", flush=True)
"""


def test_shutdown_twice_and_refused_while_a_context_lives():
    """mpx_shutdown forgets every stream it destroyed: a second
    call is a no-op; while a context is alive it is refused (MPX_ERR_STATE)
    and the context's streams keep working; a later context gets fresh ones."""
    code = SHUTDOWN_TWICE.format(pkg=os.path.join(os.path.dirname(HERE), "mpi-perf_amd"), here=HERE)
    r = subprocess.run([sys.executable, "-u", "-c", code], capture_output=True, text=True, timeout=100,
                       env=dict(os.environ))
    assert r.returncode == 0 and "shutdown ok" in r.stdout, (r.returncode, r.stdout[-400:], r.stderr[-800:])
