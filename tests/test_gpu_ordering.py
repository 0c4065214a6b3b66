"""Matched-receive order across calls (tests/ordering.py has the scenarios).

A payload of call k+1 may land in a rank's rx, ring or LL zone only after
that rank's call k+1 has started: the reference's rx is written only under a
posted receive (/root/reference/mpi_perf.c:75,79,100,104,137,141).  Rank 0
races ahead of rank 1 between two calls with a new payload:

* test_*_lagging_workgroup_*: the non-blocking loop in check mode, one of rank
  1's workgroups late to check call 1's last receive (MPX_TEST lag_wg=...), call 2
  with another length and push width.  Before the receive-posted handshake,
  rank 0's call 2 pushed into rank 1's rx while that workgroup still checked
  it: GPUTEST_r02's "1 of 300 received payloads failed the checksum".
* test_*_rx_read_between_calls_*: rank 1 reads rx on the host between the
  calls and must see call 1's last payload, in every loop, with and without
  check mode, on the kernel and SDMA engines.

Each runs in two forms: two ranks of one context on host threads, and two
processes mapped over IPC (the bench's form).
"""
import json
import os
import subprocess
import sys
import threading

import pytest

import mpx
import ordering as O

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

MODES = {"pingpong": mpx.MODE_PINGPONG, "unidir": mpx.MODE_UNIDIR, "nonblocking": mpx.MODE_NONBLOCKING}
# (n, iters): bulk pushes straight into rx (256 KiB + 13), and an LL size
# (1 KiB: the receiver unpacks into rx itself); 300 non-blocking iterations
# cross a window flush
RACE_CASES = [(262144 + 13, 20), (1024, 20)]


def run_threads(fn, engine="kernel", devs=(0, 0)):
    """two ranks of one context on host threads; rank r on GPU devs[r]"""
    c = mpx.Context(2, engine)
    try:
        bufs, sums = [], []
        for r in range(2):
            d = devs[r]
            scratch = c.alloc(d, O.CAP)
            tx, rx = c.alloc(d, O.CAP), c.alloc(d, O.CAP)
            sums.append(O.pattern_sums(c, scratch, r, 1 - r))
            c.fill(tx, O.CAP, mpx.FILL_SPLITMIX, O.key(r, 1 - r, 0))
            c.fill(rx, O.CAP, mpx.FILL_BYTE, 0)
            c.attach(r, d, tx, rx, O.CAP)
            bufs.append((tx, rx))
        out, errs = {}, {}

        def side(r):
            try:
                out[r] = fn(c, r, bufs[r][0], bufs[r][1], sums[1 - r])
            except Exception as e:  # noqa: BLE001
                errs[r] = e

        th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        return out
    finally:
        c.close()


def run_processes(tmp_path, engine, args, env_extra=None, cross=False):
    """two processes, IPC-mapped; cross: rank r on GPU r (MPX_ORDER_CROSS)"""
    env = dict(os.environ, **(env_extra or {}))
    if cross:
        env["MPX_ORDER_CROSS"] = "1"
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "order_worker.py"), str(tmp_path), str(r), engine,
                               *[str(a) for a in args]], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                              env=env) for r in (0, 1)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    assert all(p.returncode == 0 for p in procs), outs
    return {r: json.load(open(tmp_path / f"result_{r}.json")) for r in (0, 1)}


def assert_lag_ok(out):
    for r in (0, 1):
        for call in ("call1", "call2"):
            x = out[r][call]
            assert x["ok"], (r, call, x)
            assert x["check_iters"] == O.LAG_ITERS, (r, call, x)
        assert out[r]["call2"]["nwg"] == O.LAG_NWG2, out[r]
    assert out[0]["call1"]["nwg"] > O.LAG_NWG2, out   # call 2 narrows the push: every chunk boundary moves


def assert_race_ok(out):
    for r in (0, 1):
        assert out[r]["call1"]["ok"] and out[r]["call2"]["ok"], (r, out[r])
        assert out[r]["rx_after_is_call2"], (r, out[r])
    assert out[1]["rx_between_is_call1"], out[1]


def test_lagging_workgroup_layout_change_threads(monkeypatch):
    for k, v in O.lag_env().items():
        monkeypatch.setenv(k, v)
    assert_lag_ok(run_threads(O.lag))


def test_lagging_workgroup_layout_change_processes(tmp_path):
    assert_lag_ok(run_processes(tmp_path, "kernel", ["lag"], O.lag_env()))


# ---- pull mode (MPX_XFER_PULL): the sender's call waits for the peer's loads -
def test_pull_lagging_receiver_keeps_the_senders_tx_threads(monkeypatch):
    """Rank 1's last workgroup stalls before loading call 1's last payload;
    rank 0 rewrites tx as soon as its call 1 returns.  Every payload of both
    calls must still pass: rank 0's call returns only after rank 1's loads."""
    for k, v in O.lag_env().items():
        monkeypatch.setenv(k, v)
    assert_lag_ok(run_threads(lambda c, r, tx, rx, s: O.lag(c, r, tx, rx, s, pull=True)))


def test_pull_lagging_receiver_keeps_the_senders_tx_processes(tmp_path):
    assert_lag_ok(run_processes(tmp_path, "kernel-pull", ["lag"], O.lag_env()))


def test_pull_lagging_receiver_fails_without_the_wait(monkeypatch):
    """Negative control: MPX_TEST=no_pull_wait lets rank 0's call return
    before rank 1's stalled workgroup loaded its chunk; rank 0's new tx then
    lands in call 1's last payload and rank 1's check reports it."""
    for k, v in O.lag_env("no_pull_wait").items():
        monkeypatch.setenv(k, v)
    out = run_threads(lambda c, r, tx, rx, s: O.lag(c, r, tx, rx, s, pull=True))
    assert not out[1]["call1"]["ok"] and "failed the checksum" in out[1]["call1"]["error"], out


@pytest.mark.parametrize("check", [False, True])
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_pull_rx_read_between_calls_threads(engine, mode, check):
    n, iters = RACE_CASES[0]
    it = 300 if mode == "nonblocking" else iters
    out = run_threads(lambda c, r, tx, rx, s: O.race(c, r, tx, rx, s, MODES[mode], check, n, it, pull=True), engine)
    assert_race_ok(out)


@pytest.mark.parametrize("n,iters", RACE_CASES)
@pytest.mark.parametrize("check", [False, True])
@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_rx_read_between_calls_threads(engine, mode, check, n, iters):
    it = 300 if mode == "nonblocking" else iters
    out = run_threads(lambda c, r, tx, rx, s: O.race(c, r, tx, rx, s, MODES[mode], check, n, it), engine)
    assert_race_ok(out)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_rx_read_between_calls_processes(tmp_path, engine, mode):
    n, iters = RACE_CASES[0]
    it = 300 if mode == "nonblocking" else iters
    assert_race_ok(run_processes(tmp_path, engine, ["race", MODES[mode], 0, n, it]))


# ---- negative controls: the same scenarios without the handshake ----------
# MPX_TEST=no_posted restores round 2's behaviour (a sender pushes call k+1
# as soon as its own sequence and credit state allows).  Both scenarios must
# then fail, which shows they detect the race they are there for.

def test_lagging_workgroup_fails_without_the_handshake(monkeypatch):
    for k, v in O.lag_env("no_posted").items():
        monkeypatch.setenv(k, v)
    out = run_threads(O.lag)
    assert not out[1]["call1"]["ok"] and "failed the checksum" in out[1]["call1"]["error"], out


def test_rx_read_between_calls_fails_without_the_handshake(monkeypatch):
    monkeypatch.setenv("MPX_TEST", "no_posted")
    n, iters = RACE_CASES[0]
    out = run_threads(lambda c, r, tx, rx, s: O.race(c, r, tx, rx, s, mpx.MODE_PINGPONG, False, n, iters))
    assert not out[1]["rx_between_is_call1"], out
