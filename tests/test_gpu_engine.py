"""GPU parity tests of libmpx through its C-ABI (run with -m gpu on an MI355X).

Every result is checked against the oracle (oracle/mpx_oracle.c) or against
the compiled reference's golden receive accounting (tests/golden).  Pairs run
as loopback ranks on GPU 0 (two ranks of one process on one device, one host
thread each) — the same kernel, mailbox protocol and sequence bookkeeping the
cross-GPU path uses, with the peer's HBM being local HBM.
"""
import threading

import pytest

import mpx
import oracle_py as O
from pairs import Pairs

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 7, 8, 15, 16, 17, 255, 4095, 4096, 65537, (1 << 20) + 3, (2 << 20) + 5, (64 << 20) + 13]
GOLDEN = {c["name"]: c for c in O.golden()["cases"]}


@pytest.fixture(scope="module")
def ctx():
    c = mpx.Context(8, "kernel")
    yield c
    c.close()


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("pattern", [mpx.FILL_BYTE, mpx.FILL_SPLITMIX])
def test_fill_and_checksum_match_oracle(ctx, n, pattern):
    arg = ord("a") if pattern == mpx.FILL_BYTE else mpx.pattern_key(mpx.PATTERN_SEED, 1, 2, 3)
    b = ctx.alloc(0, max(n, 1))
    try:
        ctx.fill(b, n, pattern, arg)
        want = O.pattern_checksum(n, pattern, arg)
        assert ctx.checksum(b, n) == want
        if n <= 4096:
            assert ctx.read(b, n) == O.fill(n, pattern, arg)
    finally:
        ctx.free(b)


@pytest.mark.parametrize("iters", [1, 2, 7])
@pytest.mark.parametrize("n", [1, 4096 + 5, 16 << 10, (16 << 10) + 1, (128 << 10) + 1, (512 << 10) + 7, (1 << 20),
                               (1 << 20) + 3, (2 << 20) + 16, (8 << 20) + 1])
def test_copy_steps_every_size_class(ctx, monkeypatch, n, iters):
    """k_copy_steps (all copies in one launch, grid barrier between steps),
    forced at every size (MPX_COPY=steps): the grid classes of its
    defaults (1024-lane workgroups, one unit per lane: one workgroup up to
    16 KiB, <= 64 workgroups up to 1 MiB; 64 256-lane workgroups with 8
    units per lane above, in load batches) on both sides of each class
    boundary and of the 1 MiB default threshold, plus the A/B knob
    combinations (grid cap — clamped to what stays resident —, per-XCD
    counters, drain, units per lane, 256 / 512 / 1024 lanes, every working
    workgroup on one XCD) at 1 MiB + 3:
    output against the oracle's pattern, nothing written past the end."""
    monkeypatch.setenv("MPX_COPY", "steps")
    key = mpx.pattern_key(mpx.PATTERN_SEED, 1, 1, n & 0xFFFF)
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n + 64)
    try:
        ctx.fill(src, n, mpx.FILL_SPLITMIX, key)
        variants = [None] + (["64:0:1:1:256", "256:1:1:8:256", "1024:1:0:2:256", "1:0:0:1:256", "64:0:0:8:256",
                              "16:0:0:3:256", "64:0:0:1:512", "1:0:0:8:1024", "2:1:1:3:1024", "1024:0:0:1:1024",
                              "9:1:0:1:1024", "32:0:0:1:1024:1", "64:1:1:2:512:1"]
                             if n == (1 << 20) + 3 else [])
        for v in variants:
            if v:
                monkeypatch.setenv("MPX_COPY", "steps:" + v)
            ctx.fill(dst, n + 64, mpx.FILL_BYTE, 0xEE)
            t = ctx.copy(0, dst, src, n, iters)
            # one copy is one plain k_copy launch; more run as k_copy_steps
            assert t.launches == 1 and mpx.PROTOCOLS.get(t.protocol) == ("copy_steps" if iters > 1 else "copy"), \
                (v, t.protocol)
            assert ctx.checksum(dst, n) == O.pattern_checksum(n, mpx.FILL_SPLITMIX, key), v
            assert ctx.read(dst, 64, offset=n) == b"\xee" * 64
            assert t.bytes == n * iters
    finally:
        ctx.free(src)
        ctx.free(dst)


@pytest.mark.parametrize("upl", [0, 1, 2, 8, 16])
@pytest.mark.parametrize("iters", [1, 2, 3, 7])
@pytest.mark.parametrize("n", [1, 15, 16, 17, 4096 + 5, (1 << 20) + 3, (2 << 20) + 16, (4 << 20), (16 << 20) + 7])
def test_copy_pipe_every_size_class(ctx, monkeypatch, n, iters, upl):
    """k_copy_pipe (all copies in one launch; copy s+1's loads in flight
    across copy s's grid barrier; a dedicated barrier wave), forced at every
    size (MPX_COPY=pipe) and units-per-lane choice (MPX_COPY=pipe:<upl>; 0 =
    the default 4, widened until the grid stays resident): odd and even copy
    counts (the loop is unrolled by two), a tail below 16 B with and without
    a body, a grid of one: output against the oracle's pattern, nothing
    written past the end."""
    monkeypatch.setenv("MPX_COPY", f"pipe:{upl}")
    key = mpx.pattern_key(mpx.PATTERN_SEED, 2, 2, (n + upl) & 0xFFFF)
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n + 64)
    try:
        ctx.fill(src, n, mpx.FILL_SPLITMIX, key)
        ctx.fill(dst, n + 64, mpx.FILL_BYTE, 0xEE)
        t = ctx.copy(0, dst, src, n, iters)
        assert t.launches == 1 and mpx.PROTOCOLS.get(t.protocol) == ("copy_pipe" if iters > 1 else "copy"), \
            t.protocol
        assert ctx.checksum(dst, n) == O.pattern_checksum(n, mpx.FILL_SPLITMIX, key)
        assert ctx.read(dst, 64, offset=n) == b"\xee" * 64
        assert t.bytes == n * iters
    finally:
        ctx.free(src)
        ctx.free(dst)


@pytest.mark.parametrize("n,grid", [(1, 1), (4096, 1), (16 << 10, 1), ((16 << 10) + 1, 2), (32 << 10, 4),
                                    (128 << 10, 16), ((128 << 10) + 16, 9), (512 << 10, 32), ((512 << 10) + 16, 33),
                                    (1 << 20, 64)])
def test_copy_steps_grid_rule(ctx, monkeypatch, n, grid):
    """The k_copy_steps shape (mpx_kernels.hip launch_copy_steps): one
    1024-lane workgroup up to 16 KiB; 512-lane workgroups on one XCD to
    128 KiB, 1024-lane ones on one XCD to 512 KiB; up to 64 1024-lane
    workgroups over every XCD to 1 MiB (above 512 KiB only with the pipe off,
    as here).  timing.nwg = working workgroups."""
    monkeypatch.setenv("MPX_COPY", "steps")
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n)
    try:
        ctx.fill(src, n, mpx.FILL_BYTE, 0x5C)
        t = ctx.copy(0, dst, src, n, 3)
        assert (mpx.PROTOCOLS[t.protocol], t.nwg) == ("copy_steps", grid)
        assert ctx.checksum(dst, n) == ctx.checksum(src, n)
    finally:
        ctx.free(src)
        ctx.free(dst)


@pytest.mark.parametrize("n,grid", [((512 << 10) + 16, 17), (1 << 20, 32), ((1 << 20) + 16, 65), (2 << 20, 128),
                                    ((2 << 20) + 16, 129), (3 << 20, 192), (4 << 20, 256), (8 << 20, 256),
                                    ((8 << 20) + 16, 129), (16 << 20, 256)])
def test_copy_pipe_grid_rule(ctx, n, grid):
    """The one-launch form of 512 KiB - 16 MiB (k_copy_pipe): 320-lane
    workgroups (four copy waves + the barrier wave); up to 1 MiB 8 units per
    lane and one barrier counter (16-32 workgroups), above it the two-level
    barrier with up to 256 workgroups of 4-16 units per lane.
    timing.nwg = workgroups."""
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n)
    try:
        ctx.fill(src, n, mpx.FILL_BYTE, 0x5D)
        t = ctx.copy(0, dst, src, n, 3)
        assert (mpx.PROTOCOLS[t.protocol], t.nwg, t.launches) == ("copy_pipe", grid, 1)
        assert ctx.checksum(dst, n) == ctx.checksum(src, n)
    finally:
        ctx.free(src)
        ctx.free(dst)


@pytest.mark.parametrize("hier", ["0", "1"])
@pytest.mark.parametrize("iters", [2, 5])
@pytest.mark.parametrize("n,upl", [(16, 1), (4096 * 5 + 3, 1), (256 << 10, 16), ((256 << 10) + 16, 1),
                                   ((1 << 20) + 7, 2), (9 << 20, 16), ((2 << 20) + 48, 4)])
def test_copy_pipe_barrier_forms(ctx, monkeypatch, n, upl, iters, hier):
    """Both grid-barrier forms of k_copy_pipe (one counter; 8 group counters
    + release words) at grids of 1, 5, 4 (fewer workgroups than groups), 65,
    129 (groups of unequal size), 128 and 144 workgroups, odd and even copy
    counts: output against the oracle, nothing written past the end."""
    monkeypatch.setenv("MPX_COPY", f"pipe:{upl}:{hier}")
    key = mpx.pattern_key(mpx.PATTERN_SEED, 3, 3, (n + iters) & 0xFFFF)
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n + 64)
    try:
        ctx.fill(src, n, mpx.FILL_SPLITMIX, key)
        ctx.fill(dst, n + 64, mpx.FILL_BYTE, 0xEE)
        t = ctx.copy(0, dst, src, n, iters)
        assert mpx.PROTOCOLS[t.protocol] == "copy_pipe" and t.launches == 1
        assert ctx.checksum(dst, n) == O.pattern_checksum(n, mpx.FILL_SPLITMIX, key)
        assert ctx.read(dst, 64, offset=n) == b"\xee" * 64
    finally:
        ctx.free(src)
        ctx.free(dst)


def copy_path(n: int, iters: int) -> str:
    """mpx_copy's default form: one launch for all copies (k_copy_steps up to
    512 KiB, k_copy_pipe to 16 MiB), a k_copy launch per copy above"""
    if not n or iters < 2 or n > (16 << 20):
        return "copy"
    return "copy_steps" if n <= (512 << 10) else "copy_pipe"


@pytest.mark.parametrize("n", SIZES)
def test_copy_kernel_matches_oracle(ctx, n):
    key = mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, n & 0xFFFF)
    src, dst = ctx.alloc(0, max(n, 1)), ctx.alloc(0, max(n, 1) + 64)
    try:
        ctx.fill(src, n, mpx.FILL_SPLITMIX, key)
        ctx.fill(dst, n + 64, mpx.FILL_BYTE, 0xEE)
        t = ctx.copy(0, dst, src, n, 2)
        assert ctx.checksum(dst, n) == O.pattern_checksum(n, mpx.FILL_SPLITMIX, key)
        # nothing written past the end
        assert ctx.read(dst, 64, offset=n) == b"\xee" * 64
        assert t.bytes == 2 * n
        # both copies in one launch up to 16 MiB, a launch each above
        one = copy_path(n, 2) != "copy"
        assert t.launches == (1 if one else 2 if n else 0)
        if n:
            assert mpx.PROTOCOLS[t.protocol] == copy_path(n, 2)
    finally:
        ctx.free(src)
        ctx.free(dst)


# --------------------------------------------------------------------------
# loopback pairs (tests/pairs.py; every rank on GPU 0)
# --------------------------------------------------------------------------
MODES = [mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING, mpx.MODE_UNIDIR]
PAIR_SIZES = [0, 1, 8, 4097, 8192, 8193, 65541, 456131, 4 << 20]


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
@pytest.mark.parametrize("mode", MODES)
def test_loopback_pair_every_payload(engine, mode):
    P = Pairs(engine, 1, 4 << 20)
    try:
        for n in PAIR_SIZES:
            iters = 300 if (mode == mpx.MODE_NONBLOCKING and n <= 65541) else 7
            out, errs = P.run(mode, n, iters)
            assert not errs, (n, errs)
            for r in (0, 1):
                t = out[r]
                assert t.check_iters == iters and t.check_failures == 0, (n, r)
                assert t.recv_done == (O.lib().oracle_nb_waited(iters) if mode == mpx.MODE_NONBLOCKING else iters)
                assert t.bytes == n * iters * (1 if mode == mpx.MODE_UNIDIR else 2)
            # the delivered bytes: G0 rx = G1's tx; G1 rx = G0's tx (all of it,
            # or its first byte for unidir's 1-byte ack, mpi_perf.c:137,142)
            for r in (0, 1):
                m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                want = P.c.checksum(P.bufs[P.peer(r)][0], m)
                assert P.c.checksum(P.bufs[r][1], m) == want, (n, r)
    finally:
        P.close()


# (push workgroups, B): chunk = ceil(B / nwg) rounded up to 16 B; chunks of
# <= 60 KiB are pushed from LDS (stage_tx), larger ones straight from HBM; a
# width wider than B / 1 KiB is narrowed to that (run_kernel, kMinPushChunk)
PUSH_CASES = [(1, 40000), (1, 70001), (7, 456131), (8, 456131), (33, (1 << 20) + 17), (128, (4 << 20) + 3),
              (256, (20 << 20) + 5), (64, 20000), (256, 3000)]


@pytest.mark.parametrize("stream", [False, True])
@pytest.mark.parametrize("mode", MODES)
def test_push_widths_staged_and_unstaged(mode, stream):
    """Bulk pushes at explicit widths (mpx_xfer_opts.nwg, as bench.py's tuner
    sets them), with and without the streaming store hint, both sides of the
    60 KiB LDS-staging limit, ragged sizes: every payload checksummed, the
    final rx compared with the peer's tx."""
    P = Pairs("kernel", 1, (20 << 20) + 5, fill="pattern")
    try:
        for nwg, n in PUSH_CASES:
            out, errs = P.run(mode, n, 5, nwg=nwg, stream=stream)
            assert not errs, (nwg, n, errs)
            for r in (0, 1):
                pushes = mode != mpx.MODE_UNIDIR or r == 0
                if pushes:
                    assert out[r].nwg == min(nwg, -(-n // 1024)) and out[r].protocol == 1, (nwg, n, r)
                assert out[r].check_failures == 0 and out[r].check_iters == 5
                m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (nwg, n, r)
    finally:
        P.close()


@pytest.mark.parametrize("mode", MODES)
def test_sdma_graph_chunks_keep_sequence_state(mode):
    """SDMA engine without check mode replays graph-captured 256-iteration
    chunks (run_sdma) plus a plain remainder; the link's sequence numbers must
    come out exactly where the plain loop leaves them, so a checked run after
    it still validates every payload."""
    P = Pairs("sdma", 1, 65541, fill="pattern")
    try:
        for n, iters in [(65541, 519), (8, 256), (4096, 300), (1, 3)]:
            out, errs = P.run(mode, n, iters, check=False)
            assert not errs, (n, iters, errs)
            assert all(out[r].launches > 0 for r in (0, 1))
            for r in (0, 1):
                m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (n, r)
            out, errs = P.run(mode, n, 5, check=True)
            assert not errs, (n, "checked run after chunks", errs)
            assert all(out[r].check_failures == 0 and out[r].check_iters == 5 for r in (0, 1))
    finally:
        P.close()


def _digest_cases():
    """Every golden run that transfers data in the -p layout (ranks [0, p) in
    group 1, rank k paired with p + k): all mode x ppn x size cases, the
    non-blocking window quirk, defaults, 0 bytes, 0 iterations, 0 runs, -u 1
    over -x 1, the 1002-run summary case and the 2^31 - 1-byte buffer."""
    out = []
    for c in O.golden()["cases"]:
        a = c["args"]
        if c.get("returncode") or not c.get("shim") or "-d" in a or c["np"] != 2 * c["ppn"]:
            continue
        if a[a.index("-n") + 1] != "1":
            continue
        out.append(c["name"])
    return out


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
@pytest.mark.parametrize("name", _digest_cases())
def test_receive_digest_matches_reference(name, engine):
    """Runs the golden case's configuration (pairs, mode, B, iters, runs) on the
    GPU with every payload checksummed, and compares each rank's receive
    accounting — counted on the device: which receives completed (every
    Recv; the requests each Waitall of the non-blocking loop waited for),
    their bytes, and the sum of their checksums — with what the compiled
    reference's ranks received (the PMPI shim's recv_done / recv_bytes /
    recv_digest).  Nothing here comes from the oracle."""
    c = GOLDEN[name]
    a = c["args"]
    ppn = c["ppn"]
    runs = int(a[a.index("-r") + 1])
    iters = int(a[a.index("-i") + 1]) if "-i" in a else 10
    B = int(a[a.index("-b") + 1]) if "-b" in a else 456131
    mode = mpx.MODE_UNIDIR if "-u" in a else (mpx.MODE_NONBLOCKING if "-x" in a else mpx.MODE_PINGPONG)
    P = Pairs(engine, ppn, B)   # B = 0: mpx_alloc's zeroed pad, whose byte 0 the unidir ack sends (mpi_perf.c:142)
    try:
        digest = {r: [0, 0, 0] for r in range(2 * ppn)}
        for _ in range(runs):
            out, errs = P.run(mode, B, iters)
            assert not errs, errs
            for r in range(2 * ppn):
                ack = mode == mpx.MODE_UNIDIR and P.group(r) == 1
                m = 1 if ack else B
                assert out[r].check_failures == 0 and out[r].check_iters == iters
                digest[r][0] += out[r].recv_done
                digest[r][1] += out[r].recv_done * m
                digest[r][2] = (digest[r][2] + out[r].recv_digest) & 0xFFFFFFFFFFFFFFFF
        for r in range(2 * ppn):
            ref = c["shim"][str(r)]
            assert digest[r] == [ref["recv_done"], ref["recv_bytes"], ref["recv_digest"]], r
    finally:
        P.close()


NB_ITERS = [1, 254, 255, 256, 257, 511, 512, 600]


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
@pytest.mark.parametrize("n", [0, 1, 4097, 65541, 456131])
def test_nonblocking_every_payload_seeded(engine, n):
    """-x 1 with seeded payloads: every one of the (up to 256 concurrent)
    receives is checksummed on the device in a slot of its own; the device
    counts exactly the receives the reference's Waitall calls complete
    (iters - iters // 256: slot 255 of each full window is never waited
    for, mpi_perf.c:108-111) and digests them; rx ends holding the last
    payload."""
    P = Pairs(engine, 1, max(n, 1), fill="seeded")
    try:
        for iters in NB_ITERS:
            out, errs = P.run(mpx.MODE_NONBLOCKING, n, iters)
            assert not errs, (iters, errs)
            for r in (0, 1):
                t = out[r]
                assert t.check_iters == iters and t.check_failures == 0, (iters, r)
                k = iters - iters // 256
                assert k == O.lib().oracle_nb_waited(iters)
                assert t.recv_done == k, (iters, r, t.recv_done)
                one = P.expect(r, n)[0]
                assert t.recv_digest == (k * one) & 0xFFFFFFFFFFFFFFFF, (iters, r)
                assert P.c.checksum(P.bufs[r][1], n) == one
    finally:
        P.close()


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("skip", [1, 7, 256])
def test_lost_payload_fails_the_check(monkeypatch, engine, mode, skip):
    """Test knob MPX_TEST=skip_push=k: the k-th push of each call moves no
    payload bytes but is still signalled.  Check mode must then report the
    receive that never got its payload (a checker that only looked at the
    final rx, or took receive counts from elsewhere, would pass)."""
    monkeypatch.setenv("MPX_TEST", f"skip_push={skip}")
    n = 65541 if skip != 7 else 1000   # 1000 B: the LL protocol for ping-pong / unidir
    P = Pairs(engine, 1, n, fill="seeded")
    try:
        out, errs = P.run(mode, n, 300)
        for r in (0, 1):
            receives_payload = not (mode == mpx.MODE_UNIDIR and r == 0)   # G1 receives 1-byte acks
            if receives_payload:
                assert r in errs and errs[r].status == mpx.ERR_CHECK, (r, errs, out.get(r))
    finally:
        P.close()


def test_sequence_state_across_runs_and_sizes():
    """One link reused across protocols: LL -> bulk -> LL -> nb -> unidir."""
    P = Pairs("kernel", 1, 1 << 20, fill="pattern")
    try:
        for mode, n, it in [(0, 8, 5), (0, 100000, 3), (2, 4096, 9), (1, 1000, 600), (2, 300000, 4),
                            (0, 1, 11), (1, 1 << 20, 3), (2, 0, 5)]:
            out, errs = P.run(mode, n, it)
            assert not errs, (mode, n, errs)
    finally:
        P.close()


def test_concurrent_pairs():
    P = Pairs("kernel", 4, 456131, fill="pattern")
    try:
        for mode in MODES:
            out, errs = P.run(mode, 456131, 5)
            assert not errs, errs
    finally:
        P.close()


def test_timeout_when_peer_never_runs():
    P = Pairs("kernel", 1, 65536)
    try:
        out, errs = P.run(mpx.MODE_PINGPONG, 65536, 3, timeout_ms=300, ranks=[0])
        assert 0 in errs and errs[0].status == mpx.ERR_TIMEOUT
        # the link state is unknown afterwards: further transfers are refused
        out, errs = P.run(mpx.MODE_PINGPONG, 8, 1, timeout_ms=300, ranks=[0])
        assert errs[0].status == mpx.ERR_STATE
    finally:
        P.close()


@pytest.mark.parametrize("check", [True, False])
@pytest.mark.parametrize("mode", [mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING])
def test_sdma_engine_drains_fast_when_the_peer_never_runs(mode, check):
    """The SDMA engine enqueues a bounded wait per receive (hundreds per call).
    Once one of them times out, every later wait of the call returns at once,
    so the call ends in about one deadline, not one per remaining wait (an
    exited peer used to hold the stream, and the process exit, for minutes)."""
    import time
    P = Pairs("sdma", 1, 65536)
    try:
        t0 = time.monotonic()
        out, errs = P.run(mode, 4096, 600, timeout_ms=200, ranks=[0], check=check)
        took = time.monotonic() - t0
        assert 0 in errs and errs[0].status == mpx.ERR_TIMEOUT, errs
        assert took < 10, took     # 600 waits x 200 ms would be 120 s
    finally:
        P.close()


def test_check_mode_detects_missing_payload():
    """Tell the receiver to expect a different payload: every iteration fails."""
    P = Pairs("kernel", 1, 65536)
    try:
        out, errs = {}, {}
        exp1 = P.expect(1, 65536)

        def side(r, bad):
            try:
                out[r] = P.c.xfer(mpx.MODE_PINGPONG, P.group(r), r, P.peer(r), 4, P.bufs[r][0], P.bufs[r][1], 65536,
                                  check_payload=True, expect=(exp1[0] ^ 1) if bad else P.expect(r, 65536)[0],
                                  timeout_ms=5000)
            except mpx.MpxError as e:
                errs[r] = e

        th = [threading.Thread(target=side, args=(0, False)), threading.Thread(target=side, args=(1, True))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert 1 in errs and errs[1].status == mpx.ERR_CHECK
    finally:
        P.close()


def test_invalid_arguments(ctx):
    b = ctx.alloc(0, 64)
    try:
        with pytest.raises(mpx.MpxError) as e:
            ctx.attach(0, 0, b, b, 1 << 30)           # longer than the allocation
        assert e.value.status == mpx.ERR_INVALID
        with pytest.raises(mpx.MpxError):
            ctx.xfer(0, 1, 0, 1, 1, b, b, 8)          # rank 0 not attached
    finally:
        ctx.free(b)


@pytest.mark.parametrize("mode", [mpx.MODE_PINGPONG, mpx.MODE_UNIDIR])
def test_ll_full_landing_zone(monkeypatch, mode):
    """Cross-GPU links use LL up to 8 KiB (ll_max_bytes); loopback links switch
    at 2 KiB.  Force the cross-GPU threshold to cover the whole landing zone."""
    monkeypatch.setenv("MPX_LL_MAX", "8192")
    P = Pairs("kernel", 1, 8192 + 64)
    try:
        for n in (2049, 4095, 4096, 8191, 8192):
            out, errs = P.run(mode, n, 11)
            assert not errs, (n, errs)
            for r in (0, 1):
                assert out[r].check_failures == 0 and out[r].check_iters == 11
            assert out[0].protocol == PROTO_LL
    finally:
        P.close()


PROTO_LL = 0


@pytest.mark.parametrize("knobs", [
    {"WORKER_NOSTAGE": "1", "MPX_NB_PUBLISH": "1", "MPX_SDMA_GRAPH": "0", "MPX_SYNC": "event"},
    {"MPX_PUSH_STREAM": "1", "MPX_NB_PUBLISH": "256", "MPX_PUSH_WG": "7"},
    {"MPX_LL_MAX": "8192", "MPX_NB_PUBLISH": "2", "MPX_CHECK_RING_BYTES": "0"},   # one receive slot per link
])
def test_env_knob_variants(knobs):
    """The documented MPX_* knobs switch code paths that the
    defaults never take: each set runs every mode on both engines, every
    payload checked, in a process of its own (libmpx reads them once)."""
    import os
    import subprocess
    import sys
    env = dict(os.environ, **knobs)
    p = subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "knob_worker.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stderr[-1500:]


def test_link_info_between_visible_gpus():
    """mpx_link_info: every pair of visible GPUs reports its interconnect
    (xGMI, one hop, on an MI355X node); one GPU is not a link."""
    n = mpx.device_count()
    with pytest.raises(mpx.MpxError) as e:
        mpx.link_info(0, 0)
    assert e.value.status == mpx.ERR_INVALID
    with pytest.raises(mpx.MpxError):
        mpx.link_info(0, n)                       # not a visible device
    for b in range(1, n):
        li = mpx.link_info(0, b)
        assert li["type"] in mpx.LINK_TYPES.values() and li["hops"] >= 1


INT_MAX = (1 << 31) - 1    # the largest buff_len the reference's int accepts (mpi_perf.c:283, :464)


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_max_size_pairs_every_mode(engine):
    """B = 2^31 - 1 (golden `max_int_buffer`'s size) in every mode, seeded
    payloads, every payload checked: chunk offsets and buffer-resource sizes
    stay within 32 bits; nwg = 1 pushes one 2 GiB - 1 chunk."""
    P = Pairs(engine, 1, INT_MAX, fill="seeded")
    try:
        for mode in MODES:
            for nwg in ((0, 1) if engine == "kernel" else (0,)):
                out, errs = P.run(mode, INT_MAX, 2, timeout_ms=30000, nwg=nwg)
                assert not errs, (mode, nwg, errs)
                for r in (0, 1):
                    assert out[r].check_iters == 2 and out[r].check_failures == 0, (mode, nwg, r)
                    m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else INT_MAX
                    assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (mode, nwg, r)
    finally:
        P.close()


def test_copy_beyond_4gib(ctx):
    """A copy past 2^32 bytes (64-bit unit indices, > 2^20 workgroups) against
    the oracle's pattern checksum; nothing written past the end."""
    n = (4 << 30) + 13
    key = mpx.pattern_key(mpx.PATTERN_SEED, 9, 9, 9)
    src, dst = ctx.alloc(0, n), ctx.alloc(0, n + 64)
    try:
        ctx.fill(src, n, mpx.FILL_SPLITMIX, key)
        ctx.fill(dst, n + 64, mpx.FILL_BYTE, 0xEE)
        ctx.copy(0, dst, src, n, 1)
        assert ctx.checksum(dst, n) == ctx.checksum(src, n)
        assert ctx.read(dst, 64, offset=n) == b"\xee" * 64
        # the oracle's fill words over a window at the end (word k =
        # mix64((key ^ k) + G), oracle_fill): word indices above 2^29
        lo = n - 4096 - 13
        got = ctx.read(dst, n - lo, offset=lo)
        G = 0x9E3779B97F4A7C15
        want = bytearray()
        for k in range(lo // 8, (n + 7) // 8):
            want += (O.lib().oracle_mix64(((key ^ k) + G) & 0xFFFFFFFFFFFFFFFF)).to_bytes(8, "little")
        start = lo - (lo // 8) * 8
        assert got == bytes(want[start:start + (n - lo)])
    finally:
        ctx.free(src)
        ctx.free(dst)


# --------------------------------------------------------------------------
# a rank paired with itself (MPI self-send): the non-blocking loop as ONE
# launch / one stream — the form every engine, RCCL included, can run on a
# one-GPU box (RCCL refuses two ranks on one device)
# --------------------------------------------------------------------------
def _self_rank(engine, cap):
    c = mpx.Context(1, engine)
    tx, rx = c.alloc(0, cap), c.alloc(0, cap)
    c.fill(tx, cap, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, 7))
    c.fill(rx, cap, mpx.FILL_BYTE, 0)
    c.attach(0, 0, tx, rx, cap)
    if engine == "rccl":
        c.rccl_init_all()           # a one-rank communicator: send/recv to itself
    return c, tx, rx


SELF_KEY = mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, 7)   # _self_rank's tx pattern


@pytest.mark.parametrize("engine", ["kernel", "sdma", "rccl"])
def test_self_pair_nonblocking_every_payload(engine):
    """Isend + Irecv to itself for every window shape: every payload
    checksummed (check_iters == iters), the Waitall receives counted and
    digested on the device, rx = tx at the end; then the same unchecked.
    Every expected value comes from the oracle (oracle/mpx_oracle.c: the
    pattern's checksum, the reference's Waitall count), not from the device."""
    cap = 456131
    c, tx, rx = _self_rank(engine, cap)
    try:
        # mpx_xfer_prepare: SDMA graph chunks / the RCCL channel (a one-byte
        # exchange, once per pair; the second call is a no-op) — rx untouched
        rx0 = O.pattern_checksum(cap, mpx.FILL_BYTE, 0)
        assert c.checksum(rx, cap) == rx0
        for _ in range(2):
            c.prepare(mpx.MODE_NONBLOCKING, 0, 0, 0, 600, cap)
        assert c.checksum(rx, cap) == rx0
        for n in (0, 1, 4097, 65541, cap):
            want = O.pattern_checksum(n, mpx.FILL_SPLITMIX, SELF_KEY)
            for iters in (1, 255, 256, 257, 600):
                t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, iters, tx, rx, n, check_payload=True, expect=want,
                           timeout_ms=10000)
                k = O.lib().oracle_nb_waited(iters)
                assert t.check_iters == iters and t.check_failures == 0, (n, iters)
                assert t.recv_done == k and t.recv_digest == (k * want) & 0xFFFFFFFFFFFFFFFF, (n, iters)
                assert c.checksum(rx, n) == want
            t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, 600, tx, rx, n, timeout_ms=10000)
            assert t.recv_done == O.lib().oracle_nb_waited(600) and t.bytes == 2 * n * 600
        if engine == "rccl":
            assert t.protocol == 3
    finally:
        c.close()


def _self_golden_cases():
    """golden non-blocking runs of one pair (ppn 1) with the PMPI shim's
    receive accounting of both ranks"""
    return [c["name"] for c in O.golden()["cases"]
            if "-x" in c["args"] and "-u" not in c["args"] and c.get("shim") and not c.get("returncode")
            and c["ppn"] == 1]


@pytest.mark.parametrize("engine", ["kernel", "sdma", "rccl"])
@pytest.mark.parametrize("name", _self_golden_cases())
def test_self_pair_receive_digest_matches_reference(name, engine):
    """RCCL's receive accounting pinned to the compiled reference, on one GPU.
    In the golden run, rank 0 (group 1) receives group 0's 'a'-filled tx and
    rank 1 receives 'b' (mpi_perf.c:244-251).  A rank paired with itself
    whose tx holds that rank's payload receives the same bytes, so its
    device-counted receives, bytes and digest over the run's -r runs of -i
    iterations must equal that rank's PMPI shim numbers
    (tests/golden/ref_runs.json).  The RCCL engine can run no other pair on a
    one-GPU box (it refuses two ranks on one device); the kernel and SDMA
    engines run it too."""
    c = O.golden()["cases"][[x["name"] for x in O.golden()["cases"]].index(name)]
    a = c["args"]
    runs, iters = int(a[a.index("-r") + 1]), int(a[a.index("-i") + 1])
    B = int(a[a.index("-b") + 1])
    for rank, fill in ((0, "a"), (1, "b")):
        ctx = mpx.Context(1, engine)
        try:
            tx, rx = ctx.alloc(0, B), ctx.alloc(0, B)
            ctx.fill(tx, B, mpx.FILL_BYTE, ord(fill))
            ctx.attach(0, 0, tx, rx, B)
            if engine == "rccl":
                ctx.rccl_init_all()
            want = O.pattern_checksum(B, mpx.FILL_BYTE, ord(fill))
            done = nbytes = dig = 0
            for _ in range(runs):
                t = ctx.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, iters, tx, rx, B, check_payload=True, expect=want,
                             timeout_ms=10000)
                assert t.check_iters == iters and t.check_failures == 0
                done += t.recv_done
                nbytes += t.recv_done * B
                dig = (dig + t.recv_digest) & 0xFFFFFFFFFFFFFFFF
            ref = c["shim"][str(rank)]
            assert [done, nbytes, dig] == [ref["recv_done"], ref["recv_bytes"], ref["recv_digest"]], (rank, engine)
        finally:
            ctx.close()


@pytest.mark.parametrize("engine", ["kernel", "sdma", "rccl"])
def test_self_pair_lost_payload_fails(monkeypatch, engine):
    monkeypatch.setenv("MPX_TEST", "skip_push=3")
    c, tx, rx = _self_rank(engine, 65541)
    try:
        with pytest.raises(mpx.MpxError) as e:
            c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, 300, tx, rx, 65541, check_payload=True,
                   expect=O.pattern_checksum(65541, mpx.FILL_SPLITMIX, SELF_KEY), timeout_ms=10000)
        assert e.value.status == mpx.ERR_CHECK
    finally:
        c.close()


def test_self_pair_only_for_the_nonblocking_loop():
    c, tx, rx = _self_rank("kernel", 64)
    try:
        for m in (mpx.MODE_PINGPONG, mpx.MODE_UNIDIR):
            with pytest.raises(mpx.MpxError) as e:
                c.xfer(m, 1, 0, 0, 1, tx, rx, 8)
            assert e.value.status == mpx.ERR_INVALID
    finally:
        c.close()
