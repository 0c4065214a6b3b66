"""Pull mode (MPX_XFER_PULL) of the kernel and SDMA engines: parity on the GPU.

The reference's three loops (/root/reference/mpi_perf.c:66-145) with every
B-byte payload loaded by its RECEIVER from the sender's peer-mapped tx
(k_xfer_pull; the SDMA engine: a copy on the receiver's stream) instead of
stored by the sender into the receiver's rx — the
"try pull as well" of SURVEY.md §7 step 4.  What a caller sees must not
change: the same bytes land (every payload checksummed against the oracle's
pattern checksum or the peer's tx), the same receives are counted and
digested (the compiled reference's per-rank PMPI digests, tests/golden), and
rx ends holding the last payload.  Pairs run as loopback ranks on GPU 0
(tests/pairs.py); the cross-GPU form is in tests/test_gpu_multi.py.
"""
import threading

import pytest

import mpx
import oracle_py as O
from pairs import Pairs

pytestmark = pytest.mark.gpu

MODES = [mpx.MODE_PINGPONG, mpx.MODE_NONBLOCKING, mpx.MODE_UNIDIR]
PAIR_SIZES = [0, 1, 8, 2048, 2049, 4097, 8193, 65541, 456131, 4 << 20]
PROTO_LL, PROTO_PULL, PROTO_SDMA_PULL = 0, 7, 8
LL_MAX_ONE_GPU = 2048      # ll_max_bytes(same_device): LL messages stay pushes
GOLDEN = {c["name"]: c for c in O.golden()["cases"]}


def _proto(engine, mode, n):
    """the protocol a pulled call reports: the SDMA engine pulls every size,
    the kernel engine's LL messages stay pushes"""
    if engine == "sdma":
        return PROTO_SDMA_PULL
    return PROTO_PULL if (mode == mpx.MODE_NONBLOCKING or n > LL_MAX_ONE_GPU) else PROTO_LL


ENGINES = ["kernel", "sdma"]


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("mode", MODES)
def test_pull_pair_every_payload(mode, engine):
    """Every size class (0 B, LL sizes that stay pushes, ragged bulk sizes,
    4 MiB), every payload checksummed, the reference's receive count, the
    algorithmic bytes, the protocol, and the final rx = the peer's tx."""
    P = Pairs(engine, 1, 4 << 20)
    try:
        for n in PAIR_SIZES:
            iters = 300 if (mode == mpx.MODE_NONBLOCKING and n <= 65541) else 7
            out, errs = P.run(mode, n, iters, pull=True)
            assert not errs, (n, errs)
            for r in (0, 1):
                t = out[r]
                assert t.check_iters == iters and t.check_failures == 0, (n, r)
                assert t.recv_done == (O.lib().oracle_nb_waited(iters) if mode == mpx.MODE_NONBLOCKING else iters)
                assert t.bytes == n * iters * (1 if mode == mpx.MODE_UNIDIR else 2)
                assert t.protocol == _proto(engine, mode, n), (n, r, t.protocol)
            for r in (0, 1):
                m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (n, r)
    finally:
        P.close()


# (workgroups, B): chunk = ceil(B / nwg) rounded up to 16 B, pulled 8 units
# per lane at a time; ragged tails; a width wider than B / 1 KiB is narrowed
PULL_CASES = [(1, 40000), (1, 70001), (7, 456131), (8, 456131), (33, (1 << 20) + 17), (128, (4 << 20) + 3),
              (256, (20 << 20) + 5), (64, 20000), (256, 3000)]


@pytest.mark.parametrize("mode", MODES)
def test_pull_widths(mode):
    P = Pairs("kernel", 1, (20 << 20) + 5, fill="pattern")
    try:
        for nwg, n in PULL_CASES:
            out, errs = P.run(mode, n, 5, nwg=nwg, pull=True)
            assert not errs, (nwg, n, errs)
            for r in (0, 1):
                assert out[r].nwg == min(nwg, -(-n // 1024)) and out[r].protocol == PROTO_PULL, (nwg, n, r)
                assert out[r].check_failures == 0 and out[r].check_iters == 5
                m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (nwg, n, r)
    finally:
        P.close()


def _digest_cases():
    """the golden runs of tests/test_gpu_engine.py's digest test"""
    out = []
    for c in O.golden()["cases"]:
        a = c["args"]
        if c.get("returncode") or not c.get("shim") or "-d" in a or c["np"] != 2 * c["ppn"]:
            continue
        if a[a.index("-n") + 1] != "1":
            continue
        out.append(c["name"])
    return out


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("name", _digest_cases())
def test_pull_receive_digest_matches_reference(name, engine):
    """The golden case's pairs, mode, B, iters and runs in pull mode: each
    rank's device-counted receives, bytes and digest equal the compiled
    reference's ranks' (PMPI shim)."""
    c = GOLDEN[name]
    a = c["args"]
    ppn = c["ppn"]
    runs = int(a[a.index("-r") + 1])
    iters = int(a[a.index("-i") + 1]) if "-i" in a else 10
    B = int(a[a.index("-b") + 1]) if "-b" in a else 456131
    mode = mpx.MODE_UNIDIR if "-u" in a else (mpx.MODE_NONBLOCKING if "-x" in a else mpx.MODE_PINGPONG)
    P = Pairs(engine, ppn, B)
    try:
        digest = {r: [0, 0, 0] for r in range(2 * ppn)}
        for _ in range(runs):
            out, errs = P.run(mode, B, iters, pull=True)
            assert not errs, errs
            for r in range(2 * ppn):
                m = 1 if (mode == mpx.MODE_UNIDIR and P.group(r) == 1) else B
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


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("n", [0, 1, 4097, 65541, 456131])
def test_pull_nonblocking_every_payload_seeded(n, engine):
    """-x 1 pulled, every window shape: every receive checksummed on the
    device; the Waitall receives (iters - iters // 256, mpi_perf.c:108-111)
    counted and digested; rx ends holding the last payload."""
    P = Pairs(engine, 1, max(n, 1), fill="seeded")
    try:
        for iters in NB_ITERS:
            out, errs = P.run(mpx.MODE_NONBLOCKING, n, iters, pull=True)
            assert not errs, (iters, errs)
            for r in (0, 1):
                t = out[r]
                assert t.check_iters == iters and t.check_failures == 0, (iters, r)
                k = O.lib().oracle_nb_waited(iters)
                one = P.expect(r, n)[0]
                assert t.recv_done == k and t.recv_digest == (k * one) & 0xFFFFFFFFFFFFFFFF, (iters, r)
                assert P.c.checksum(P.bufs[r][1], n) == one
            # unchecked: the count only
            out, errs = P.run(mpx.MODE_NONBLOCKING, n, iters, check=False, pull=True)
            assert not errs and all(out[r].recv_done == O.lib().oracle_nb_waited(iters) for r in (0, 1))
    finally:
        P.close()


@pytest.mark.parametrize("engine", ENGINES)
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("skip", [1, 7, 256])
def test_pull_lost_payload_fails_the_check(monkeypatch, mode, skip, engine):
    """MPX_TEST=skip_push=k in pull mode: the k-th receive of each call loads
    nothing (its ready word and credit still go), so check mode must report
    the receive whose bytes never came."""
    monkeypatch.setenv("MPX_TEST", f"skip_push={skip}")
    P = Pairs(engine, 1, 65541, fill="seeded")
    try:
        out, errs = P.run(mode, 65541, 300, pull=True)
        for r in (0, 1):
            if not (mode == mpx.MODE_UNIDIR and r == 0):   # G1 receives 1-byte acks (LL pushes)
                assert r in errs and errs[r].status == mpx.ERR_CHECK, (r, errs, out.get(r))
    finally:
        P.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_push_and_pull_calls_share_a_link(engine):
    """One link alternating push and pull calls, across protocols, sizes and
    widths: the sequence numbers, credits and the receive-posted word stay
    consistent, every payload checked.  (Unchecked calls too: the SDMA
    engine replays graph-captured chunks of 256 iterations there.)"""
    P = Pairs(engine, 1, 1 << 20, fill="pattern")
    try:
        plan = [(0, 100000, 3, 0), (1, 1000, 600, 0), (2, 300000, 4, 5), (0, 8, 5, 0), (1, 1 << 20, 3, 64),
                (2, 4096, 9, 0), (0, 65541, 7, 3), (1, 0, 300, 0), (2, 1, 5, 0), (1, 4097, 257, 2)]
        for k, (mode, n, it, nwg) in enumerate(plan):
            for pull in (k % 2 == 0, k % 2 == 1):
                out, errs = P.run(mode, n, it, nwg=nwg, pull=pull)
                assert not errs, (mode, n, pull, errs)
                assert all(out[r].check_failures == 0 and out[r].check_iters == it for r in (0, 1))
                out, errs = P.run(mode, n, it, nwg=nwg, pull=pull, check=False)
                assert not errs, (mode, n, pull, "unchecked", errs)
                for r in (0, 1):
                    m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                    assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (mode, n, pull, r)
    finally:
        P.close()


def test_pull_concurrent_pairs():
    """four loopback pairs at once (eight persistent kernels on one GPU)"""
    P = Pairs("kernel", 4, 456131, fill="pattern")
    try:
        for mode in MODES:
            out, errs = P.run(mode, 456131, 5, pull=True)
            assert not errs, errs
            assert all(out[r].protocol == PROTO_PULL for r in range(8))
    finally:
        P.close()


def test_pull_max_size_pairs_every_mode():
    """B = 2^31 - 1 pulled in every mode, one workgroup (one 2 GiB - 1 chunk:
    offsets and resource sizes within 32 bits) and the default width."""
    n = (1 << 31) - 1
    P = Pairs("kernel", 1, n, fill="seeded")
    try:
        for mode in MODES:
            for nwg in (0, 1):
                out, errs = P.run(mode, n, 2, timeout_ms=30000, nwg=nwg, pull=True)
                assert not errs, (mode, nwg, errs)
                for r in (0, 1):
                    assert out[r].check_iters == 2 and out[r].check_failures == 0, (mode, nwg, r)
                    m = 1 if (mode == mpx.MODE_UNIDIR and r == 0) else n
                    assert P.c.checksum(P.bufs[r][1], m) == P.c.checksum(P.bufs[P.peer(r)][0], m), (mode, nwg, r)
    finally:
        P.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_pull_self_pair_nonblocking(engine):
    """A rank paired with itself (Isend + Irecv to itself) in pull mode: it
    loads its own tx; the oracle's pattern checksum and Waitall count."""
    cap = 456131
    key = mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, 7)
    c = mpx.Context(1, engine)
    try:
        tx, rx = c.alloc(0, cap), c.alloc(0, cap)
        c.fill(tx, cap, mpx.FILL_SPLITMIX, key)
        c.fill(rx, cap, mpx.FILL_BYTE, 0)
        c.attach(0, 0, tx, rx, cap)
        for n in (0, 1, 4097, cap):
            want = O.pattern_checksum(n, mpx.FILL_SPLITMIX, key)
            for iters in (1, 256, 600):
                t = c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, iters, tx, rx, n, check_payload=True, expect=want,
                           timeout_ms=10000, pull=True)
                k = O.lib().oracle_nb_waited(iters)
                assert t.protocol == _proto(engine, 1, n) and t.check_iters == iters and t.check_failures == 0
                assert t.recv_done == k and t.recv_digest == (k * want) & 0xFFFFFFFFFFFFFFFF, (n, iters)
                assert c.checksum(rx, n) == want
    finally:
        c.close()


def test_pull_refused_by_the_rccl_engine():
    """MPX_XFER_PULL is a kernel / SDMA engine mode: RCCL (a rank paired with
    itself, the form one GPU runs) refuses it."""
    c = mpx.Context(1, "rccl")
    try:
        tx, rx = c.alloc(0, 4096), c.alloc(0, 4096)
        c.attach(0, 0, tx, rx, 4096)
        c.rccl_init_all()
        with pytest.raises(mpx.MpxError) as e:
            c.xfer(mpx.MODE_NONBLOCKING, 0, 0, 0, 1, tx, rx, 4096, pull=True)
        assert e.value.status == mpx.ERR_UNSUPPORTED
    finally:
        c.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_pull_timeout_when_peer_never_runs(engine):
    """A receiver whose peer never publishes gives up at its deadline, like a
    push receiver; so does a sender whose peer never loads."""
    P = Pairs(engine, 1, 65536)
    try:
        out, errs = P.run(mpx.MODE_PINGPONG, 65536, 3, timeout_ms=300, ranks=[1], pull=True)   # G0 waits
        assert errs[1].status == mpx.ERR_TIMEOUT, errs
    finally:
        P.close()
    P = Pairs(engine, 1, 65536)
    try:
        out, errs = P.run(mpx.MODE_UNIDIR, 65536, 3, timeout_ms=300, ranks=[0], pull=True)     # G1 waits
        assert errs[0].status == mpx.ERR_TIMEOUT, errs
    finally:
        P.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_pull_check_detects_a_wrong_expectation(engine):
    """Tell one receiver to expect another payload: every iteration fails."""
    P = Pairs(engine, 1, 65536)
    try:
        out, errs = {}, {}

        def side(r, bad):
            try:
                exp = P.expect(r, 65536)[0]
                out[r] = P.c.xfer(mpx.MODE_PINGPONG, P.group(r), r, P.peer(r), 4, P.bufs[r][0], P.bufs[r][1], 65536,
                                  check_payload=True, expect=exp ^ 1 if bad else exp, timeout_ms=5000, pull=True)
            except mpx.MpxError as e:
                errs[r] = e

        th = [threading.Thread(target=side, args=(0, False)), threading.Thread(target=side, args=(1, True))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert 1 in errs and errs[1].status == mpx.ERR_CHECK and "4 of 4" in str(errs[1]), errs
        assert 0 not in errs, errs
    finally:
        P.close()
