"""Pairs that span GPUs: every rank on a GPU of its own, bytes over xGMI.

These tests need as many GPUs as ranks and skip (with the reason) on a box
with fewer; the one-GPU box runs the same paths as loopback pairs
(tests/test_gpu_engine.py, test_gpu_host.py).  Their ids name the BASELINE
configuration each covers:

  cfg3  2 x MI355X, one pair over xGMI (scripts/run-1-pair.sh:24-28)
  cfg4  8 x MI355X, all 28 pairs in concurrent rounds, kernel vs SDMA vs RCCL
        (scripts/run-hbv3.sh:22-28 with every pair of the node)
  cfg5  8 x MI355X, RCCL all-pairs stress with checksum validation and
        kusto_ingest-ready records

Every payload is checksummed on the receiving device; receive accounting is
compared with the compiled reference's golden runs where one exists.

On a box with ONE GPU visible (the driver's `pytest -m gpu` box) this module
runs as its one-GPU rehearsal instead of skipping: a fixture sets
MPX_MULTI_REHEARSE=1 and MPX_LL_MAX=8192 (the cross-GPU LL threshold) for
each test (monkeypatch, not the whole run's environment; subprocess workers
inherit them), every rank on GPU 0 and N = MPX_MULTI_REHEARSE_N (default 4)
ranks where a test uses the whole node.  It proves the tests' own code, not
the links.  What only distinct GPUs have is skipped then, with the reason:
RCCL (it refuses two ranks on one GPU), the link table, and the "every pair
spans two GPUs" check.  With two or more GPUs visible the distinct-GPU form
runs; MPX_MULTI_REHEARSE=1 in the environment forces the rehearsal there too
(tools/gpu.sh multi_rehearse).
"""
import glob
import json
import os
import re
import socket
import subprocess
import sys

import pytest

import mpx
import oracle_py as O
from pairs import Pairs, cross_gpu_devs, rehearsing

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
GOLDEN = {c["name"]: c for c in O.golden()["cases"]}
MODES = {"pingpong": mpx.MODE_PINGPONG, "nonblocking": mpx.MODE_NONBLOCKING, "unidir": mpx.MODE_UNIDIR}
ENGINES = ["kernel", "sdma", "rccl"]
INT_MAX = (1 << 31) - 1


def ngpus() -> int:
    return mpx.device_count()


# What each BASELINE configuration reports on a multi-GPU node, and the
# north_star target it is held to (BASELINE.json): named in every skip reason,
# so a one-GPU run says what it did not measure.
CFG = {
    "cfg3": "BASELINE cfg3 (2 x MI355X, one pair over xGMI): per-pair unidir GB/s at 4 MiB, target >= 85 % of "
            "the link (130.6 GB/s of the stated 153.6 per direction, SURVEY.md:361; 65.3 of 76.8 beside it, the "
            "unsourced per-direction reading), and the 8 B half round trip, target < 3 us",
    "cfg4": "BASELINE cfg4 (8 x MI355X, all 28 pairs in concurrent rounds): every pair's payloads checked, "
            "aggregate GB/s per round reported (bench.py)",
    "cfg5": "BASELINE cfg5 (8 x MI355X, RCCL all-pairs stress): every payload checksummed, receive digests = "
            "the reference's, kusto_ingest-ready records",
}
# STATED: ~153 GB/s per link per direction as SURVEY.md:361 / BASELINE.md:51
# state the bar (the primary verdict); READING: 153.6 read as both directions
# summed, 76.8 each way (from memory, unsourced until a node run)
XGMI_STATED_PER_DIRECTION_GBPS, XGMI_PER_DIRECTION_READING_GBPS = 153.6, 76.8
TARGET_LINK_FRAC, TARGET_HALF_RTT_US = 0.85, 3.0


@pytest.fixture(autouse=True)
def one_gpu_rehearsal(monkeypatch):
    """One GPU visible: this test runs in its rehearsal form (every rank on
    GPU 0, the cross-GPU LL threshold), set for this test only."""
    if rehearsing() or ngpus() == 1:
        monkeypatch.setenv("MPX_MULTI_REHEARSE", "1")
        monkeypatch.setenv("MPX_LL_MAX", "8192")
        monkeypatch.setenv("MPX_MULTI_REHEARSE_N", os.environ.get("MPX_MULTI_REHEARSE_N", "4"))
    yield


def need(n: int, engine: str = "", distinct: bool = False, cfg: str = "cfg3"):
    if rehearsing():
        if engine == "rccl" or distinct:
            pytest.skip(f"needs distinct GPUs (one-GPU rehearsal); {CFG[cfg]}")
        assert os.environ.get("MPX_LL_MAX") == "8192", "rehearse with the cross-GPU LL threshold: MPX_LL_MAX=8192"
        return
    if ngpus() < n:
        pytest.skip(f"needs {n} GPUs, {ngpus()} visible; {CFG[cfg]}")


def report_target(record_property, name: str, value: float, unit: str, target: str, passed: bool) -> None:
    """A north_star number with its target beside it: in the junit properties
    and on stdout (pytest -s / -rP), whatever the verdict."""
    record_property(name, dict(value=value, unit=unit, target=target, meets_target=passed))
    print(f"[target] {name}: {value:.3f} {unit} (target {target}): {'MEETS' if passed else 'MISSES'}")


# 8191 / 8192: the cross-GPU LL protocol's largest messages; 8193: bulk
CFG3_SIZES = [0, 1, 8, 4097, 8191, 8192, 8193, 65541, 456131, 4 << 20]


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("engine", ENGINES + ["kernel-pull"])
def test_cfg3_cross_gpu_pair_every_payload(engine, mode):
    """GPU 0 (group 1) <-> GPU 1 (group 0), threads of one process: every
    size around the cross-GPU LL threshold and up to 4 MiB, every payload
    checksummed on the receiver (reads of bytes the peer wrote over xGMI, or
    in pull mode that the receiver loaded over xGMI), receives counted on the
    device, final rx = the peer's tx."""
    need(2, engine)
    pull = engine == "kernel-pull"
    P = Pairs("kernel" if pull else engine, 1, 4 << 20, fill="seeded", devs=cross_gpu_devs(2))
    m = MODES[mode]
    try:
        for n in CFG3_SIZES:
            iters = 300 if m == mpx.MODE_NONBLOCKING else 9
            out, errs = P.run(m, n, iters, pull=pull)
            assert not errs, (n, errs)
            for r in (0, 1):
                t = out[r]
                assert t.check_iters == iters and t.check_failures == 0, (n, r)
                assert t.recv_done == (iters - iters // 256 if m == mpx.MODE_NONBLOCKING else iters), (n, r)
                k = 1 if (m == mpx.MODE_UNIDIR and r == 0) else n
                assert P.c.checksum(P.bufs[r][1], k) == P.c.checksum(P.bufs[P.peer(r)][0], k), (n, r)
                if engine.startswith("kernel"):   # LL up to 8 KiB across GPUs (ll_max_bytes), bulk above
                    assert t.protocol == (0 if m != mpx.MODE_NONBLOCKING and n <= 8192 else 7 if pull else 1), (n, r)
    finally:
        P.close()


@pytest.mark.parametrize("engine", ENGINES)
def test_cfg3_cross_gpu_max_int_buffer(engine):
    """B = 2^31 - 1 (the reference's largest int buffer) across GPUs, every
    mode, every payload checked."""
    need(2, engine)
    P = Pairs(engine, 1, INT_MAX, fill="seeded", devs=cross_gpu_devs(2))
    try:
        for m in MODES.values():
            out, errs = P.run(m, INT_MAX, 2, timeout_ms=30000)
            assert not errs, (m, errs)
            for r in (0, 1):
                assert out[r].check_iters == 2 and out[r].check_failures == 0, (m, r)
    finally:
        P.close()


def _golden_cross_cases():
    out = []
    for c in O.golden()["cases"]:
        a = c["args"]
        if c.get("returncode") or not c.get("shim") or "-d" in a or c["np"] != 2 * c["ppn"]:
            continue
        if a[a.index("-n") + 1] != "1" or not re.match(r"(pingpong|nonblocking|unidir)_p\d_b\d+_i\d+$|"
                                                       r"nonblocking_window_", c["name"]):
            continue
        out.append(c["name"])
    return out


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
@pytest.mark.parametrize("name", _golden_cross_cases())
def test_cfg3_receive_digest_matches_reference_across_gpus(name, engine):
    """The golden run's pairs with every rank on its own GPU (2 x ppn GPUs):
    device-counted receives, bytes and checksum digest per rank equal the
    compiled reference's (PMPI shim) numbers."""
    _receive_digest_across_gpus(name, engine, "cfg3")


@pytest.mark.parametrize("name", _golden_cross_cases())
def test_cfg5_rccl_receive_digest_matches_reference_across_gpus(name):
    """BASELINE config 5's receive check: the RCCL engine's device-counted
    receives, bytes and digest per rank, each rank on its own GPU, equal the
    compiled reference's ranks' (PMPI shim, tests/golden/ref_runs.json) in
    every loop, ppn 1-4, and the non-blocking window cases — the independent
    check of RCCL's receive accounting that one GPU cannot run (RCCL refuses
    two ranks on one device; tests/test_gpu_engine.py pins its self-pair
    form to the same golden digests)."""
    _receive_digest_across_gpus(name, "rccl", "cfg5")


def _receive_digest_across_gpus(name, engine, cfg):
    c = GOLDEN[name]
    ppn = c["ppn"]
    need(2 * ppn, engine, cfg=cfg)
    a = c["args"]
    runs = int(a[a.index("-r") + 1])
    iters = int(a[a.index("-i") + 1]) if "-i" in a else 10
    B = int(a[a.index("-b") + 1]) if "-b" in a else 456131
    m = mpx.MODE_UNIDIR if "-u" in a else (mpx.MODE_NONBLOCKING if "-x" in a else mpx.MODE_PINGPONG)
    P = Pairs(engine, ppn, B, devs=cross_gpu_devs(2 * ppn))
    try:
        digest = {r: [0, 0, 0] for r in range(2 * ppn)}
        for _ in range(runs):
            out, errs = P.run(m, B, iters)
            assert not errs, errs
            for r in range(2 * ppn):
                k = 1 if (m == mpx.MODE_UNIDIR and P.group(r) == 1) else B
                digest[r][0] += out[r].recv_done
                digest[r][1] += out[r].recv_done * k
                digest[r][2] = (digest[r][2] + out[r].recv_digest) & 0xFFFFFFFFFFFFFFFF
        for r in range(2 * ppn):
            ref = c["shim"][str(r)]
            assert digest[r] == [ref["recv_done"], ref["recv_bytes"], ref["recv_digest"]], r
    finally:
        P.close()


@pytest.mark.parametrize("engine", ["kernel", "sdma", "kernel-pull"])
def test_cfg3_cross_gpu_two_processes_ipc(tmp_path, engine):
    """Two processes, rank r on GPU r, each mapping the other's rx, ring and
    mailbox through IPC (bench.py's one-process-per-GPU path)."""
    need(2, engine)
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "ipc_worker.py"), str(tmp_path), str(r), engine,
                               "cross"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in (0, 1)]
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=100)[0])
        except subprocess.TimeoutExpired:
            p.kill()
            outs.append(p.communicate()[0])
    assert all(p.returncode == 0 for p in procs), outs
    for r in (0, 1):
        for x in json.load(open(tmp_path / f"result_{r}.json")):
            assert x["final_rx_ok"], (r, x)
            assert x["check_failures"] == 0 and x["check_iters"] == x["iters"], (r, x)


@pytest.mark.parametrize("mode", ["pingpong", "unidir", "nonblocking"])
@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_cfg3_rx_read_between_calls_across_gpus(engine, mode):
    """Matched-receive order across xGMI (tests/test_gpu_ordering.py's race
    scenario with rank r on GPU r): rank 1 reads rx on the host between two
    calls while rank 0 races into the second with a new payload; rx must
    still hold call 1's last payload, and call 2's afterwards."""
    need(2, engine)
    import ordering as OR
    import test_gpu_ordering as T
    m = {"pingpong": mpx.MODE_PINGPONG, "unidir": mpx.MODE_UNIDIR, "nonblocking": mpx.MODE_NONBLOCKING}[mode]
    for n in (262144 + 13, 1024):
        it = 300 if m == mpx.MODE_NONBLOCKING else 20
        out = T.run_threads(lambda c, r, tx, rx, s: OR.race(c, r, tx, rx, s, m, True, n, it), engine,
                            devs=cross_gpu_devs(2))
        T.assert_race_ok(out)


def test_cfg3_lagging_workgroup_layout_change_across_gpus(tmp_path):
    """The non-blocking check-mode regression (GPUTEST_r02) across xGMI, two
    processes, rank r on GPU r: one receiver workgroup late to check call
    1's last receive, call 2 with another length and push width."""
    need(2)
    import ordering as OR
    import test_gpu_ordering as T
    T.assert_lag_ok(T.run_processes(tmp_path, "kernel", ["lag"], OR.lag_env(), cross=True))


def test_cfg3_pull_lagging_receiver_keeps_the_senders_tx_across_gpus(tmp_path):
    """Pull mode's buffer-reuse order across xGMI, two processes: a receiver
    workgroup late to load call 1's last payload from the other GPU's tx;
    the sender's call must not return (and rewrite tx) before that load."""
    need(2)
    import ordering as OR
    import test_gpu_ordering as T
    T.assert_lag_ok(T.run_processes(tmp_path, "kernel-pull", ["lag"], OR.lag_env(), cross=True))


def test_cfg3_8B_half_rtt_reported_against_3us_target(record_property):
    """Ping-pong 8 B across GPUs (SURVEY §8d cfg3, 10^5 iterations): the half
    round trip, reported beside north_star's target (< 3 us device-initiated)
    with its verdict.  The test fails only on a broken measurement (> 50 us);
    the target's verdict is the reported field, and bench.py's
    extras.targets carries the same check for the driver's line."""
    need(2)
    P = Pairs("kernel", 1, 64, fill="seeded", devs=cross_gpu_devs(2))
    try:
        out, errs = P.run(mpx.MODE_PINGPONG, 8, 100000, check=False)
        assert not errs, errs
        half_rtt_us = max(out[0].device_s, out[1].device_s) / (2 * 100000) * 1e6
        report_target(record_property, "cfg3_8B_half_rtt_us", half_rtt_us, "us", f"< {TARGET_HALF_RTT_US}",
                      half_rtt_us < TARGET_HALF_RTT_US)
        assert 0 < half_rtt_us < 50
    finally:
        P.close()


def test_cfg3_unidir_4MiB_reported_against_85pct_link_target(record_property):
    """One pair, unidir 4 MiB x 500 (the bench's headline shape, G1 -> G0
    over one link): per-pair GB/s from the G1 launch's device time, reported
    beside north_star's >= 85 % of link peak.  The primary verdict is against
    the stated bar (153.6 GB/s per link per direction, SURVEY.md:361); the
    per-direction reading (76.8 GB/s each way, DESIGN.md §7, unsourced) is
    reported beside it.  Fails only on a broken measurement (< 1 GB/s)."""
    need(2)
    n, iters = 4 << 20, 500
    P = Pairs("kernel", 1, n, fill="seeded", devs=cross_gpu_devs(2))
    try:
        out, errs = P.run(mpx.MODE_UNIDIR, n, 3)                 # every payload checked first
        assert not errs, errs
        out, errs = P.run(mpx.MODE_UNIDIR, n, iters, check=False)
        assert not errs, errs
        gbps = n * iters / out[0].device_s / 1e9
        report_link_targets(record_property, "cfg3_unidir_4MiB", gbps)
        assert gbps > 1
        # the same loop pulled (MPX_XFER_PULL: G0 loads G1's tx over the
        # link), every payload checked first; reported beside the push
        out, errs = P.run(mpx.MODE_UNIDIR, n, 3, pull=True)
        assert not errs, errs
        out, errs = P.run(mpx.MODE_UNIDIR, n, iters, check=False, pull=True)
        assert not errs, errs
        pull_gbps = n * iters / out[0].device_s / 1e9
        report_link_targets(record_property, "cfg3_pull_unidir_4MiB", pull_gbps)
        assert pull_gbps > 1
    finally:
        P.close()


def report_link_targets(record_property, name: str, gbps: float) -> None:
    """The primary verdict against the stated bar, the reading beside it."""
    report_target(record_property, f"{name}_GBps", gbps, "GB/s",
                  f">= {TARGET_LINK_FRAC} x {XGMI_STATED_PER_DIRECTION_GBPS} per direction (SURVEY.md:361)",
                  gbps >= TARGET_LINK_FRAC * XGMI_STATED_PER_DIRECTION_GBPS)
    report_target(record_property, f"{name}_GBps_per_direction_reading", gbps, "GB/s",
                  f">= {TARGET_LINK_FRAC} x {XGMI_PER_DIRECTION_READING_GBPS} (unsourced per-direction reading, "
                  f"DESIGN.md §7)", gbps >= TARGET_LINK_FRAC * XGMI_PER_DIRECTION_READING_GBPS)


# ---- mpx_perf on every GPU of the node -------------------------------------
def _perf(tmp_path, args, env_extra=None, timeout=300):
    g1 = tmp_path / "group1"
    logs = tmp_path / "logs"
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(logs)) for a in args]
    env = dict(os.environ, MPX_HOSTNAME="localhost", **(env_extra or {}))
    return subprocess.run([PERF, "-t", "10000"] + argv, capture_output=True, text=True, env=env, timeout=timeout)


def _files(tmp_path):
    recs, side = [], []
    for f in sorted(glob.glob(str(tmp_path / "logs" / "tcp-*.log"))):
        recs += [line.rstrip("\n").split(",") for line in open(f)]
    for f in sorted(glob.glob(str(tmp_path / "logs" / "gpu-*.csv"))):
        side += [line.rstrip("\n").split(",") for line in open(f)][1:]
    return recs, side


def _world():
    if rehearsing():
        return int(os.environ.get("MPX_MULTI_REHEARSE_N", "4"))
    n = ngpus()
    return n - (n & 1)


@pytest.mark.parametrize("engine", ENGINES)
def test_cfg4_all_pairs_rounds_every_gpu(tmp_path, engine):
    """mpx_perf -w N -a 1 on every GPU (N = 8 on an MI355X node: 7 rounds x
    4 concurrent pairs = all 28 pairs), unidir 456131 B x 10 (run-hbv3's
    shape), seeded payloads, every payload checked, records for runs 1..N-1
    covering every pair once."""
    need(2, engine, cfg="cfg4")
    N = _world()
    (tmp_path / "group1").write_text("vm\n")
    names = ",".join(["vm"] * (N // 2) + ["runsc"] * (N // 2))
    p = _perf(tmp_path, ["-w", str(N), "-a", "1", "-e", engine, "-f", "@G1", "-n", "1", "-p", str(N // 2), "-u", "1",
                         "-r", str(N), "-i", "10", "-b", "456131", "-c", "2", "-l", "@LOGS"],
              {"MPX_PROCESSOR_NAMES": names})
    assert p.returncode == 0, p.stderr[-800:]
    recs, side = _files(tmp_path)
    from mpx.schedule import all_pairs_rounds
    assert {(int(f[2]), int(f[6])) for f in side} == {q for rnd in all_pairs_rounds(N) for q in rnd}
    assert len(recs) == (N - 1) * (N // 2)
    assert all(int(f[16]) == 0 and int(f[15]) == 10 and int(f[18]) == 10 for f in side)
    if not rehearsing():
        assert all(f[5] != f[7] for f in side)             # every pair spans two GPUs


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_cfg4_all_28_pairs_shape_rehearsed(tmp_path, monkeypatch, engine):
    """The node's own shape in the one-GPU rehearsal: N = 8 ranks, 7 rounds
    x 4 concurrent pairs = all 28 pairs (the rehearsal's default N is 4),
    every payload checked; on a multi-GPU node the test above already runs
    the whole node."""
    if not rehearsing():
        pytest.skip("multi-GPU node: test_cfg4_all_pairs_rounds_every_gpu runs the node's N")
    monkeypatch.setenv("MPX_MULTI_REHEARSE_N", "8")
    test_cfg4_all_pairs_rounds_every_gpu(tmp_path, engine)


def test_cfg5_rccl_all_pairs_stress_processes(tmp_path):
    """BASELINE config 5: one mpx_perf process per GPU (the reference's
    process model), RCCL engine, all-pairs rounds twice over, seeded payloads
    checked, and the records are what kusto_ingest.py would upload."""
    need(2, "rccl", cfg="cfg5")
    N = _world()
    (tmp_path / "group1").write_text("vm\n")
    names = ",".join(["vm"] * (N // 2) + ["runsc"] * (N // 2))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = []
    logs = tmp_path / "logs"
    for r in range(N):
        env = dict(os.environ, MPX_RANK=str(r), MPX_SIZE=str(N), MPX_LOCAL_RANK=str(r), MPX_PROCESSOR_NAMES=names,
                   MPX_BOOTSTRAP=f"127.0.0.1:{port}", MPX_BOOTSTRAP_TIMEOUT="120", MPX_HOSTNAME="localhost")
        ps.append(subprocess.Popen([PERF, "-t", "10000", "-e", "rccl", "-a", "1", "-f", str(tmp_path / "group1"), "-n",
                                    "1", "-p", str(N // 2), "-u", "1", "-r", str(2 * (N - 1) + 1), "-i", "20", "-b",
                                    "456131", "-c", "2", "-l", str(logs)], stdout=subprocess.PIPE,
                                   stderr=subprocess.PIPE, text=True, env=env))
    errs = [p.communicate(timeout=300)[1] for p in ps]
    assert [p.returncode for p in ps] == [0] * N, "".join(errs)[-1500:]
    recs, side = _files(tmp_path)
    from mpx.schedule import all_pairs_rounds
    assert {(int(f[2]), int(f[6])) for f in side} == {q for rnd in all_pairs_rounds(N) for q in rnd}
    assert all(f[3] == "rccl" and int(f[16]) == 0 and int(f[15]) == 20 for f in side)
    import kusto_rule as K
    for f in glob.glob(str(logs / "tcp-*.log")):
        for line in open(f):
            row = K.parse_row(line)
            assert row["BufferSize"] == 456131 and row["NumOfBuffers"] == 20 and row["NumOfFlows"] == N // 2


def test_link_types_between_all_gpus():
    """Every pair of visible GPUs is one xGMI hop apart (full mesh)."""
    need(2, distinct=True, cfg="cfg4")
    for a in range(ngpus()):
        for b in range(ngpus()):
            if a != b:
                li = mpx.link_info(a, b)
                assert li["type"] == "xgmi" and li["hops"] == 1, (a, b, li)


def test_concurrent_pairs_on_disjoint_links():
    """N/2 pairs at once, one per pair of GPUs (a round of cfg4), every
    payload checked in all three modes."""
    need(4, cfg="cfg4")
    N = _world()
    P = Pairs("kernel", N // 2, 4 << 20, fill="seeded", devs=cross_gpu_devs(N))
    try:
        for m in MODES.values():
            out, errs = P.run(m, 4 << 20, 20 if m != mpx.MODE_NONBLOCKING else 300)
            assert not errs, (m, errs)
            assert all(out[r].check_failures == 0 for r in out)
    finally:
        P.close()

