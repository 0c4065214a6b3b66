"""Host logic of mpx_perf (mpi-perf_amd/host, pure C) against the reference's
golden runs: group/peer rule, all-pairs schedule, record / INFO / summary /
bandwidth formats, log names, and the CLI's error exits.  CPU-only: the error
paths all end before any GPU call.
"""
import ctypes as C
import itertools
import os
import re
import signal
import subprocess

import pytest

import oracle_py as O
from mpx.schedule import all_pairs_rounds, pairing_from_groups

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "mpi-perf_amd", "lib", "libmpx_host.so")
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
G = O.golden()
CASES = {c["name"]: c for c in G["cases"]}


@pytest.fixture(scope="module")
def H():
    L = C.CDLL(HOSTLIB)
    L.mpxh_in_group1.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.mpxh_pairing.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 4
    L.mpxh_round_pairs.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int)]
    L.mpxh_round_role.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.mpxh_format_record.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_int,
                                     C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_double, C.c_longlong]
    L.mpxh_format_info.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                   C.c_int, C.c_char_p, C.c_char_p, C.c_char_p]
    L.mpxh_format_summary.argtypes = [C.c_char_p, C.c_size_t, C.c_longlong, C.c_double, C.c_double, C.c_double,
                                      C.c_double, C.c_int]
    L.mpxh_format_bandwidth.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_longlong, C.c_int, C.c_int, C.c_int,
                                        C.c_double]
    L.mpxh_log_name.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_char_p, C.c_int, C.c_char_p]
    L.mpxh_processor_name.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.c_int, C.c_char_p]
    L.mpxh_uuid.argtypes = [C.c_char_p]
    L.mpxh_format_dotnet.argtypes = [C.c_char_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_char_p, C.c_char_p,
                                     C.c_int, C.c_int, C.c_int]
    return L


def lines_blob(lines):
    return b"".join((ln + "\n").encode().ljust(128, b"\0")[:128] for ln in lines)


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if len(c["info"]) == c["np"] and c["info"]])
def test_group_and_pairing_match_reference(H, name):
    c = CASES[name]
    blob = lines_blob(c["group1_lines"])
    groups = [H.mpxh_in_group1(d["name"].encode(), blob, len(c["group1_lines"])) for d in c["info"]]
    assert groups == [d["group"] for d in c["info"]]
    n = len(groups)
    g = (C.c_int * n)(*groups)
    gr, gs, pe = (C.c_int * n)(), (C.c_int * n)(), (C.c_int * n)()
    H.mpxh_pairing(n, g, gr, gs, pe)
    assert list(gr) == [d["group_rank"] for d in c["info"]]
    assert list(gs) == [d["group_size"] for d in c["info"]]
    assert list(pe) == [d["peer"] for d in c["info"]]
    assert pairing_from_groups(groups) == (list(gr), list(pe))


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if len(c["info"]) == c["np"] and c["info"]][:12])
def test_info_line_format(H, name):
    c = CASES[name]
    for d in c["info"]:
        out = C.create_string_buffer(1024)
        H.mpxh_format_info(out, 1024, d["name"].encode(), d["rank"], d["world"], d["group"], d["group_size"],
                           d["group_rank"], d["peer"], d["ip"].encode(), d["peer_host"].encode(),
                           d["peer_ip"].encode())
        line = out.value.decode()
        m = re.match(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d+), group_size: (\d+), "
                     r"group_rank: (\d+), my_peer: (-?\d+), hostname: (\S+) \((\S*)\), peer_host: (\S+) \((\S*)\)",
                     line)
        assert m and m[1] == d["name"] and int(m[7]) == d["peer"] and m[10] == d["peer_host"]


@pytest.mark.parametrize("n", [2, 4, 6, 8, 16])
def test_all_pairs_rounds_cover_every_pair_once(H, n):
    seen = set()
    for r in range(n - 1):
        pairs = (C.c_int * n)()
        assert H.mpxh_round_pairs(n, r, pairs) == n // 2
        ps = [(pairs[2 * k], pairs[2 * k + 1]) for k in range(n // 2)]
        assert sorted(itertools.chain(*ps)) == list(range(n))       # a perfect matching
        assert ps == all_pairs_rounds(n)[r]                          # Python mirror agrees
        for a, b in ps:
            key = (min(a, b), max(a, b))
            assert key not in seen
            seen.add(key)
            grp, peer = C.c_int(), C.c_int()
            assert H.mpxh_round_role(n, r, a, C.byref(grp), C.byref(peer)) == 0
            assert (grp.value, peer.value) == (1, b)
    assert len(seen) == n * (n - 1) // 2
    assert H.mpxh_round_pairs(3, 0, (C.c_int * 4)()) == -1


@pytest.mark.parametrize("mode", ["pingpong", "nonblocking", "unidir"])
@pytest.mark.parametrize("n", [2, 4, 8])
def test_every_round_is_a_reference_run_with_ppn_half(H, n, mode):
    """round r of the N-GPU schedule is the reference's own run
    with ppn = N/2 on two hosts (golden <mode>_p<N/2>_*: ranks [0, N/2) are
    group 1, rank l's peer is l +- N/2, mpi_perf.c:225-233,447-450) under the
    rank relabelling sigma_r(l) = order_r[l] for l < N/2 and
    order_r[3N/2 - 1 - l] for l >= N/2, where order_r is the circle method's
    seating of round r (rank 0 fixed, the rest rotated r places:
    mpxh_round_pairs pairs seat k with seat N-1-k).  The reference run's
    group / peer of every logical rank, mapped through sigma_r, must be what
    mpxh_round_role gives the GPU rank sigma_r(l) in round r."""
    ref = CASES[f"{mode}_p{n // 2}_b8_i10"]
    info = {d["rank"]: d for d in ref["info"]}
    assert sorted(info) == list(range(n))
    for r in range(n - 1):
        pairs = (C.c_int * n)()
        assert H.mpxh_round_pairs(n, r, pairs) == n // 2
        # seat k of round r: the G1 end of pair k for k < N/2, the G0 end of
        # pair N-1-k otherwise
        order = [0] * n
        for k in range(n // 2):
            order[k], order[n - 1 - k] = pairs[2 * k], pairs[2 * k + 1]
        sigma = [order[l] if l < n // 2 else order[3 * n // 2 - 1 - l] for l in range(n)]
        assert sorted(sigma) == list(range(n))                        # a relabelling
        for l in range(n):
            grp, peer = C.c_int(), C.c_int()
            assert H.mpxh_round_role(n, r, sigma[l], C.byref(grp), C.byref(peer)) == 0
            assert (grp.value, peer.value) == (info[l]["group"], sigma[info[l]["peer"]]), (r, l)
        # the round's senders (record writers, mpi_perf.c:545) are sigma of the
        # reference's record ranks
        writers = sorted({rec["rank"] for rec in ref["records"]})
        assert writers == list(range(n // 2))
        assert sorted(sigma[w] for w in writers) == sorted(pairs[2 * k] for k in range(n // 2))


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if c["records"]][:20])
def test_record_format_matches_reference(H, name):
    c = CASES[name]
    ppn = int(c["args"][c["args"].index("-p") + 1])
    for rec in c["records"]:
        out = C.create_string_buffer(1024)
        H.mpxh_format_record(out, 1024, b"T", b"U", rec["rank"], c["np"], ppn, rec["local_ip"].encode(),
                             rec["remote_ip"].encode(), rec["buffer_size"], rec["num_buffers"],
                             float(rec["time_ms_text"]) / 1000.0, rec["run_id"])
        fld = out.value.decode().rstrip("\n").split(",")
        assert fld[9] == rec["time_ms_text"]
        fld[9] = "X"
        assert ",".join(fld) == rec["line_masked"]


def test_summary_bandwidth_logname_formats(H):
    out = C.create_string_buffer(512)
    H.mpxh_format_summary(out, 512, 1000, 0.012345, 0.001, 0.002, 0.006, 4)
    assert out.value.decode() == "[Run#: 1000]: Total time: 12.35 ms, Min: 1.00 ms, Max: 2.00 ms, Avg: 1.50 ms\n"
    H.mpxh_format_bandwidth(out, 512, 3, 7, 4194304, 5000, 0, 2.0)
    assert out.value.decode() == \
        f"[Rank: 3 Run#: 7]: Total Gbits: {8 * 4194304 * 5000 * 2 * 1e-9:f}, Bandwidth: " \
        f"{8 * 4194304 * 5000 * 2 * 1e-9 / 2.0:.2f} Gbps\n"
    H.mpxh_log_name(out, 512, b"/mnt/tcp-logs", b"U", 3, b"2026-01-02-03-04-05")
    assert out.value == b"/mnt/tcp-logs/tcp-U-3-2026-01-02-03-04-05.log"
    H.mpxh_format_dotnet(out, 512, 1, 2, 3, b"10.0.0.2", b"10.0.0.1", 8, 10, 1)
    assert out.value.decode().endswith("server 10.0.0.1 40002 1 1 8 10 0 true\n")
    H.mpxh_format_dotnet(out, 512, 0, 3, 2, b"10.0.0.1", b"10.0.0.2", 8, 10, 1)
    assert out.value.decode().endswith("client 10.0.0.1 40002 1 8 10 0 true\n")


def test_processor_names_and_uuid(H):
    out = C.create_string_buffer(128)
    H.mpxh_processor_name(out, b"node", 5, 4, None)
    assert out.value == b"node-1"
    H.mpxh_processor_name(out, b"node", 2, 1, b"vm,vm,runsc,runsc")
    assert out.value == b"runsc"
    u = C.create_string_buffer(37)
    H.mpxh_uuid(u)
    assert re.fullmatch(rb"[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}", u.value)


# ---- CLI error exits, compared with the reference's (golden) -------------
def run_perf(args, tmp_path, lines=("vm",), names="vm,runsc"):
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(tmp_path / "logs")) for a in args]
    # MPX_HOSTNAME=localhost: this host's IPv4 is 127.0.0.1, as the golden
    # runs resolved their ranks' processor names (mpi_perf.c:236-237)
    env = dict(os.environ, MPX_PROCESSOR_NAMES=names, MPX_HOSTNAME="localhost")
    return subprocess.run([PERF] + argv, capture_output=True, text=True, env=env, timeout=60)


@pytest.mark.parametrize("name", ["err_unknown_flag", "err_h_flag", "err_bad_group_size", "err_zero_group_size",
                                  "err_missing_group_file", "err_all_in_group1_no_peer", "err_bidir_no_ppn_sigfpe"])
def test_cli_error_exits_match_reference(tmp_path, name):
    c = CASES[name]
    names = ",".join([c["host1"]] * c["ppn"] + [c["host0"]] * (c["np"] - c["ppn"]))
    p = run_perf(["-w", str(c["np"])] + c["args"], tmp_path, lines=c["group1_lines"], names=names)
    if c["returncode"] == signal.SIGFPE:      # mpiexec reports the rank's signal number
        assert p.returncode == -signal.SIGFPE
    else:
        assert p.returncode == c["returncode"] == 255
    for msg in c["messages"]:
        assert msg in p.stderr, (msg, p.stderr[-400:])
    assert ("UUID: " in p.stderr) == c["uuid_printed"] or name in ("err_unknown_flag", "err_h_flag")


def test_dotnet_mode_matches_reference(tmp_path):
    """-d 1 prints the launcher command per rank per run and writes no record
    (mpi_perf.c:147-168, :545); it needs no GPU, like the reference.  The
    lines are compared whole, IPv4 addresses included."""
    c = CASES["dotnet_print_only"]
    p = run_perf(["-w", "2"] + c["args"], tmp_path, lines=c["group1_lines"], names="vm,runsc")
    assert p.returncode == 0, p.stderr[-500:]
    mine = sorted(re.findall(r"^dotnet .*$", p.stderr, flags=re.M))
    assert mine == sorted(c["dotnet"])
    logs = tmp_path / "logs"
    assert len(list(logs.glob("tcp-*.log"))) == len(c["files"]) == 1
    assert all(f.stat().st_size == 0 for f in logs.glob("tcp-*.log")) and c["n_records"] == 0
    assert ("[Run#: 0]" in p.stderr) == (c["summaries"] == [0])


def test_kusto_file_selection_on_a_directory_mpx_perf_wrote(tmp_path):
    """kusto_ingest.py:32-40's selection rule (tests/kusto_rule.py) applied to
    the log directory an mpx_perf run really wrote: -d 1 (no GPU needed),
    rotation every run (MPX_LOG_REFRESH_SEC), so several tcp-*.log files and
    their gpu-*.csv side files.  Only tcp files are picked, oldest first,
    all but the newest n; the side files never."""
    import time
    import kusto_rule as K
    g1 = tmp_path / "group1"
    g1.write_text("vm\n")
    logs = tmp_path / "logs"
    env = dict(os.environ, MPX_PROCESSOR_NAMES="vm,runsc", MPX_LOG_REFRESH_SEC="0")
    for k in range(3):     # three jobs: log names differ by UUID (and second)
        p = subprocess.run([PERF, "-w", "2", "-f", str(g1), "-n", "1", "-p", "1", "-d", "1", "-r", "2",
                            "-l", str(logs)], capture_output=True, text=True, env=env, timeout=60)
        assert p.returncode == 0, p.stderr[-400:]
        time.sleep(0.02)
    written = sorted(os.listdir(logs))
    tcp = [f for f in written if f.startswith("tcp-")]
    side = [f for f in written if f.startswith("gpu-")]
    assert len(tcp) >= 3 and len(side) == len(tcp)
    for n in (1, 2):
        picked = K.select(str(logs), n)
        assert [os.path.basename(f) for f in picked] == \
            sorted(tcp, key=lambda f: os.path.getmtime(logs / f))[:-n]
        assert not any(os.path.basename(f).startswith("gpu-") for f in picked)


# ---- properties over random layouts (hypothesis) ---------------------------
from hypothesis import given, settings, strategies as st  # noqa: E402


@settings(max_examples=200, deadline=None)
@given(st.lists(st.integers(0, 1), min_size=1, max_size=64))
def test_pairing_matches_oracle_for_any_group_layout(H, groups):
    """Any group assignment of up to 64 ranks (MPX_MAX_RANKS): the C rule
    (mpxh_pairing), its Python mirror and the oracle's restatement of
    mpi_perf.c:225-233,447-450 agree on group rank and peer, including ranks
    left without a peer (-1)."""
    n = len(groups)
    g = (C.c_int * n)(*groups)
    gr, gs, pe = (C.c_int * n)(), (C.c_int * n)(), (C.c_int * n)()
    H.mpxh_pairing(n, g, gr, gs, pe)
    assert pairing_from_groups(groups) == (list(gr), list(pe))
    assert O.pairing(groups) == (list(gr), list(pe))
    assert list(gs) == [groups.count(x) for x in groups]


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 32).map(lambda k: 2 * k))
def test_rounds_are_perfect_matchings_covering_every_pair(H, n):
    """Every even N up to 64: N-1 rounds, each a perfect matching, all
    N(N-1)/2 pairs exactly once, and mpxh_round_role consistent with it."""
    seen = set()
    for r in range(n - 1):
        pairs = (C.c_int * n)()
        assert H.mpxh_round_pairs(n, r, pairs) == n // 2
        ps = [(pairs[2 * k], pairs[2 * k + 1]) for k in range(n // 2)]
        assert sorted(itertools.chain(*ps)) == list(range(n))
        for a, b in ps:
            seen.add((min(a, b), max(a, b)))
            grp, peer = C.c_int(), C.c_int()
            assert H.mpxh_round_role(n, r, b, C.byref(grp), C.byref(peer)) == 0 and (grp.value, peer.value) == (0, a)
    assert len(seen) == n * (n - 1) // 2
