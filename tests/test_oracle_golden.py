"""Pin the oracle (CPU restatement, oracle/mpx_oracle.c) against the compiled
reference's golden runs (tests/golden/ref_runs.json, gen_golden.py).

CPU-only.  Covers the group/peer rule (mpi_perf.c:433-450, :200-238), the three
loop semantics' receive accounting (mpi_perf.c:66-145), the nonblocking window
quirk (:108-117), the CSV record and file name (:494, :550-554) and the
bandwidth formula (:538-539).
"""
import re

import pytest

import oracle_py as O

G = O.golden()
CASES = {c["name"]: c for c in G["cases"]}
MODE_OF = {"pingpong": 0, "nonblocking": 1, "unidir": 2}


def _mode(case):
    a = case["args"]
    if "-u" in a and a[a.index("-u") + 1] == "1":
        return 2
    if "-x" in a and a[a.index("-x") + 1] == "1":
        return 1
    return 0


def _arg(case, flag, default):
    a = case["args"]
    return int(a[a.index(flag) + 1]) if flag in a else default


def test_golden_has_every_mode_and_ppn():
    names = set(CASES)
    for m in MODE_OF:
        for p in (1, 2, 4):
            assert any(n.startswith(f"{m}_p{p}_") for n in names)


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if c["info"]])
def test_group_and_peer_rule(name):
    c = CASES[name]
    names = {d["rank"]: d["name"] for d in c["info"]}
    groups = [O.in_group1(names[r], c["group1_lines"]) for r in sorted(names)]
    assert groups == [d["group"] for d in c["info"]]
    if len(c["info"]) == c["np"]:
        gr, peer = O.pairing(groups)
        assert gr == [d["group_rank"] for d in c["info"]]
        assert peer == [d["peer"] for d in c["info"]]
        for d in c["info"]:
            assert d["group_size"] == groups.count(d["group"])


def test_strnicmp_prefix_semantics():
    # name_len chars of the processor name are compared (mpi_perf.c:440)
    assert O.in_group1("vm", ["VMX"]) == 1
    assert O.in_group1("vm", ["v"]) == 0
    assert O.in_group1("vm", ["nohost", "vm"]) == 1
    assert O.in_group1("runsc", ["vm"]) == 0


LOOP_CASES = [c["name"] for c in G["cases"] if re.match(r"(pingpong|nonblocking|unidir)_p\d_b\d+_i\d+$", c["name"])]
LOOP_CASES += ["defaults_unidir", "zero_bytes_pingpong", "zero_bytes_unidir", "zero_bytes_nonblocking",
               "group_upper_prefix_line"]


@pytest.mark.parametrize("name", LOOP_CASES)
def test_loop_receive_accounting_matches_reference(name):
    """The oracle's loops receive exactly what the reference's loops received."""
    c = CASES[name]
    ppn, runs = c["ppn"], _arg(c, "-r", 1)
    iters, B = _arg(c, "-i", 10), _arg(c, "-b", 456131)
    mode = _mode(c)
    tot = [dict(recv_done=0, recv_bytes=0, recv_digest=0) for _ in range(2 * ppn)]
    for _ in range(runs):
        st, _ = O.run_pairs(ppn, mode, iters, B)
        for r in range(2 * ppn):
            for k in tot[r]:
                tot[r][k] = (tot[r][k] + st[r][k]) & 0xFFFFFFFFFFFFFFFF
    for r in range(2 * ppn):
        ref = c["shim"][str(r)]
        assert (tot[r]["recv_done"], tot[r]["recv_bytes"], tot[r]["recv_digest"]) == \
            (ref["recv_done"], ref["recv_bytes"], ref["recv_digest"]), f"rank {r}"


@pytest.mark.parametrize("name", [n for n in CASES if n.startswith("nonblocking_window_")])
def test_nonblocking_window_quirk(name):
    c = CASES[name]
    iters, runs = _arg(c, "-i", 10), _arg(c, "-r", 1)
    for r in ("0", "1"):
        assert c["shim"][r]["recv_done"] == runs * O.lib().oracle_nb_waited(iters)


def test_max_int_buffer_digest():
    c = CASES["max_int_buffer"]
    B = 2147483647
    # G0 (rank 1) received 'b' * B twice, G1 (rank 0) received 'a' once per run
    one_b = O.lib().oracle_checksum(b"b" * 0, 0)  # noqa: F841 (warm the lib)
    assert c["shim"]["1"]["recv_bytes"] == 2 * B
    assert c["shim"]["0"]["recv_bytes"] == 2
    assert c["shim"]["0"]["recv_digest"] == (2 * O.checksum(b"a")) & 0xFFFFFFFFFFFFFFFF


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if c["records"]])
def test_record_format(name):
    c = CASES[name]
    for rec in c["records"]:
        assert rec["n_fields"] == 11 and rec["timestamp_ok"] and rec["uuid_ok"]
        t_s = float(rec["time_ms_text"]) / 1000.0
        line = O.format_record("T", "U", rec["rank"], c["np"], c["ppn"] if "-p" in c["args"] else 1,
                               rec["local_ip"], rec["remote_ip"], rec["buffer_size"], rec["num_buffers"], t_s,
                               rec["run_id"]).rstrip("\n")
        fld = line.split(",")
        fld[9] = "X"
        assert ",".join(fld) == rec["line_masked"]
        # only group-1 ranks write, only for run_idx > 0 (mpi_perf.c:545)
        assert rec["rank"] in [d["rank"] for d in c["info"] if d["group"] == 1]
        assert 1 <= rec["run_id"] < _arg(c, "-r", 1)


@pytest.mark.parametrize("name", [c["name"] for c in G["cases"] if c["returncode"] == 0 and c["info"]])
def test_records_and_files_per_sender(name):
    c = CASES[name]
    runs = _arg(c, "-r", 1)
    senders = [d["rank"] for d in c["info"] if d["group"] == 1]
    dotnet = "-d" in c["args"] and c["args"][c["args"].index("-d") + 1] == "1"
    # records: senders only, runs 1.. only, never in .NET mode (mpi_perf.c:545)
    assert c["n_records"] == (0 if dotnet else len(senders) * max(0, runs - 1))
    assert all(f["shape_ok"] for f in c["files"])
    # a sender opens its log before its first run (mpi_perf.c:479-497)
    assert sorted(f["rank"] for f in c["files"]) == (sorted(senders) if runs != 0 else [])


def test_summary_every_1000_runs():
    assert CASES["summary_every_1000"]["summaries"] == [0, 1000]


def test_bandwidth_formula():
    # mpi_perf.c:538-539: 8*B*iters*(uni?1:2)*1e-9 / t
    assert O.lib().oracle_gbps(4194304, 5000, 0, 2.0) == pytest.approx(8 * 4194304 * 5000 * 2 * 1e-9 / 2.0)
    assert O.lib().oracle_gbps(456131, 10, 1, 0.5) == pytest.approx(8 * 456131 * 10 * 1e-9 / 0.5)


def test_log_name():
    import ctypes
    out = ctypes.create_string_buffer(512)
    O.lib().oracle_log_name(out, 512, b"/mnt/tcp-logs", b"U", 3, b"2026-01-02-03-04-05")
    assert out.value == b"/mnt/tcp-logs/tcp-U-3-2026-01-02-03-04-05.log"


def test_checksum_definition():
    # known answers of the shared checksum definition: empty
    # buffer, tail handling, position dependence, order independence
    assert O.checksum(b"") == 0
    a = O.checksum(b"\x01" + b"\x00" * 15)
    b = O.checksum(b"\x00" * 8 + b"\x01" + b"\x00" * 7)
    assert a != b
    assert O.checksum(b"abc") != O.checksum(b"abc\x00")   # length is mixed in
    x = O.fill(1000, 1, 12345)
    assert len(x) == 1000 and O.checksum(x) == O.pattern_checksum(1000, 1, 12345)
    assert O.fill(9, 0, ord("a")) == b"a" * 9
