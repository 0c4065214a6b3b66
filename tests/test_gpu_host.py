"""The mpx_perf executable on the GPU (two or four ranks sharing GPU 0):
records, log files and check mode, compared with the reference's golden
runs (same flags) and the record format."""
import glob
import os
import pathlib
import re
import subprocess
import tempfile

import pytest

from proc import run_bounded

import oracle_py as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
GOLDEN = {c["name"]: c for c in O.golden()["cases"]}


def run(tmp_path, args, lines=("vm",), names="vm,runsc", gpus="0,0", env_extra=None):
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    logs = tmp_path / "logs"
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(logs)) for a in args]
    # MPX_HOSTNAME=localhost: the ranks' host IPv4 is 127.0.0.1, as in the
    # golden runs, so whole record lines compare (mpi_perf.c:236-237,551-554)
    env = dict(os.environ, MPX_PROCESSOR_NAMES=names, MPX_HOSTNAME="localhost", **(env_extra or {}))
    p = run_bounded([PERF, "-g", gpus, "-t", "5000"] + argv, env=env)
    recs = []
    for f in sorted(glob.glob(str(logs / "tcp-*.log"))):
        recs += [line.rstrip("\n").split(",") for line in open(f)]
    side = []
    for f in sorted(glob.glob(str(logs / "gpu-*.csv"))):
        side += [line.rstrip("\n").split(",") for line in open(f)][1:]
    return p, recs, side


def _record_cases():
    """every golden run that moves data in the -p layout with one -f line"""
    return [c["name"] for c in O.golden()["cases"]
            if not c.get("returncode") and c.get("shim") and "-d" not in c["args"] and c["np"] == 2 * c["ppn"]
            and c["args"][c["args"].index("-n") + 1] == "1"]


@pytest.mark.parametrize("name", _record_cases())
def test_records_match_reference_run(tmp_path, name):
    c = GOLDEN[name]
    names = ",".join([c["host1"]] * c["ppn"] + [c["host0"]] * c["ppn"])
    gpus = ",".join(["0"] * c["np"])
    p, recs, side = run(tmp_path, ["-w", str(c["np"])] + c["args"] + ["-c", "1"], lines=c["group1_lines"],
                        names=names, gpus=gpus)
    assert p.returncode == 0, p.stderr[-600:]
    assert len(recs) == c["n_records"]
    # whole record lines (timestamp, job id and time masked), LocalIP /
    # RemoteIP included; the golden keeps a sample of long runs' records
    assert_records_match(recs, c)
    for f in recs:
        assert len(f) == 11 and re.fullmatch(r"\d{4}-\d\d-\d\d \d\d:\d\d:\d\d", f[0])
        assert re.fullmatch(r"\d+\.\d\d", f[9])
    # INFO lines carry the same pairing as the reference's
    info = re.findall(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d), group_size: (\d+), "
                      r"group_rank: (\d+), my_peer: (-?\d+)", p.stderr)
    assert sorted((int(x[1]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in info) == \
        sorted((d["rank"], d["group"], d["group_size"], d["group_rank"], d["peer"]) for d in c["info"])
    # every payload checked and passed, in every mode; each run's receives,
    # counted on the device, are the reference's (shim totals over all runs)
    runs = int(c["args"][c["args"].index("-r") + 1])
    for f in side:
        assert int(f[16]) == 0 and int(f[15]) == int(f[9])
        ref = c["shim"][f[2]]
        assert int(f[18]) * runs == ref["recv_done"]
        assert (int(f[19]) * runs) & 0xFFFFFFFFFFFFFFFF == ref["recv_digest"]


def assert_records_match(recs, c):
    from collections import Counter
    mine = Counter(mask_record(f) for f in recs)
    ref = Counter(r["line_masked"] for r in c["records"])
    assert not ref - mine, (ref - mine, sorted(mine)[:8])
    if len(c["records"]) == c["n_records"]:
        assert mine == ref


def mask_record(f):
    """a tcp-*.log record with the fields the golden masks (mpi_perf.c:551):
    timestamp T, job id U, time X"""
    return ",".join(["T", "U"] + f[2:9] + ["X", f[10]])


def test_seeded_pattern_check_and_sweep(tmp_path):
    p, recs, side = run(tmp_path, ["-w", "2", "-f", "@G1", "-n", "1", "-p", "1", "-r", "3", "-i", "5", "-S",
                                   "1:1048576", "-c", "2", "-l", "@LOGS"])
    assert p.returncode == 0, p.stderr[-600:]
    sizes = sorted({int(f[7]) for f in recs})
    assert sizes == [1 << k for k in range(21)]
    assert len(recs) == 21 * 2


def test_all_pairs_rounds_on_one_gpu(tmp_path):
    p, recs, side = run(tmp_path, ["-w", "4", "-a", "1", "-f", "@G1", "-n", "1", "-p", "2", "-u", "1", "-r", "7",
                                   "-i", "4", "-b", "65536", "-c", "1", "-l", "@LOGS"], names="vm,vm,runsc,runsc",
                        gpus="0,0,0,0")
    assert p.returncode == 0, p.stderr[-600:]
    rounds = re.findall(r"ROUND (\d+): (.*)", p.stderr)
    assert len(rounds) == 3
    # 6 of 7 runs are recorded, 2 senders each
    assert len(recs) == 6 * 2
    pairs = {(int(f[2]), int(f[6])) for f in side}
    assert len(pairs) >= 3


def test_engines_sdma(tmp_path):
    p, recs, side = run(tmp_path, ["-w", "2", "-e", "sdma", "-f", "@G1", "-n", "1", "-p", "1", "-r", "3", "-i", "20",
                                   "-b", "1048576", "-c", "1", "-l", "@LOGS"])
    assert p.returncode == 0, p.stderr[-600:]
    assert len(recs) == 2 and all(f[13] == "sdma" for f in side)


@pytest.mark.parametrize("mode_args", [[], ["-x", "1"], ["-u", "1"]])
def test_kernel_engine_pull_mode_from_the_environment(tmp_path, mode_args):
    """MPX_XFER_PULL=1 (how mpx_perf and the reference-side binding select
    pull mode): the kernel engine's B-byte payloads are loaded by their
    receivers; every payload checked, the side file names the protocol."""
    p, recs, side = run(tmp_path, ["-w", "2", "-f", "@G1", "-n", "1", "-p", "1", "-r", "3", "-i", "20",
                                   "-b", "1048576", "-c", "1", "-l", "@LOGS"] + mode_args,
                        env_extra={"MPX_XFER_PULL": "1"})
    assert p.returncode == 0, p.stderr[-600:]
    assert len(recs) == 2
    assert all(f[13] == "pull" and int(f[16]) == 0 and int(f[15]) == 20 for f in side), side


def test_unidir_without_ppn_raises_sigfpe_like_reference(tmp_path):
    c = GOLDEN["err_unidir_no_ppn_sigfpe"]
    p, recs, side = run(tmp_path, ["-w", "2"] + c["args"])
    assert p.returncode == -8 and c["returncode"] == 8
    assert len(re.findall(r"INFO: ", p.stderr)) == len(c["info"])


@pytest.mark.parametrize("name", ["zero_iters", "unidir_wins_over_nonblocking", "zero_runs"])
def test_degenerate_loops_match_reference(tmp_path, name):
    c = GOLDEN[name]
    p, recs, side = run(tmp_path, ["-w", "2"] + c["args"])
    assert p.returncode == 0, p.stderr[-600:]
    assert len(recs) == c["n_records"]
    assert len(list((tmp_path / "logs").glob("tcp-*.log")) if (tmp_path / "logs").exists() else []) == len(c["files"])
    assert sorted(int(x) for x in re.findall(r"\[Run#: (\d+)\]", p.stderr)) == c["summaries"]
    if name == "unidir_wins_over_nonblocking":
        assert {f[4] for f in side} == {"2"}            # unidir mode ran


def test_log_rotation_and_ingest_hook(tmp_path):
    """LOG_REFRESH_TIME_SEC rotation (mpi_perf.c:479-497) with the ingest hook
    (mpi_perf.c:355-365) called by node-local rank 0 at every open."""
    hook = tmp_path / "hook.log"
    env_cmd = f"echo ingest >> {hook}"
    g1 = tmp_path / "group1"
    g1.write_text("vm\n")
    env = dict(os.environ, MPX_PROCESSOR_NAMES="vm,runsc", MPX_LOG_REFRESH_SEC="0.001", MPX_INGEST_CMD=env_cmd,
               MPX_HOSTNAME="localhost")
    p = run_bounded([PERF, "-g", "0,0", "-w", "2", "-f", str(g1), "-n", "1", "-p", "1", "-u", "1", "-r", "6",
                        "-i", "20000", "-b", "8", "-l", str(tmp_path / "logs")], env=env)
    assert p.returncode == 0, p.stderr[-600:]
    opened = hook.read_text().count("ingest") if hook.exists() else 0
    files = list((tmp_path / "logs").glob("tcp-*.log"))
    # every run takes >= 6 ms (20000 iterations), far above the 1 ms refresh:
    # the log rotates at every run (file names collide within one second)
    assert opened >= 2 and len(files) >= 1
    total = sum(len(f.read_text().splitlines()) for f in files)
    assert 1 <= total <= 5
    # what kusto_ingest.py would upload from this directory (kusto_ingest.py:
    # 32-40, n = 1): every selected file parses as PerfLogsMPI rows
    # (mpi_perf.c:550-554) of this job; the gpu-*.csv side files are never
    # selected
    import kusto_rule as K
    picked = K.select(str(tmp_path / "logs"), 1)
    assert len(picked) == len(files) - 1
    assert not any(os.path.basename(f).startswith("gpu-") for f in picked)
    for f in picked:
        for line in open(f):
            row = K.parse_row(line)
            assert row["Rank"] == 0 and row["VMCount"] == 2 and row["NumOfFlows"] == 1
            assert row["BufferSize"] == 8 and row["NumOfBuffers"] == 20000 and 1 <= row["RunId"] <= 5
            assert row["LocalIP"] == row["RemoteIP"] == "127.0.0.1"


# ---- processes mode: one mpx_perf process per rank (the reference's model) --
def run_procs(tmp_path, args, n, names, lines=("vm",)):
    """n mpx_perf processes on GPU 0 (launcher variables MPX_RANK/MPX_SIZE,
    -g maps every node-local rank to GPU 0); IPC-mapped peers."""
    import socket
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    logs = tmp_path / "logs"
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(logs)) for a in args]
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = []
    for r in range(n):
        env = dict(os.environ, MPX_RANK=str(r), MPX_SIZE=str(n), MPX_LOCAL_RANK=str(r), MPX_PROCESSOR_NAMES=names,
                   MPX_BOOTSTRAP=f"127.0.0.1:{port}", MPX_BOOTSTRAP_TIMEOUT="60", MPX_HOSTNAME="localhost")
        ps.append(subprocess.Popen([PERF, "-g", ",".join(["0"] * n), "-t", "5000"] + argv, stdout=subprocess.PIPE,
                                   stderr=subprocess.PIPE, text=True, env=env))
    errs = [p.communicate(timeout=120)[1] for p in ps]
    recs, side = [], []
    for f in sorted(glob.glob(str(logs / "tcp-*.log"))):
        recs += [line.rstrip("\n").split(",") for line in open(f)]
    for f in sorted(glob.glob(str(logs / "gpu-*.csv"))):
        side += [line.rstrip("\n").split(",") for line in open(f)][1:]
    return [p.returncode for p in ps], "".join(errs), recs, side


@pytest.mark.parametrize("engine,name", [("kernel", "pingpong_p1_b456131_i3"), ("kernel", "unidir_p2_b4096_i7"),
                                         ("kernel", "nonblocking_p2_b8_i10"), ("sdma", "pingpong_p1_b456131_i3")])
def test_processes_mode_records_match_reference_run(tmp_path, engine, name):
    c = GOLDEN[name]
    names = ",".join(["vm"] * c["ppn"] + ["runsc"] * c["ppn"])
    rcs, err, recs, side = run_procs(tmp_path, c["args"] + ["-e", engine, "-c", "1"], c["np"], names)
    assert rcs == [0] * c["np"], err[-800:]
    assert len(recs) == c["n_records"]
    ref = sorted((r["rank"], r["vmcount"], r["flows"], r["buffer_size"], r["num_buffers"], r["run_id"])
                 for r in c["records"])
    mine = sorted((int(f[2]), int(f[3]), int(f[6]), int(f[7]), int(f[8]), int(f[10])) for f in recs)
    assert mine == ref
    assert len({f[1] for f in recs}) == 1             # one JobId: rank 0's UUID, broadcast
    info = re.findall(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d), group_size: (\d+), "
                      r"group_rank: (\d+), my_peer: (-?\d+)", err)
    assert sorted((int(x[1]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in info) == \
        sorted((d["rank"], d["group"], d["group_size"], d["group_rank"], d["peer"]) for d in c["info"])
    assert_records_match(recs, c)
    runs = int(c["args"][c["args"].index("-r") + 1])
    for f in side:
        assert f[3] == engine
        assert int(f[16]) == 0 and int(f[15]) == int(f[9])
        assert int(f[18]) * runs == c["shim"][f[2]]["recv_done"]


def test_processes_mode_all_pairs_seeded_payloads(tmp_path):
    rcs, err, recs, side = run_procs(tmp_path, ["-a", "1", "-f", "@G1", "-n", "1", "-p", "2", "-u", "1", "-r", "7",
                                                "-i", "5", "-b", "300001", "-c", "2", "-l", "@LOGS"], 4,
                                     "vm,vm,runsc,runsc")
    assert rcs == [0, 0, 0, 0], err[-800:]
    assert len(re.findall(r"ROUND (\d+): ", err)) == 3
    assert len(recs) == 6 * 2
    from mpx.schedule import all_pairs_rounds
    assert {(int(f[2]), int(f[6])) for f in side} == {p for rnd in all_pairs_rounds(4) for p in rnd}
    assert all(int(f[16]) == 0 and int(f[15]) == 5 for f in side)


@pytest.mark.parametrize("mode_args", [[], ["-u", "1"], ["-x", "1"]])
def test_sdma_engine_graph_chunks_from_concurrent_threads(tmp_path, mode_args):
    """-e sdma without -c: every rank thread captures and replays its own
    hipGraph chunks (run_sdma) while the other pair's threads do the same
    (thread-local capture); records for every run, no timeouts."""
    p, recs, side = run(tmp_path, ["-w", "4", "-e", "sdma", "-f", "@G1", "-n", "1", "-p", "2", "-r", "3", "-i", "300",
                                   "-b", "4096", "-l", "@LOGS"] + mode_args, names="vm,vm,runsc,runsc", gpus="0,0,0,0")
    assert p.returncode == 0, p.stderr[-600:]
    assert len(recs) == 2 * 2               # runs 1..2, two senders each
    assert all(int(f[8]) == 300 and int(f[7]) == 4096 for f in recs)


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_processes_mode_eight_ranks_all_28_pairs(tmp_path, engine):
    """BASELINE config 4's process structure on one GPU: eight mpx_perf
    processes (one per rank, as under mpiexec -n 8), -a 1 circle-method
    rounds (7 rounds x 4 pairs = all 28 pairs), seeded payloads, every
    payload checked."""
    names = ",".join(["vm"] * 4 + ["runsc"] * 4)
    rcs, err, recs, side = run_procs(tmp_path, ["-e", engine, "-a", "1", "-f", "@G1", "-n", "1", "-p", "4", "-u", "1",
                                                "-r", "8", "-i", "5", "-b", "65541", "-c", "2", "-l", "@LOGS"], 8, names)
    assert rcs == [0] * 8, err[-800:]
    assert len(re.findall(r"ROUND (\d+): ", err)) == 7
    from mpx.schedule import all_pairs_rounds
    assert {(int(f[2]), int(f[6])) for f in side} == {p for rnd in all_pairs_rounds(8) for p in rnd}
    assert all(int(f[16]) == 0 and int(f[15]) == 5 for f in side)


@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_windows_front_end_runs_and_records(tmp_path, engine):
    """bin/mpx_perf_win (windows/mpi-perf.cpp's positional command line):
    unidirectional runs, records of runs 1.. by the group-1 rank, 7-character
    job id in the records and the log name (:175-184, :333, :354-357), INFO
    lines on stdout, every payload checked."""
    win = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf_win")
    g1 = tmp_path / "group1"
    g1.write_text("10.0.0.2\n")
    logs = tmp_path / "logs"
    env = dict(os.environ, MPX_PROCESSOR_NAMES="10.0.0.1,10.0.0.2")
    p = run_bounded([win, str(g1), "1", "1", "20", "65541", "4", str(logs), "-g", "0,0", "-e", engine,
                     "-c", "1", "-t", "5000"], env=env)
    assert p.returncode == 0, p.stderr[-600:]
    assert len(re.findall(r"^INFO: ", p.stdout, re.M)) == 2 and "UUID:" not in p.stderr
    assert re.search(r"\[Run#: 0\]: Total time: ", p.stderr)
    files = glob.glob(str(logs / "tcp-*.log"))
    assert len(files) == 1
    m = re.fullmatch(r"tcp-([0-9a-f]{7})-1-\d{4}-\d\d-\d\d-\d\d-\d\d-\d\d\.log", os.path.basename(files[0]))
    assert m, files[0]
    recs = [line.rstrip("\n").split(",") for line in open(files[0])]
    assert [int(f[10]) for f in recs] == [1, 2, 3]
    for f in recs:
        assert f[1] == m[1] and f[2] == "1" and f[3] == "2" and f[6] == "1" and f[7] == "65541" and f[8] == "20"
    side = []
    for f in glob.glob(str(logs / "gpu-*.csv")):
        side += [line.rstrip("\n").split(",") for line in open(f)][1:]
    assert len(side) == 3
    for f in side:
        assert f[4] == "2" and int(f[15]) == 20 and int(f[16]) == 0   # unidir, 20 checked, 0 failures


# ---- random runs against the live reference --------------------------------
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

# the LL/bulk protocol switch (2 KiB on one GPU, 8 KiB across GPUs: ll_max_bytes,
# csrc/mpx_internal.h) and 16-B unit tails on either side of it
LL_EDGES = [15, 16, 17, 2047, 2048, 2049, 4096, 8191, 8192, 8193, 16383, 16384, 16385]

REF = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")
WRAP = os.path.join(ROOT, "oracle", "ref_wrap.sh")
MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(MPIEXEC)), reason="compiled reference not built")
@settings(max_examples=int(os.environ.get("MPX_FUZZ_EXAMPLES", "20")), deadline=None,
          derandomize=not os.environ.get("MPX_FUZZ_EXAMPLES"),
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(mode=st.sampled_from([[], ["-x", "1"], ["-u", "1"], ["-u", "1", "-x", "1"]]), ppn=st.sampled_from([1, 2]),
       B=st.one_of(st.integers(0, 64), st.sampled_from(LL_EDGES), st.integers(65, 300000),
                   st.integers(300001, 8 << 20)),
       iters=st.integers(1, 30), runs=st.integers(0, 4),
       engine=st.sampled_from(["kernel", "sdma"]))
def test_random_runs_records_match_the_live_reference(tmp_path, mode, ppn, B, iters, runs, engine):
    """mpx_perf (GPU 0, every payload checked) and the compiled reference
    (host, MPICH shm) with the same random flags: the same record lines
    (timestamp, job id and time masked; mpi_perf.c:545-555 — only group 1,
    only runs 1..), the same INFO pairing, and every payload passed."""
    np_ = 2 * ppn
    d = pathlib.Path(tempfile.mkdtemp(dir=tmp_path))
    (d / "group1").write_text("localhost\n")
    args = ["-f", str(d / "group1"), "-n", "1", "-p", str(ppn), "-r", str(runs), "-i", str(iters), "-b", str(B)] + mode
    (d / "ref_logs").mkdir()
    ref = run_bounded([MPIEXEC, "-np", str(np_), "-genv", "PPN", str(ppn), "-genv", "HOST1", "localhost", "-genv",
                       "HOST0", "127.0.0.1", WRAP, REF] + args + ["-l", str(d / "ref_logs")], timeout=60, cwd=d)
    assert ref.returncode == 0, ref.stderr[-600:]
    want = []
    for f in sorted(glob.glob(str(d / "ref_logs" / "tcp-*.log"))):
        want += [mask_record(line.rstrip("\n").split(",")) for line in open(f)]
    names = ",".join(["localhost"] * ppn + ["127.0.0.1"] * ppn)
    env = dict(os.environ, MPX_PROCESSOR_NAMES=names, MPX_HOSTNAME="localhost")
    ours = run_bounded([PERF, "-w", str(np_), "-g", ",".join(["0"] * np_), "-e", engine, "-t", "5000", "-c", "1"] + args
                       + ["-l", str(d / "logs")], env=env, cwd=d)
    assert ours.returncode == 0, ours.stderr[-600:]
    got, side = [], []
    for f in sorted(glob.glob(str(d / "logs" / "tcp-*.log"))):
        got += [mask_record(line.rstrip("\n").split(",")) for line in open(f)]
    for f in sorted(glob.glob(str(d / "logs" / "gpu-*.csv"))):
        side += [line.rstrip("\n").split(",") for line in open(f)][1:]
    assert sorted(got) == sorted(want), (args, engine)
    assert all(int(f[16]) == 0 and int(f[15]) == iters for f in side), side[:2]
    info = lambda e: sorted(re.findall(r"INFO: \S+, rank (\d+) out of (\d+) ranks, my_group: (\d), "  # noqa: E731
                                       r"group_size: (\d+), group_rank: (\d+), my_peer: (-?\d+)", e))
    assert info(ours.stderr) == info(ref.stderr)
