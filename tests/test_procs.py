"""mpx_perf's processes mode (one process per rank under a launcher, like the
reference's `mpirun -np N mpi_perf`) and its TCP job communicator
(host/mpx_boot.c), on CPU.

* the collectives (allgather, bcast, barrier, allreduce) across 4 processes;
* the GPU-free `-d 1` mode, started as separate processes by hand and under
  MPICH's mpiexec, against the reference's golden run: pairing, INFO lines,
  launcher lines, log files, summary;
* the CLI error exits: every process of the job ends the way the reference's
  job does, and the message is printed once (by rank 0).
The GPU side of the same mode is in test_gpu_host.py.
"""
import json
import os
import re
import signal
import socket
import subprocess
import sys

import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
WORKER = os.path.join(ROOT, "tests", "boot_worker.py")
MPIEXEC = "/opt/conda/bin/mpiexec"
CASES = {c["name"]: c for c in O.golden()["cases"]}


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("size", [1, 2, 4, 7])
def test_boot_collectives(size):
    port = free_port()
    ps = [subprocess.Popen([sys.executable, WORKER, str(r), str(size), str(port)], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True) for r in range(size)]
    outs = [p.communicate(timeout=60) for p in ps]
    assert all(p.returncode == 0 for p in ps), [o[1][-300:] for o in outs]
    res = sorted((json.loads(o[0]) for o in outs), key=lambda d: d["rank"])
    want = []
    for r in range(size):
        want += [r, r * r, 0xABCD0000 + r]
    for r, d in enumerate(res):
        assert d["rank"] == r and d["size"] == size
        assert d["allgather"] == want
        assert d["bcast"] == "rank0-says-hello"
        assert d["reduce"] == [0.25, 0.25 + size - 1, sum(0.25 + q for q in range(size))]
        assert d["big_ok"]


def test_boot_reports_a_missing_rank():
    port = free_port()
    ps = [subprocess.Popen([sys.executable, WORKER, str(r), "3", str(port), "1.5"], stdout=subprocess.PIPE,
                           stderr=subprocess.PIPE, text=True) for r in range(2)]
    outs = [p.communicate(timeout=60) for p in ps]
    hub = json.loads(outs[0][0])
    assert ps[0].returncode == 3 and "only 2 of 3 ranks joined" in hub["error"]
    assert ps[1].returncode != 0      # the leaf loses its hub


def run_job(tmp_path, args, n, names, lines=("vm",), extra_env=None):
    """n mpx_perf processes, ranks from MPX_RANK/MPX_SIZE (the launcher variables)."""
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(tmp_path / "logs")) for a in args]
    port = free_port()
    ps = []
    for r in range(n):
        env = dict(os.environ, MPX_RANK=str(r), MPX_SIZE=str(n), MPX_LOCAL_RANK=str(r),
                   MPX_BOOTSTRAP=f"127.0.0.1:{port}", MPX_PROCESSOR_NAMES=names, MPX_BOOTSTRAP_TIMEOUT="30")
        env.update(extra_env or {})
        ps.append(subprocess.Popen([PERF] + argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                   env=env, cwd=tmp_path))
    outs = [p.communicate(timeout=120) for p in ps]
    return [p.returncode for p in ps], [o[1] for o in outs]


def _mask_ip(line):
    return re.sub(r"\d+\.\d+\.\d+\.\d+(:gpu\d+)?", "IP", line)


INFO = re.compile(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d), group_size: (\d+), "
                  r"group_rank: (\d+), my_peer: (-?\d+)")


def test_dotnet_mode_as_processes_matches_reference(tmp_path):
    c = CASES["dotnet_print_only"]
    rcs, errs = run_job(tmp_path, c["args"], 2, "vm,runsc", lines=c["group1_lines"])
    assert rcs == [0, 0], errs
    allerr = "".join(errs)
    mine = sorted(_mask_ip(x) for x in re.findall(r"^dotnet .*$", allerr, flags=re.M))
    assert mine == sorted(_mask_ip(x) for x in c["dotnet"])
    info = sorted((int(x[1]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in INFO.findall(allerr))
    assert info == sorted((d["rank"], d["group"], d["group_size"], d["group_rank"], d["peer"]) for d in c["info"])
    # each process prints only its own INFO line (mpi_perf.c:460-461)
    assert [len(INFO.findall(e)) for e in errs] == [1, 1]
    assert allerr.count("UUID: ") == 1 and allerr.count("[Run#: 0]") == 1
    logs = tmp_path / "logs"
    assert len(list(logs.glob("tcp-*.log"))) == len(c["files"]) == 1


@pytest.mark.skipif(not os.path.exists(MPIEXEC), reason="MPICH mpiexec not in this image")
@pytest.mark.parametrize("ppn", [1, 2, 4])
def test_dotnet_mode_under_mpiexec(tmp_path, ppn):
    """Started by a real MPI launcher (PMI_RANK / PMI_SIZE / MPI_LOCALRANKID):
    the pairing equals the reference's for the same layout (golden
    pingpong_p<ppn> cases, mpi_perf.c:437-458)."""
    ref = CASES[f"pingpong_p{ppn}_b8_i10"]
    (tmp_path / "group1").write_text("vm\n")
    names = ",".join(["vm"] * ppn + ["runsc"] * ppn)
    p = subprocess.run([MPIEXEC, "-n", str(2 * ppn), "-genv", "MPX_PROCESSOR_NAMES", names, "-genv",
                        "MPX_BOOTSTRAP", f"127.0.0.1:{free_port()}", PERF, "-f", "group1", "-n", "1", "-p",
                        str(ppn), "-d", "1", "-r", "2", "-i", "10", "-b", "8", "-l", "logs"],
                       capture_output=True, text=True, cwd=tmp_path, timeout=120)
    assert p.returncode == 0, p.stderr[-600:]
    info = sorted((int(x[1]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in INFO.findall(p.stderr))
    assert info == sorted((d["rank"], d["group"], d["group_size"], d["group_rank"], d["peer"]) for d in ref["info"])
    assert len(re.findall(r"^dotnet .* server ", p.stderr, flags=re.M)) == 2 * ppn   # G1 ranks x 2 runs


@pytest.mark.parametrize("name", ["err_unknown_flag", "err_bad_group_size", "err_zero_group_size",
                                  "err_missing_group_file", "err_all_in_group1_no_peer", "err_bidir_no_ppn_sigfpe"])
def test_cli_error_exits_as_processes(tmp_path, name):
    c = CASES[name]
    names = ",".join([c["host1"]] * c["ppn"] + [c["host0"]] * (c["np"] - c["ppn"]))
    rcs, errs = run_job(tmp_path, c["args"], c["np"], names, lines=c["group1_lines"])
    if c["returncode"] == signal.SIGFPE:
        assert rcs == [-signal.SIGFPE] * c["np"]
    else:
        assert rcs == [255] * c["np"], errs
    allerr = "".join(errs)
    for msg in c["messages"]:
        assert msg in allerr, (msg, allerr[-400:])
        if "getaddrinfo" not in msg:
            assert allerr.count(msg) == 1, msg        # printed by rank 0 only


def test_world_flag_must_match_the_launcher(tmp_path):
    rcs, errs = run_job(tmp_path, ["-w", "4", "-f", "@G1", "-n", "1", "-p", "1", "-d", "1", "-r", "1"], 2,
                        "vm,runsc")
    assert rcs == [255, 255]
    assert "-w 4 but the launcher started 2 ranks" in "".join(errs)


def test_threads_mode_can_be_forced_under_a_launcher(tmp_path):
    """MPX_LAUNCH=threads: one process runs every rank even with launcher
    variables in its environment (e.g. started from a torchrun worker)."""
    g1 = tmp_path / "group1"
    g1.write_text("vm\n")
    env = dict(os.environ, MPX_RANK="0", MPX_SIZE="2", MPX_LAUNCH="threads", MPX_PROCESSOR_NAMES="vm,runsc")
    p = subprocess.run([PERF, "-w", "2", "-f", str(g1), "-n", "1", "-p", "1", "-d", "1", "-r", "1", "-i", "1",
                        "-b", "8", "-l", str(tmp_path / "logs")], capture_output=True, text=True, env=env,
                       timeout=60)
    assert p.returncode == 0, p.stderr[-400:]
    assert len(INFO.findall(p.stderr)) == 2


def run_nodes(tmp_path, args, hosts, lines=("nodeA",), extra_env=None):
    """One mpx_perf process per rank; rank r reports host hosts[r]
    (MPX_HOSTNAME) and its node-local rank, as a launcher spanning several
    nodes would start them (multi-node rehearsal on one machine)."""
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(tmp_path / "logs")) for a in args]
    port = free_port()
    ps = []
    n = len(hosts)
    for r in range(n):
        local = hosts[:r].count(hosts[r])
        env = dict(os.environ, MPX_RANK=str(r), MPX_SIZE=str(n), MPX_LOCAL_RANK=str(local),
                   MPX_BOOTSTRAP=f"127.0.0.1:{port}", MPX_PROCESSOR_NAMES="", MPX_HOSTNAME=hosts[r],
                   MPX_BOOTSTRAP_TIMEOUT="30", HIP_VISIBLE_DEVICES="")
        env.update(extra_env or {})
        ps.append(subprocess.Popen([PERF] + argv, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                   env=env, cwd=tmp_path))
    outs = [p.communicate(timeout=120) for p in ps]
    return [p.returncode for p in ps], [o[1] for o in outs]


def test_multi_node_groups_by_host_name(tmp_path):
    """Ranks on two nodes: the processor name is the host
    name, as MPI_Get_processor_name gives it (mpi_perf.c:433-434), so the -f
    file lists nodes and --map-by ppr:2:node pairs rank k with rank 2+k, the
    reference's pingpong_p2 layout.  The ingest hook runs on node-local rank 0
    of the group-1 node only (mpi_perf.c:355-365, :378-384)."""
    ref = CASES["pingpong_p2_b8_i10"]
    rcs, errs = run_nodes(tmp_path, ["-f", "@G1", "-n", "1", "-p", "2", "-d", "1", "-r", "2", "-i", "10", "-b", "8",
                                     "-l", "@LOGS"], ["nodeA", "nodeA", "nodeB", "nodeB"],
                          extra_env={"MPX_INGEST_CMD": "touch ingest-$MPX_RANK"})
    assert rcs == [0] * 4, errs
    allerr = "".join(errs)
    info = INFO.findall(allerr)
    assert sorted((int(x[1]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in info) == \
        sorted((d["rank"], d["group"], d["group_size"], d["group_rank"], d["peer"]) for d in ref["info"])
    assert {(int(x[1]), x[0]) for x in info} == {(0, "nodeA"), (1, "nodeA"), (2, "nodeB"), (3, "nodeB")}
    assert sorted(p.name for p in tmp_path.glob("ingest-*")) == ["ingest-0"]


def test_kernel_engine_refuses_a_pair_across_nodes(tmp_path):
    """The kernel and SDMA engines write into the peer's HBM: a pair spanning
    two nodes is a configuration error, reported before any GPU call; the
    RCCL engine passes the check (and here, without a GPU, stops at the
    device query)."""
    args = ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r", "2", "-l", "@LOGS"]
    for engine in ("kernel", "sdma"):
        rcs, errs = run_nodes(tmp_path, args + ["-e", engine], ["nodeA", "nodeB"])
        assert rcs == [255, 255], errs
        assert "are on different hosts: the %s engine needs both on one node (use -e rccl)" % engine in "".join(errs)
    rcs, errs = run_nodes(tmp_path, args + ["-e", "rccl"], ["nodeA", "nodeB"])
    assert "different hosts" not in "".join(errs)
    assert all(rc != 0 for rc in rcs) and "hipGetDeviceCount" in "".join(errs)


def test_same_node_pairs_pass_the_node_check(tmp_path):
    rcs, errs = run_nodes(tmp_path, ["-f", "@G1", "-n", "1", "-p", "1", "-u", "1", "-r", "2", "-l", "@LOGS"],
                          ["nodeA", "nodeA"], lines=("nodeA-0",),
                          extra_env={"MPX_PROCESSOR_NAMES": "nodeA-0,nodeA-1"})
    assert "different hosts" not in "".join(errs)
    assert "hipGetDeviceCount" in "".join(errs)


REF = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")
WRAP = os.path.join(ROOT, "oracle", "ref_wrap.sh")


@pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(MPIEXEC)),
                    reason="compiled reference not built (make -C oracle ref)")
@pytest.mark.parametrize("flows", [8, 10])
def test_hbv3_shape_pairing_matches_the_live_reference(tmp_path, flows):
    """run-hbv3.sh's launch shape, 2 hosts x `flows` ranks (scripts/run-hbv3.sh:
    -np 20 --map-by ppr:10:node, -p 10): beyond the golden fixtures' ppn <= 4,
    so the compiled reference runs here, live, as the checker (-d 1: no
    transfer).  mpx_perf -w 2*flows must print the same pairing (mpi_perf.c:
    437-461) and the same number of launcher lines (:147-168)."""
    n = 2 * flows
    (tmp_path / "group1").write_text("vm\n")
    args = ["-f", "group1", "-n", "1", "-p", str(flows), "-u", "1", "-d", "1", "-r", "2", "-i", "10", "-b", "456131",
            "-l", "logs"]
    (tmp_path / "logs").mkdir()
    ref = subprocess.run([MPIEXEC, "-np", str(n), "-genv", "PPN", str(flows), "-genv", "HOST1", "vm", "-genv", "HOST0",
                          "runsc", WRAP, REF] + args, capture_output=True, text=True, cwd=tmp_path, timeout=120)
    assert ref.returncode == 0, ref.stderr[-600:]
    names = ",".join(["vm"] * flows + ["runsc"] * flows)
    ours = subprocess.run([PERF, "-w", str(n)] + args, capture_output=True, text=True, cwd=tmp_path, timeout=60,
                          env=dict(os.environ, MPX_PROCESSOR_NAMES=names, MPX_HOSTNAME="localhost"))
    assert ours.returncode == 0, ours.stderr[-600:]

    def pairing(err):
        return sorted((int(x[1]), int(x[2]), int(x[3]), int(x[4]), int(x[5]), int(x[6])) for x in INFO.findall(err))

    want = pairing(ref.stderr)
    assert len(want) == n and all(r[5] == (r[0] + flows) % n for r in want)
    assert pairing(ours.stderr) == want
    count = lambda err: len(re.findall(r"^dotnet ", err, flags=re.M))  # noqa: E731
    assert count(ours.stderr) == count(ref.stderr) == 2 * n
