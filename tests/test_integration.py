"""The reference-side binding, compiled and run.

oracle/_ref/mpi_perf_mpx is the reference's own mpi_perf.c (compiled from
/root/reference by `make -C oracle ref-mpx`) with its three transfer loops and
allocate_tx_rx_buffers replaced at link time by integration/mpx_binding.c,
which calls libmpx through include/mpx.h.  Its main() — options, group/peer
rule, run loop, records — is the reference's, untouched; only the bytes move
through the GPU.

CPU: the link really routes main's calls into the binding (symbols, and a
run that reaches libmpx and fails there when no GPU exists), and the GPU-free
`-d 1` mode still matches the reference's golden run.
GPU (-m gpu): two or four MPICH ranks on GPU 0 run the golden cases with
every payload checksummed on the device (MPX_CHECK=1); each rank's receives
completed, bytes and digest are compared with the reference's own ranks
(golden "shim"), and the records with the reference's record lines.
"""
import glob
import json
import os
import pathlib
import re
import subprocess
import tempfile

import pytest

from proc import run_bounded

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "oracle", "_ref", "mpi_perf_mpx")
WRAP = os.path.join(ROOT, "oracle", "ref_wrap.sh")
MPIEXEC = "/opt/conda/bin/mpiexec"
GOLDEN = {c["name"]: c for c in O.golden()["cases"]}
INFO_RE = re.compile(r"INFO: \S+, rank (\d+) out of (\d+) ranks, my_group: (\d+), group_size: (\d+), "
                     r"group_rank: (\d+), my_peer: (-?\d+)")

needs_bin = pytest.mark.skipif(not (os.path.exists(BIN) and os.path.exists(MPIEXEC)),
                               reason="patched reference not built (needs /root/reference: make -C oracle ref-mpx)")


def launch(tmp_path, case, env_extra=None, timeout=90):
    """The golden case's launch (tests/golden/gen_golden.py), with the patched
    binary.  Host names localhost / 127.0.0.1 resolve anywhere, so the record
    IPs are 127.0.0.1 as in the golden runs."""
    c = GOLDEN[case]
    g1 = tmp_path / "group1"
    g1.write_text("localhost\n")
    logs = tmp_path / "logs"
    logs.mkdir()
    argv = [a.replace("@G1", str(g1)).replace("@LOGS", str(logs)) for a in c["args"]]
    ppn = str(c["ppn"])
    env = dict(os.environ, PPN=ppn, HOST1="localhost", HOST0="127.0.0.1", **(env_extra or {}))
    cmd = [MPIEXEC, "-np", str(c["np"]), "-genv", "PPN", ppn, "-genv", "HOST1", "localhost", "-genv", "HOST0",
           "127.0.0.1"]
    for k, v in (env_extra or {}).items():
        cmd += ["-genv", k, v]
    cmd += [WRAP, BIN] + argv
    p = run_bounded(cmd, timeout=timeout, env=env, cwd=tmp_path)
    recs = []
    for f in sorted(glob.glob(str(logs / "tcp-*.log"))):
        recs += [line.rstrip("\n").split(",") for line in open(f)]
    return p, recs


@needs_bin
def test_main_calls_the_binding_not_the_reference_loops():
    """The four patched functions and free() resolve into the binding: the
    reference's own definitions were weakened and dropped from the link."""
    out = subprocess.run(["nm", BIN], capture_output=True, text=True, check=True).stdout
    syms = {}
    for line in out.splitlines():
        f = line.split()
        if len(f) == 3:
            syms.setdefault(f[2], []).append(f[1])
    for name in ("do_mpi_benchmark", "do_mpi_benchmark_nonblocking", "do_mpi_benchmark_unidir",
                 "allocate_tx_rx_buffers", "mpxb_free", "MPI_Finalize"):
        assert syms.get(name) == ["T"], (name, syms.get(name))
    dis = subprocess.run(["objdump", "-d", "--no-show-raw-insn", BIN], capture_output=True, text=True,
                         check=True).stdout
    main = dis[dis.index("<main>:"):]
    main = main[:main.index("\n\n")]
    for name in ("allocate_tx_rx_buffers", "do_mpi_benchmark", "do_mpi_benchmark_nonblocking",
                 "do_mpi_benchmark_unidir", "mpxb_free", "MPI_Finalize"):
        assert re.search(rf"call\s+[0-9a-f]+ <{name}>", main), name
    assert "mpx_xfer" in subprocess.run(["nm", "-D", "--undefined-only", BIN], capture_output=True, text=True,
                                        check=True).stdout


@needs_bin
def test_dotnet_mode_matches_reference(tmp_path):
    """-d 1 never allocates or transfers (mpi_perf.c:465,502-507): the patched
    binary prints the reference's launcher lines and exits 0."""
    p, recs = launch(tmp_path, "dotnet_print_only")
    assert p.returncode == GOLDEN["dotnet_print_only"]["returncode"] == 0, p.stderr[-600:]
    got = sorted(re.findall(r"^dotnet .*$", p.stderr, flags=re.M))
    want = GOLDEN["dotnet_print_only"]["dotnet"]
    assert len(got) == len(want)
    # the golden ran with host names vm/runsc; here both resolve to 127.0.0.1 as there
    assert got == want
    assert recs == []


@needs_bin
@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU node: the loop would run (covered by -m gpu)")
def test_loops_reach_libmpx_without_gpu(tmp_path):
    """Without a GPU the first GPU call fails inside the binding with the
    reference's print-and-exit convention (mpi_perf.c:55-64): proof that
    main's allocation and loops go to libmpx, not to MPI."""
    p, _ = launch(tmp_path, "pingpong_p1_b8_i10", timeout=60)
    assert p.returncode != 0
    assert re.search(r"\[\S*mpx_binding\.c:\d+\] mpx call failed with \d+", p.stderr), p.stderr[-600:]


GPU_CASES = ["pingpong_p1_b1_i10", "pingpong_p1_b456131_i3", "unidir_p1_b8_i10", "unidir_p1_b456131_i3",
             "nonblocking_p1_b4096_i7", "nonblocking_window_i600", "pingpong_p2_b4096_i7", "unidir_p2_b456131_i3",
             "zero_bytes_pingpong", "zero_bytes_unidir", "zero_bytes_nonblocking", "zero_iters",
             "unidir_wins_over_nonblocking", "summary_every_1000", "max_int_buffer"]


def engine_env(engine: str) -> dict:
    """the binding's engine (MPX_ENGINE); "<engine>-pull": that engine with
    every B-byte payload pulled by its receiver (MPX_XFER_PULL=1)"""
    if engine.endswith("-pull"):
        return {"MPX_ENGINE": engine[:-len("-pull")], "MPX_XFER_PULL": "1"}
    return {"MPX_ENGINE": engine}


@pytest.mark.gpu
@needs_bin
@pytest.mark.parametrize("engine", ["kernel", "sdma", "kernel-pull", "sdma-pull"])
@pytest.mark.parametrize("case", GPU_CASES)
def test_patched_reference_receives_match_reference(tmp_path, case, engine):
    c = GOLDEN[case]
    out = str(tmp_path / "recv")
    p, recs = launch(tmp_path, case, {"MPX_CHECK": "1", "MPX_RECV_OUT": out, **engine_env(engine)})
    assert p.returncode == 0, p.stderr[-1500:]
    # pairing printed by the reference's own main (mpi_perf.c:460)
    info = sorted((tuple(int(x) for x in m.groups()) for m in INFO_RE.finditer(p.stderr)))
    assert info == sorted((d["rank"], d["world"], d["group"], d["group_size"], d["group_rank"], d["peer"])
                          for d in c["info"])
    # every payload was checksummed on the device; the totals per rank are
    # the reference ranks' receive accounting
    for r in range(c["np"]):
        d = json.load(open(f"{out}.{r}.json"))
        ref = c["shim"][str(r)]
        assert (d["recv_done"], d["recv_bytes"], d["recv_digest"]) == \
            (ref["recv_done"], ref["recv_bytes"], ref["recv_digest"]), (r, d, ref)
    # the reference's run summary every 1000 runs (mpi_perf.c:564-568)
    assert sorted(int(m) for m in re.findall(r"^\[Run#: (\d+)\]: Total time", p.stderr, flags=re.M)) == \
        c["summaries"]
    # records: the reference's own writer (mpi_perf.c:551-554); everything
    # but time / uuid / timestamp compares, first 8 by (rank, run id) as kept
    recs.sort(key=lambda f: (int(f[2]), int(f[10])))
    assert len(recs) == c["n_records"]
    assert [",".join(["T", "U"] + f[2:9] + ["X"] + f[10:]) for f in recs[:8]] == \
        [x["line_masked"] for x in c["records"]]


# ---- random configurations against the live reference (GPU box) -----------
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

# the LL/bulk protocol switch (2 KiB on one GPU, 8 KiB across GPUs: ll_max_bytes,
# csrc/mpx_internal.h) and 16-B unit tails on either side of it
LL_EDGES = [15, 16, 17, 2047, 2048, 2049, 4096, 8191, 8192, 8193, 16383, 16384, 16385]

REF = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")


def _shim_json(prefix, np_):
    return [json.load(open(f"{prefix}.{r}.json")) for r in range(np_)]


@pytest.mark.gpu
@needs_bin
@pytest.mark.skipif(not os.path.exists(REF), reason="compiled reference not built")
@settings(max_examples=int(os.environ.get("MPX_FUZZ_EXAMPLES", "30")), deadline=None,
          derandomize=not os.environ.get("MPX_FUZZ_EXAMPLES"),
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(mode=st.sampled_from(["pingpong", "nonblocking", "unidir"]), ppn=st.sampled_from([1, 2]),
       B=st.one_of(st.integers(0, 64), st.sampled_from(LL_EDGES), st.integers(65, 300000),
                   st.integers(300001, 8 << 20)), iters=st.integers(1, 40),
       window=st.booleans(), engine=st.sampled_from(["kernel", "sdma", "kernel-pull"]))
def test_random_runs_match_the_live_reference(tmp_path, mode, ppn, B, iters, window, engine):
    """A random (loop, ppn, B, iterations) — beyond the golden fixtures — run
    twice: by the compiled reference itself on the host (MPICH shared memory,
    the PMPI shim digesting every receive it completes) and by the same
    reference main() over libmpx on GPU 0 (every payload checksummed on the
    device).  Per rank: receives completed, bytes and digest must be equal.
    The non-blocking loop sometimes runs 255-600 iterations (its window)."""
    if mode == "nonblocking" and window:
        iters = 255 + iters * 9          # 264 .. 615: one or two flushes, slot 255 left pending
    np_ = 2 * ppn
    d = pathlib.Path(tempfile.mkdtemp(dir=tmp_path))
    (d / "group1").write_text("localhost\n")
    (d / "logs").mkdir()
    args = ["-f", "group1", "-n", "1", "-p", str(ppn), "-r", "2", "-i", str(iters), "-b", str(B), "-l", "logs"]
    args += {"pingpong": [], "nonblocking": ["-x", "1"], "unidir": ["-u", "1"]}[mode]
    base = [MPIEXEC, "-np", str(np_), "-genv", "PPN", str(ppn), "-genv", "HOST1", "localhost", "-genv", "HOST0",
            "127.0.0.1"]
    shim = str(d / "shim")
    ref = run_bounded(base + ["-genv", "SHIM_OUT", shim, WRAP, REF] + args, timeout=60, cwd=d,
                      env=dict(os.environ, SHIM_OUT=shim))
    assert ref.returncode == 0, ref.stderr[-800:]
    out = str(d / "recv")
    env = {"MPX_CHECK": "1", "MPX_RECV_OUT": out, **engine_env(engine)}
    ours = run_bounded(base + sum((["-genv", k, v] for k, v in env.items()), []) + [WRAP, BIN] + args, timeout=60,
                       cwd=d, env=dict(os.environ, **env))
    assert ours.returncode == 0, ours.stderr[-800:]
    want = [(x["recv_done"], x["recv_bytes"], x["recv_digest"]) for x in _shim_json(shim, np_)]
    got = [(x["recv_done"], x["recv_bytes"], x["recv_digest"]) for x in _shim_json(out, np_)]
    assert got == want, (mode, ppn, B, iters, engine)
