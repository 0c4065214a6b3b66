"""The command line against the compiled reference, live.

Random flag combinations (hypothesis) run through the reference under MPICH
(oracle/_ref/mpi_perf via oracle/ref_wrap.sh: ranks [0, np/2) report host
"vm", the rest "runsc") and through mpx_perf -w np with the same processor
names.  Every combination carries -d 1, so neither side moves data
(mpi_perf.c:465,502-507) and the comparison runs on the CPU.  Compared: the
exit status (0, 255 for MPI_Abort, SIGFPE for the reference's division by a
zero ppn), the error message, every rank's INFO pairing (mpi_perf.c:460), the
launcher lines (:147-168) and the rank-0 summaries (:564-568).  Beyond the
63 golden fixtures, this covers the option parser, defaults and validation
(:257-339, :388-403) on inputs nobody wrote down.
"""
import os
import pathlib
import re
import signal
import subprocess
import tempfile

import pytest
from hypothesis import HealthCheck, given, settings, strategies as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")
WRAP = os.path.join(ROOT, "oracle", "ref_wrap.sh")
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
MPIEXEC = "/opt/conda/bin/mpiexec"

pytestmark = pytest.mark.skipif(not (os.path.exists(REF) and os.path.exists(MPIEXEC)),
                                reason="compiled reference not built (make -C oracle ref)")

INFO = re.compile(r"INFO: \S+, rank (\d+) out of (\d+) ranks, my_group: (\d+), group_size: (\d+), "
                  r"group_rank: (\d+), my_peer: (-?\d+)")
MESSAGES = ("invalid group_size", "getaddrinfo error", "Usage: <program>", "cannot open group1 file")


def _mask(line: str) -> str:
    return re.sub(r"\d+\.\d+\.\d+\.\d+", "IP", line)


def observe(rc: int, err: str) -> dict:
    """What both programs must agree on.  The reference's ranks run as
    processes under mpiexec (a signal shows as its number), mpx_perf's as
    threads of one process (a signal shows as -number)."""
    if rc < 0:
        rc = -rc
    out = dict(rc=rc, messages=[m for m in MESSAGES if m in err])
    if rc == 0:
        out["info"] = sorted(tuple(int(x) for x in m.groups()) for m in INFO.finditer(err))
        out["dotnet"] = sorted(_mask(x) for x in re.findall(r"^dotnet .*$", err, flags=re.M))
        out["summaries"] = sorted(int(x) for x in re.findall(r"^\[Run#: (\d+)\]", err, flags=re.M))
    return out


flag = st.fixed_dictionaries({}, optional={
    "-n": st.integers(0, 3), "-p": st.integers(0, 3), "-u": st.integers(0, 1), "-x": st.integers(0, 1),
    "-r": st.integers(0, 3), "-i": st.integers(1, 5), "-b": st.sampled_from([1, 8, 100]),
    "-h": st.just(1), "-z": st.just(1)})   # no case for -h, unknown -z: usage + abort (mpi_perf.c:329-331)


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(np_=st.sampled_from([2, 4]), lines=st.sampled_from([("vm",), ("VM",), ("runsc",), ("nohost",), ("nohost", "vm")]),
       flags=flag)
def test_cli_matches_the_live_reference(tmp_path, np_, lines, flags):
    ppn_layout = np_ // 2
    d = pathlib.Path(tempfile.mkdtemp(dir=tmp_path))   # hypothesis may replay an example
    (d / "group1").write_text("".join(x + "\n" for x in lines))
    (d / "logs").mkdir()
    args = ["-f", "group1", "-d", "1", "-l", "logs"]
    for k, v in flags.items():
        args += [k, str(v)]
    ref = subprocess.run([MPIEXEC, "-np", str(np_), "-genv", "PPN", str(ppn_layout), "-genv", "HOST1", "vm",
                          "-genv", "HOST0", "runsc", WRAP, REF] + args,
                         capture_output=True, text=True, cwd=d, timeout=60)
    names = ",".join(["vm"] * ppn_layout + ["runsc"] * ppn_layout)
    ours = subprocess.run([PERF, "-w", str(np_)] + args, capture_output=True, text=True, cwd=d, timeout=60,
                          env=dict(os.environ, MPX_PROCESSOR_NAMES=names, MPX_HOSTNAME="localhost"))
    want, got = observe(ref.returncode, ref.stderr), observe(ours.returncode, ours.stderr)
    if want["rc"] == signal.SIGFPE:   # the reference's crash: only the status and the silence matter
        assert got["rc"] == signal.SIGFPE, (args, ours.stderr[-400:])
        return
    if want["rc"] == 255:   # MPI_Abort: mpiexec may kill the job before it forwards the message
        assert got["rc"] == 255 and got["messages"] and set(want["messages"]) <= set(got["messages"]), \
            (args, ref.stderr[-600:], ours.stderr[-600:])
        return
    assert got == want, (args, ref.stderr[-600:], ours.stderr[-600:])
