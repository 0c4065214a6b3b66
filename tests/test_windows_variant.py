"""The Windows / MS-MPI variant's front end (bin/mpx_perf_win, host/mpx_host.c
mpxh_*_windows) against the reference's windows/mpi-perf.cpp.

That source needs MS-MPI and Winsock, so it cannot be built or run here: the
expectations below are read from its code (cited per test) and from the
oracle's restatement of its group rule (oracle_win_*).  Parity of this row is
therefore unpinned by reference runs.  CPU-only: every path checked here ends
before the first GPU call (the INFO lines precede the device query).
"""
import ctypes as C
import os
import random
import re
import signal
import subprocess

import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTLIB = os.path.join(ROOT, "mpi-perf_amd", "lib", "libmpx_host.so")
WIN = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf_win")
PERF = os.path.join(ROOT, "mpi-perf_amd", "bin", "mpx_perf")
INFO = re.compile(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d), group_size: (\d+), "
                  r"group_rank: (\d+), my_peer: (-?\d+), hostname: (\S+) \((\S*)\), peer_host: (\S+) \((\S*)\)")


@pytest.fixture(scope="module")
def H():
    L = C.CDLL(HOSTLIB)
    L.mpxh_in_group1_windows.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.mpxh_in_group1.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    L.mpxh_pairing_windows.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 4
    L.mpxh_pairing.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 4
    L.mpxh_uuid_windows.argtypes = [C.c_char_p]
    O.lib().oracle_win_in_group1.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    O.lib().oracle_win_pairing.argtypes = [C.c_int] + [C.POINTER(C.c_int)] * 3
    return L


def blob(lines, newline=True):
    return b"".join(((ln + "\n") if newline else ln).encode().ljust(128, b"\0")[:128] for ln in lines)


def run(tmp_path, args, lines=("10.0.0.2",), names="10.0.0.1,10.0.0.2"):
    g1 = tmp_path / "group1"
    g1.write_text("".join(x + "\n" for x in lines))
    argv = [str(a).replace("@G1", str(g1)).replace("@LOGS", str(tmp_path / "logs")) for a in args]
    env = dict(os.environ, MPX_PROCESSOR_NAMES=names, HIP_VISIBLE_DEVICES="")
    return subprocess.run([WIN] + argv, capture_output=True, text=True, env=env, timeout=60)


# --- host library vs the oracle's restatement --------------------------------

CASES = [
    ("10.0.0.1", ["10.0.0.1"], 1),
    ("10.0.0.1", ["10.0.0.10"], 0),        # mpi_perf.c would match (prefix of the line)
    ("10.0.0.10", ["10.0.0.1"], 0),
    ("VM-A", ["vm-a"], 1),                 # my_strnicmp: case-insensitive
    ("vm-a", ["vm-b", "VM-A"], 1),
    ("vm", ["vm-a"], 0),
    ("", [""], 1),
]


@pytest.mark.parametrize("addr,lines,want", CASES)
def test_whole_address_membership(H, addr, lines, want):
    """windows/mpi-perf.cpp:283-289: my_strnicmp(my_ipaddr, line, MAX_HOST_SZ)
    over lines whose newline was cut (:259)."""
    got = H.mpxh_in_group1_windows(addr.encode(), blob(lines, newline=False), len(lines))
    assert got == want
    assert O.lib().oracle_win_in_group1(addr.encode(), blob(lines, newline=True), len(lines)) == want


def test_membership_differs_from_linux_prefix_rule(H):
    """The same file groups differently: mpi_perf.c:440 compares only
    strlen(name) characters, so a name that is a prefix of a line matches."""
    lines = blob(["10.0.0.10"])
    assert H.mpxh_in_group1(b"10.0.0.1", lines, 1) == 1
    assert H.mpxh_in_group1_windows(b"10.0.0.1", blob(["10.0.0.10"], newline=False), 1) == 0


def test_random_membership_and_pairing_match_oracle(H):
    rng = random.Random(1234)
    pool = ["10.0.0.%d" % i for i in range(1, 13)] + ["Host%d" % i for i in range(4)] + ["host1"]
    for _ in range(300):
        n = rng.choice([2, 4, 6, 8, 16])
        names = [rng.choice(pool) for _ in range(n)]
        lines = rng.sample(pool, rng.randint(1, 5))
        groups = [H.mpxh_in_group1_windows(x.encode(), blob(lines, newline=False), len(lines)) for x in names]
        assert groups == [O.lib().oracle_win_in_group1(x.encode(), blob(lines), len(lines)) for x in names]
        g = (C.c_int * n)(*groups)
        gr, gs, pe = (C.c_int * n)(), (C.c_int * n)(), (C.c_int * n)()
        H.mpxh_pairing_windows(n, g, gr, gs, pe)
        ogr, ope = (C.c_int * n)(), (C.c_int * n)()
        O.lib().oracle_win_pairing(n, g, ogr, ope)
        assert list(gr) == list(ogr) and list(pe) == list(ope)
        # two groups keyed by world rank: the last match is the only match
        lgr, lgs, lpe = (C.c_int * n)(), (C.c_int * n)(), (C.c_int * n)()
        H.mpxh_pairing(n, g, lgr, lgs, lpe)
        assert list(pe) == list(lpe)


def test_job_id_is_seven_hex_digits(H):
    """generate_uuid (:175-184) formats into sizeof(char *) bytes: 7 characters."""
    seen = set()
    for _ in range(50):
        out = C.create_string_buffer(64)
        H.mpxh_uuid_windows(out)
        assert re.fullmatch(r"[0-9a-f]{7}", out.value.decode())
        seen.add(out.value)
    assert len(seen) > 40


# --- the executable's front end ----------------------------------------------

@pytest.mark.parametrize("nargs", range(0, 7))
def test_missing_positional_argument_crashes(tmp_path, nargs):
    """parse_args reads argv[1..7] unconditionally (:187-197): with fewer, the
    reference hands argv[argc] == NULL to strncpy / atoi and faults."""
    args = ["@G1", "1", "1", "10", "100", "2", "@LOGS"][:nargs]
    p = run(tmp_path, args)
    assert p.returncode == -signal.SIGSEGV


@pytest.mark.parametrize("size", ["0", "-1", "x"])
def test_invalid_group_size(tmp_path, size):
    """:238-242: group_size <= 0 (atoi) -> message + MPI_Abort; uni_dir is
    always 1 here, so the ppn condition never applies."""
    p = run(tmp_path, ["@G1", size, "1", "10", "100", "2", "@LOGS"])
    assert p.returncode == 255
    assert f"invalid group_size: {int(size) if size != 'x' else 0}, world_size: 2, ppn: 1" in p.stderr


def test_bidirectional_validation_does_not_apply(tmp_path):
    """mpi_perf.c would reject -n 3 with 2 ranks in bidirectional mode; the
    Windows variant is unidirectional (:228), so it pairs the ranks."""
    p = run(tmp_path, ["@G1", "3", "1", "10", "100", "2", "@LOGS"])
    assert "invalid group_size" not in p.stderr
    assert len(INFO.findall(p.stdout)) == 2


def test_cannot_open_group_file(tmp_path):
    p = run(tmp_path, [tmp_path / "missing", "1", "1", "10", "100", "2", "@LOGS"])
    assert p.returncode == 255 and "cannot open group1 file:" in p.stderr


def test_no_peer_crashes(tmp_path):
    """A rank without a peer leaves peer_node_info NULL; the INFO fprintf
    (:303-306) dereferences it."""
    p = run(tmp_path, ["@G1", "1", "1", "10", "100", "2", "@LOGS"], lines=("10.0.0.9",))
    assert p.returncode == -signal.SIGSEGV


def test_info_lines_on_stdout_and_address_pairing(tmp_path):
    """INFO goes to stdout (:303), hostname (address); no "UUID:" line (the
    Windows variant prints none).  The line "10.0.0.10" puts only rank 1 in
    group 1; mpi_perf.c's prefix rule would put both ranks there."""
    p = run(tmp_path, ["@G1", "1", "1", "10", "100", "2", "@LOGS"], lines=("10.0.0.10",),
            names="10.0.0.1,10.0.0.10")
    assert "UUID:" not in p.stderr
    info = INFO.findall(p.stdout)
    assert [(int(x[1]), int(x[3]), int(x[5]), int(x[6])) for x in info] == [(0, 0, 0, 1), (1, 1, 0, 0)]
    assert info[0][8] == "10.0.0.1" and info[0][10] == "10.0.0.10"
    assert not INFO.search(p.stderr)
    # the same names and file under mpi_perf.c's rule: both in group 1, no peer
    g1 = tmp_path / "group1"
    q = subprocess.run([PERF, "-f", str(g1), "-n", "1", "-p", "1", "-u", "1", "-l", str(tmp_path / "l2")],
                       capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, MPX_PROCESSOR_NAMES="10.0.0.1,10.0.0.10", HIP_VISIBLE_DEVICES=""))
    assert q.returncode == 255 and "has no peer" in q.stderr


def test_names_that_are_not_addresses_match_as_written(tmp_path):
    """Virtual hosts of one node have no address of their own: the name is
    the key (case-insensitive)."""
    p = run(tmp_path, ["@G1", "1", "2", "10", "100", "2", "@LOGS"], lines=("NODE-B",),
            names="node-a,node-a,node-b,node-b")
    info = INFO.findall(p.stdout)
    assert sorted((int(x[1]), int(x[3]), int(x[6])) for x in info) == [(0, 0, 2), (1, 0, 3), (2, 1, 0), (3, 1, 1)]


def test_extension_flags_after_positionals(tmp_path):
    """argv[8..] are ignored by the reference; here they carry -w/-g/-e/...,
    never the reference's own letters."""
    p = run(tmp_path, ["@G1", "1", "1", "10", "100", "2", "@LOGS", "-u", "0"])
    assert p.returncode == 255
    p = run(tmp_path, ["@G1", "1", "1", "10", "100", "2", "@LOGS", "-e", "bogus"])
    assert p.returncode == 255
    p = run(tmp_path, ["@G1", "1", "2", "10", "100", "2", "@LOGS", "-w", "4"],
            names="10.0.0.1,10.0.0.1,10.0.0.2,10.0.0.2")
    assert len(INFO.findall(p.stdout)) == 4


def test_processes_mode_info_per_rank(tmp_path):
    """Under a launcher (one process per rank, the reference's mpiexec model)
    every process prints its own INFO line on stdout; rank 0's options and
    group file reach the others (MPI_Bcast, windows/mpi-perf.cpp:264-274)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    g1 = tmp_path / "group1"
    g1.write_text("10.0.0.2\n")
    ps = []
    for r in range(2):
        env = dict(os.environ, MPX_RANK=str(r), MPX_SIZE="2", MPX_LOCAL_RANK=str(r), MPX_BOOTSTRAP=f"127.0.0.1:{port}",
                   MPX_PROCESSOR_NAMES="10.0.0.1,10.0.0.2", MPX_BOOTSTRAP_TIMEOUT="30", HIP_VISIBLE_DEVICES="")
        # only rank 0 reads the file: the other rank names one that does not exist
        ps.append(subprocess.Popen([WIN, str(g1) if r == 0 else str(tmp_path / "absent"), "1", "1", "10", "100", "2",
                                    str(tmp_path / "logs")], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                   text=True, env=env))
    outs = [p.communicate(timeout=60) for p in ps]
    infos = [INFO.findall(o[0]) for o in outs]
    assert [len(i) for i in infos] == [1, 1], [o[1][-300:] for o in outs]
    assert [(int(i[0][1]), int(i[0][3]), int(i[0][6])) for i in infos] == [(0, 0, 1), (1, 1, 0)]
