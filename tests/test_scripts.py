"""scripts/run-gpu-pair.sh and scripts/run-gpu-rounds.sh, the MI355X
counterparts of the reference's launchers scripts/run-1-pair.sh (one pair,
-x 1, 4 MiB, 5000 iterations, 10 runs) and scripts/run-hbv3.sh (concurrent
unidirectional flows, 456131 B, 10 iterations, runs forever).

CPU: the launch shape, through mpx_perf's GPU-free `-d 1` mode (pairing,
rounds, flags).  GPU (-m gpu): short runs with every rank on GPU 0 and every
payload checked, records in the log folder."""
import glob
import os
import re

import pytest

from proc import run_bounded

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAIR = os.path.join(ROOT, "scripts", "run-gpu-pair.sh")
ROUNDS = os.path.join(ROOT, "scripts", "run-gpu-rounds.sh")
INFO = re.compile(r"INFO: (\S+), rank (\d+) out of (\d+) ranks, my_group: (\d), group_size: (\d+), "
                  r"group_rank: (\d+), my_peer: (-?\d+)")


def run(script, tmp_path, env, *args, timeout=90):
    # MPX_DEBUG: libmpx traces its teardown, so a run that stalls at exit says so
    e = dict(os.environ, MPX_PROCESSOR_NAMES="", MPX_HOSTNAME="node", LOGFOLDER=str(tmp_path / "logs"), MPX_DEBUG="1")
    e.update(env)
    return run_bounded(["bash", script, *args], timeout=timeout, env=e, cwd=tmp_path)


def records(tmp_path):
    out = []
    for f in sorted(glob.glob(str(tmp_path / "logs" / "tcp-*.log"))):
        out += [line.rstrip("\n").split(",") for line in open(f)]
    return out


def test_pair_script_launch_shape(tmp_path):
    p = run(PAIR, tmp_path, {"RUNS": "3", "ITERS": "5"}, "-d", "1")
    assert p.returncode == 0, p.stderr[-600:]
    info = sorted((x[0], int(x[1]), int(x[3]), int(x[6])) for x in INFO.findall(p.stderr))
    assert info == [("node-0", 0, 1, 1), ("node-1", 1, 0, 0)]
    # -x 1 (non-blocking), the reference's run-1-pair.sh sizes, FLOWS = 1
    assert len(re.findall(r"^dotnet .* server .* 4194304 5 ", p.stderr, re.M)) == 3


def test_pair_script_flows(tmp_path):
    p = run(PAIR, tmp_path, {"RUNS": "1", "FLOWS": "3", "GPUS": "0,1,2,3,4,5"}, "-d", "1")
    assert p.returncode == 0, p.stderr[-600:]
    peers = sorted((int(x[1]), int(x[6])) for x in INFO.findall(p.stderr))
    assert peers == [(0, 3), (1, 4), (2, 5), (3, 0), (4, 1), (5, 2)]      # --map-by ppr:3:node


def test_rounds_script_covers_every_pair(tmp_path):
    p = run(ROUNDS, tmp_path, {"RUNS": "7", "ITERS": "1"}, "-d", "1")
    assert p.returncode == 0, p.stderr[-600:]
    rounds = re.findall(r"^ROUND (\d+): (.*)$", p.stderr, re.M)
    assert len(rounds) == 7
    pairs = [tuple(sorted(map(int, m))) for _, body in rounds for m in re.findall(r"\((\d+),(\d+)\)", body)]
    assert len(pairs) == 28 and len(set(pairs)) == 28


def test_rounds_script_fixed_pairs(tmp_path):
    p = run(ROUNDS, tmp_path, {"RUNS": "1", "ALL_PAIRS": "0"}, "-d", "1")
    assert p.returncode == 0, p.stderr[-600:]
    peers = sorted((int(x[1]), int(x[6])) for x in INFO.findall(p.stderr))
    assert peers == [(k, (k + 4) % 8) for k in range(8)]


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["kernel", "sdma"])
def test_pair_script_on_gpu(tmp_path, engine):
    p = run(PAIR, tmp_path, {"RUNS": "3", "ITERS": "300", "BUFF_SZ": "65536", "GPUS": "0,0", "ENGINE": engine},
            "-c", "1", "-t", "5000")
    assert p.returncode == 0, p.stderr[-600:]
    recs = records(tmp_path)
    assert [(int(f[2]), int(f[7]), int(f[8]), int(f[10])) for f in recs] == [(0, 65536, 300, 1), (0, 65536, 300, 2)]


@pytest.mark.gpu
def test_rounds_script_on_gpu(tmp_path):
    """7 runs = the 7 rounds, 4 concurrent pairs each, all eight ranks on GPU
    0, every payload checked; 6 recorded runs x 4 senders."""
    p = run(ROUNDS, tmp_path, {"RUNS": "7", "ITERS": "10", "GPUS": "0,0,0,0,0,0,0,0"}, "-c", "1", "-t", "5000")
    assert p.returncode == 0, p.stderr[-600:]
    recs = records(tmp_path)
    assert len(recs) == 6 * 4
    assert {int(f[7]) for f in recs} == {456131} and {int(f[8]) for f in recs} == {10}
