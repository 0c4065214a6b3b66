"""BASELINE config 1 on this machine: the compiled reference (oracle/_ref)
under MPICH shared memory, 2 ranks, the survey's sizes and iteration counts
(SURVEY.md §8d cfg1), every mode; median of runs 1..5 of -r 6.
One JSON line per (mode, size).  CPU only."""
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")
SIZES = [1, 8, 64, 512, 4096, 32768, 262144, 1 << 20, 4 << 20]
MODES = {"unidir": ["-u", "1"], "pingpong": [], "nonblocking": ["-x", "1"]}
quick = len(sys.argv) > 1 and sys.argv[1] == "quick"


def iters_for(b):
    return 20000 if b <= 4096 else (5000 if b <= 262144 else 500)


for mode, flag in MODES.items():
    for b in SIZES:
        it = iters_for(b) // (10 if quick else 1)
        tmp = tempfile.mkdtemp()
        try:
            open(os.path.join(tmp, "g1"), "w").write("localhost\n")
            os.mkdir(os.path.join(tmp, "logs"))
            cmd = ["/opt/conda/bin/mpiexec", "-np", "2", "-genv", "PPN", "1", "-genv", "HOST1", "localhost", "-genv",
                   "HOST0", "127.0.0.1", os.path.join(ROOT, "oracle", "ref_wrap.sh"), REF, "-f", "g1", "-n", "1",
                   "-p", "1", "-r", "6", "-i", str(it), "-b", str(b), "-l", "logs"] + flag
            env = dict(os.environ, PPN="1", HOST1="localhost", HOST0="127.0.0.1")
            env.pop("SHIM_OUT", None)
            p = subprocess.run(cmd, cwd=tmp, env=env, capture_output=True, text=True, timeout=600)
            ts = [float(line.split(",")[9]) / 1000 for f in glob.glob(os.path.join(tmp, "logs", "tcp-*"))
                  for line in open(f)]
            t = statistics.median(ts)
            factor = 1 if mode == "unidir" else 2
            print(json.dumps(dict(mode=mode, bytes=b, iters=it, us_per_iter=round(t / it * 1e6, 3),
                                  GBps=round(b * it * factor / t / 1e9, 3), cores=2, rc=p.returncode,
                                  cpus=os.cpu_count())), flush=True)
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
