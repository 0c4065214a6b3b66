"""Where the reference's ranks run decides its host rate.

Round 5's bench.py bound nothing, and the compiled reference's 4 MiB rate
read 8.0 / 42.1 / 22.5 GB/s per pair at N = 2 / 4 / 8 and 13.9-41.9 GB/s
(ping-pong) across boxes.  This tool runs the same reference loops (MPICH
shm, bench.run_reference) under explicit placements, each `REPS` times, and
prints one JSON document: the placement, the cores, and every run's rate.

  unbound        mpiexec's default (what round 5 ran)
  bench          bench.py's binding now: one physical core per rank on one
                 NUMA node (bench.reference_cores), -membind bind:<node>
  smt_siblings   the two ranks on the two hardware threads of one core
  cross_node     one rank on each of two NUMA nodes (no -membind)

Loops: ping-pong 4 MiB x 500 (config 1's GBps_4MiB) and unidir 4 MiB x 500
(cpu_baseline_pairs' per pair, N = 2 and, unbound / bench only, N = 4, 8).
CPU only; about a minute on a GPU box's host.

    python3 tools/ref_placement.py [REPS]
"""
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

B, ITERS, RUNS = 4 << 20, 500, 6


def siblings(c):
    return bench._cpulist(bench._read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") or str(c))


def placements(n):
    pick = bench.reference_cores(n)
    out = {"unbound": []}
    if pick["complete"]:
        out["bench"] = ["-bind-to", "user:" + ",".join(map(str, pick["cores"])), "-membind", f"bind:{pick['numa_node']}"]
    if n == 2 and pick["cores"]:
        sib = [x for x in siblings(pick["cores"][0]) if x in os.sched_getaffinity(0)]
        if len(sib) >= 2:
            out["smt_siblings"] = ["-bind-to", f"user:{sib[0]},{sib[1]}"]
        nodes = sorted(int(os.path.basename(d)[4:]) for d in glob.glob("/sys/devices/system/node/node[0-9]*"))
        if len(nodes) >= 2:
            a = bench.reference_cores(1)["cores"]
            other = [c for c in bench._cpulist(bench._read(f"/sys/devices/system/node/node{nodes[1]}/cpulist"))
                     if c in os.sched_getaffinity(0)]
            if a and other:
                out["cross_node"] = ["-bind-to", f"user:{a[0]},{other[0]}"]
    return out


def rates(n, args, place, pingpong):
    r = bench.run_reference(n, n // 2, args, 300, placement=place)
    if r["rc"] != 0:
        return dict(error=f"rc {r['rc']}: {r['stderr'][-200:]}")
    per_run = {}
    for k, t in r["times"]:
        per_run.setdefault(k, []).append(t)
    ts = [max(v) for _, v in sorted(per_run.items()) if len(v) == n // 2]
    f = 2 if pingpong else 1     # the reference's own formula per loop (mpi_perf.c:535-542)
    g = [round(f * B * ITERS / t / 1e9, 3) for t in ts]
    return dict(GBps_per_run=g, median=statistics.median(g), leftover=r["leftover"])


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    out = dict(tool="tools/ref_placement.py", affinity_cpus=len(os.sched_getaffinity(0)),
               numa_nodes=len(glob.glob("/sys/devices/system/node/node[0-9]*")), bytes=B, iters=ITERS, cases={})
    loops = [("pingpong", 2, ["-b", str(B), "-i", str(ITERS), "-r", str(RUNS)], True)]
    loops += [(f"unidir_n{n}", n, ["-u", "1", "-b", str(B), "-i", str(ITERS), "-r", str(RUNS)], False)
              for n in (2, 4, 8)]
    for name, n, args, pp in loops:
        for pname, place in placements(n).items():
            if n > 2 and pname not in ("unbound", "bench"):
                continue
            reps_out = [rates(n, args, place, pp) for _ in range(reps)]
            meds = [x["median"] for x in reps_out if "median" in x]
            out["cases"][f"{name}/{pname}"] = dict(binding=" ".join(place) or "none", reps=reps_out,
                                                  median_of_medians=statistics.median(meds) if meds else None,
                                                  spread=[min(meds), max(meds)] if meds else None)
            print(f"[ref_placement] {name}/{pname}: {meds}", file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
