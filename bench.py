#!/usr/bin/env python3
"""bench.py — the driver's benchmark of mpi_perf's hot path on MI355X.

    python bench.py [--gpus N --steps K --warmup W]          (N = 1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

A "step" is one run of the reference's loop (mpi_perf.c:474-569: barrier ->
`iters` x transfer -> barrier) over one batch of synthetic bytes:

* N = 1 — BASELINE config 2, the 1-GPU local device-to-device copy: each step
  is `iters` launches of the HBM copy kernel moving B = 1 GiB tx -> rx (the
  loop's degenerate pair, both ends on one GPU).  value = B*iters*K / T.
  After the timed steps: config 2's sweep (1 B .. 1 GiB), the same copy held
  for 10 s (sustained rate), loopback pair latency / rate, the runtime's copy.
* N >= 2 — BASELINE config 4, all-pairs concurrent rounds (run-hbv3-style,
  unidirectional): step s runs round s mod (N-1) of the circle-method
  schedule; each of the N/2 pairs moves `iters` x 4 MiB G1 -> G0 over xGMI
  with the 1-byte ack (mpi_perf.c:127-145).  value = sum of bytes over all
  pairs / T, with T the max over ranks (weak scaling: every GPU is in one
  pair per step).  Before the timed steps every round is validated once
  (check mode, seeded payloads, a barrier per round) and the bulk push
  variant (workgroups per push x streaming store hint) is tuned on round 0's
  links.  After them come the per-pair table of every covered pair, a
  checked small-message ping-pong on every link, the 8 B latency (10^5
  ping-pong iterations on round 0, 10^4 on every pair), config 3's pair
  sweep, run-hbv3's 456131 B x 10 rounds, the same rounds at 64 MiB (the
  link rate with the per-iteration protocol cost amortised away: the
  reference point of the 4 MiB headline), and the SDMA and RCCL comparison
  engines under a watchdog.  A kernel-engine failure before or inside the
  timed steps falls back to SDMA (labelled); a failure after them nulls only
  its own numbers.

Rank 0 prints one JSON line, and it is the only thing on stdout (library
output on fd 1 is routed to stderr).  `roofline` is computed for the dominant kernel
from HIP-event time measured inside this process (libmpx records the events
on the stream it launches on); `cpu_baseline` times the compiled reference
(oracle/_ref, under MPICH shared memory) or, if absent, the oracle's CPU port.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
from mpx.schedule import all_pairs_rounds, round_role  # noqa: E402  (pure Python, no GPU)

HBM_PEAK_GBPS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# xGMI: BASELINE.json quotes ~153 GB/s per link.  Read here as the link's
# two directions summed (AMD's datasheet convention, from memory: 153.6 GB/s
# per link, 7 links; x16 at 38.4 Gb/s per lane = 76.8 GB/s each way — not
# verifiable offline).  A unidirectional pair uses one
# direction of its one link, so 76.8 is its roofline; the fraction against
# 153.6 is reported beside it, and the targets carry both verdicts.
XGMI_LINK_PEAK_BIDIR_GBPS = 153.6
XGMI_LINK_PEAK_GBPS = XGMI_LINK_PEAK_BIDIR_GBPS / 2
# north_star's targets (BASELINE.json): per-pair unidirectional bandwidth
# >= 85 % of xGMI link peak at >= 4 MB, device-initiated 8 B latency < 3 us
TARGET_LINK_FRAC, TARGET_HALF_RTT_US = 0.85, 3.0
# The bar as SURVEY/BASELINE state it: ~153 GB/s per link PER DIRECTION
# (SURVEY.md:361; BASELINE.md:51 "~130 of ~153 GB/s") — the primary verdict.
STATED_LINK_PEAK_GBPS = XGMI_LINK_PEAK_BIDIR_GBPS


def link_target(achieved: float, nbytes: int) -> dict:
    """extras.targets.per_pair_unidir_GBps: `meets` is judged against the
    stated bar (0.85 x 153.6 GB/s per direction, SURVEY.md:361); the
    per-direction reading of 153.6 as two directions summed (0.85 x 76.8,
    DESIGN.md §7, from memory) goes beside it as `meets_per_direction_reading`,
    unsourced until a node measurement settles which reading is the link."""
    return dict(value=round(achieved, 2), bytes=nbytes,
                target=f">= {TARGET_LINK_FRAC} x {STATED_LINK_PEAK_GBPS} GB/s per direction of one link "
                       f"(SURVEY.md:361, BASELINE.md:51)",
                meets=achieved >= TARGET_LINK_FRAC * STATED_LINK_PEAK_GBPS,
                per_direction_reading=f">= {TARGET_LINK_FRAC} x {XGMI_LINK_PEAK_GBPS} GB/s: 153.6 read as both "
                                      f"directions summed (DESIGN.md §7; unsourced, from memory, until a node run "
                                      f"measures the link)",
                meets_per_direction_reading=achieved >= TARGET_LINK_FRAC * XGMI_LINK_PEAK_GBPS)
EXTRAS_DEADLINE_S = 150      # 64 MiB rounds + comparison engines at N > 1 (see main)
CEILING_BYTES, CEILING_ITERS = 64 << 20, 20   # extras: the kernel engine at 64 MiB (see main)


# N = 1 baseline: 1 GiB x 40 per run (bound ranks move ~24 GB/s: ~1.7 s a run)
CPU_BASELINE_ITERS = 40
# every reference leg of one bench run ends by this time.monotonic() (set in
# main): at N >= 2 the other ranks wait in the process-group init meanwhile
# (its 180 s timeout), so the legs together must end well inside it
REF_BUDGET_S = 120.0
_ref_deadline = [None]
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "mpi_perf")
REF_SHIM = os.path.join(ROOT, "oracle", "_ref", "libshim.so")
MPIEXEC = "/opt/conda/bin/mpiexec"
MPICH = "MPICH 3.3.2 shm"
PROFILER_ENV = ("ROCP_TOOL_LIBRARIES", "ROCPROF_COUNTERS", "ROCPROFILER_LIBRARY_CTOR")


def under_profiler() -> str | None:
    """The profiler variable set in this process's environment, if any."""
    return next((k for k in PROFILER_ENV if os.environ.get(k)), None)


def reference_available() -> bool:
    return all(os.path.exists(x) for x in (REF_BIN, REF_SHIM, MPIEXEC))


def _cpulist(text: str) -> list[int]:
    out = []
    for part in text.strip().split(","):
        if part:
            lo, _, hi = part.partition("-")
            out += range(int(lo), int(hi or lo) + 1)
    return out


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return ""


def reference_cores(nranks: int, sysfs: str = "/sys/devices/system") -> dict:
    """The host cores the reference's ranks are bound to, chosen the way its
    launchers choose them: one NUMA node
    (`numactl --cpunodebind=0 --membind 0`, scripts/run-1-pair.sh:62), one
    rank per physical core in order (`--bind-to cpulist:ordered --cpu-list
    8..17`, scripts/run-hbv3.sh:23).  Node 0 when it has nranks allowed
    physical cores (else the node with the most); one hardware thread per
    core (the lowest sibling); the first 8 cores of the node skipped when it
    has 8 + nranks of them (run-hbv3's list starts at 8), else from its first.
    Only CPUs in this process's affinity mask are used."""
    allowed = set(os.sched_getaffinity(0))
    nodes = {}
    for d in sorted(glob.glob(os.path.join(sysfs, "node", "node[0-9]*"))):
        cpus = [c for c in _cpulist(_read(os.path.join(d, "cpulist"))) if c in allowed]
        nodes[int(os.path.basename(d)[4:])] = cpus
    if not nodes:
        nodes = {0: sorted(allowed)}
    phys = {}
    for n, cpus in nodes.items():
        seen, cores = set(), []
        for c in cpus:
            sib = _cpulist(_read(os.path.join(sysfs, "cpu", f"cpu{c}", "topology", "thread_siblings_list")) or str(c))
            first = min(sib)
            if first not in seen and first in allowed:
                seen.add(first)
                cores.append(first)
        phys[n] = cores
    node = 0 if len(phys.get(0, [])) >= nranks else max(phys, key=lambda k: len(phys[k]))
    cores = phys[node]
    skip = 8 if len(cores) >= 8 + nranks else 0
    chosen = cores[skip:skip + nranks]
    return dict(cores=chosen, numa_node=node, node_physical_cores=len(cores), skipped_first=skip,
                complete=len(chosen) == nranks)


def _procs() -> dict:
    """Every live process from /proc: pid -> pid, ppid, name, state, start
    (the start time in clock ticks after boot: with the pid it names one
    process, whatever pids are reused later)."""
    procs = {}
    for d in glob.glob("/proc/[0-9]*"):
        st = _read(os.path.join(d, "stat"))
        if not st or ")" not in st:
            continue
        f = st[st.rindex(")") + 2:].split()
        pid = int(os.path.basename(d))
        procs[pid] = dict(pid=pid, ppid=int(f[1]), state=f[0], start=int(f[19]),
                          name=st[st.index("(") + 1:st.rindex(")")])
    return procs


def descendants(root: int | None = None, procs: dict | None = None) -> list[dict]:
    """Every live process below `root` (default: this one) in the parent
    tree, from /proc: pid, ppid, name, state, start (bench.py's exit census;
    zombies not yet reaped by their parent are listed too)."""
    root = os.getpid() if root is None else root
    procs = _procs() if procs is None else procs
    out, frontier = [], {root}
    while frontier:
        kids = [q for q in procs.values() if q["ppid"] in frontier and q["pid"] != root]
        out += kids
        frontier = {q["pid"] for q in kids}
    return out


def run_tracked(cmd: list[str], timeout: float, **popen_kw) -> dict:
    """Run cmd to its end (or `timeout`), tracking every process below it.
    MPICH's hydra puts each proxy and each rank in a session of its own
    (setsid), so neither a process group nor a session can find them once
    mpiexec is gone: their pids (with start times) are collected from the
    parent tree while it runs, every 0.25 s.  When cmd returns, any of them
    still alive (same pid and start time, not a zombie) is named in
    `leftover` and killed.  stdout / stderr go to
    files, so no descendant can hold a pipe open."""
    import signal
    seen = {}
    with tempfile.TemporaryFile("w+") as fo, tempfile.TemporaryFile("w+") as fe:
        p = subprocess.Popen(cmd, stdout=fo, stderr=fe, text=True, start_new_session=True, **popen_kw)
        deadline, timed_out = time.monotonic() + timeout, False
        while p.poll() is None:
            for q in descendants(p.pid):
                seen[q["pid"]] = q
            if time.monotonic() > deadline:
                timed_out = True
                break
            time.sleep(0.25)
        def alive(now):
            # the same process (pid and start time: a reused pid is not it), not a zombie
            return [q for q in seen.values()
                    if q["pid"] in now and now[q["pid"]]["start"] == q["start"] and now[q["pid"]]["state"] != "Z"]

        def kill(qs):
            for q in qs:
                try:
                    os.kill(q["pid"], signal.SIGKILL)
                except (ProcessLookupError, PermissionError):
                    pass

        if timed_out:
            for q in descendants(p.pid):
                seen[q["pid"]] = q
            p.kill()
            kill(alive(_procs()))
            t_end = time.monotonic() + 2.0     # SIGKILL lands asynchronously
            while alive(_procs()) and time.monotonic() < t_end:
                time.sleep(0.02)
        p.wait()
        left = [dict(pid=q["pid"], name=q["name"]) for q in alive(_procs())]
        kill(left)
        if left:
            print(f"[bench] {os.path.basename(cmd[0])} left {left} alive: killed", file=sys.stderr)
        fo.seek(0)
        fe.seek(0)
        out, err = fo.read(), fe.read()
    if timed_out:
        err = f"timed out after {timeout} s; " + err
    return dict(rc=p.returncode, stdout=out, stderr=err, leftover=left, tracked=len(seen), timed_out=timed_out)


def run_reference(nranks: int, ppn: int, args: list[str], timeout: float, placement: list[str] | None = None) -> dict:
    """One mpiexec run of the compiled reference (oracle/_ref) under MPICH
    shared memory, its ranks bound like its launchers bind them
    (reference_cores: `-bind-to user:<cores>`, `-membind bind:<node>`).
    Every process below mpiexec is tracked (run_tracked): none outlives the
    leg (the reference itself finalizes cleanly, mpi_perf.c:579-581).  This
    process keeps off the ranks' cores meanwhile (its own affinity without
    them), so its polling never preempts a rank.  Returns rc, stderr tail,
    the records' (run, time_s) pairs, binding, leftover.
    `placement` (tools/ref_placement.py) replaces the binding arguments:
    one form, tried once ([] = mpiexec's default placement)."""
    pick = reference_cores(nranks)
    tmp = tempfile.mkdtemp(prefix="cpu_base_")
    out = dict(rc=None, stderr="", times=[], leftover=[], binding=None, cores=pick["cores"],
               numa_node=pick["numa_node"], tracked=0)
    mask = os.sched_getaffinity(0)
    try:
        if pick["complete"] and mask - set(pick["cores"]):
            os.sched_setaffinity(0, mask - set(pick["cores"]))
        with open(os.path.join(tmp, "group1"), "w") as f:
            f.write("localhost\n")
        os.mkdir(os.path.join(tmp, "logs"))
        env = dict(os.environ)
        env.pop("SHIM_OUT", None)
        tail = ["-genv", "PPN", str(ppn), "-genv", "HOST1", "localhost", "-genv", "HOST0", "127.0.0.1",
                os.path.join(ROOT, "oracle", "ref_wrap.sh"), REF_BIN, "-f", "group1", "-n", "1", "-p", str(ppn)] + args \
            + ["-l", "logs"]
        forms = [["-bind-to", "user:" + ",".join(map(str, pick["cores"])), "-membind", f"bind:{pick['numa_node']}"],
                 ["-bind-to", "user:" + ",".join(map(str, pick["cores"]))], []] if pick["complete"] else [[]]
        if placement is not None:
            forms = [placement]
        for form in forms:
            for x in glob.glob(os.path.join(tmp, "logs", "*")):
                os.remove(x)
            left_s = timeout if _ref_deadline[0] is None else _ref_deadline[0] - time.monotonic()
            if left_s < 2:
                out["rc"], out["stderr"] = None, f"not run: the reference legs' {REF_BUDGET_S:.0f} s budget is spent"
                break
            r = run_tracked([MPIEXEC, "-np", str(nranks)] + form + tail, min(timeout, left_s), cwd=tmp, env=env)
            out["leftover"] += r["leftover"]
            out["tracked"] = max(out["tracked"], r["tracked"])
            out["rc"], out["stderr"] = r["rc"], r["stderr"][-400:]
            out["binding"] = " ".join(form) if form else "none (mpiexec's default placement)"
            if r["rc"] == 0 or r["timed_out"]:   # a run that hung is not retried in another form
                break
        for path in glob.glob(os.path.join(tmp, "logs", "tcp-*.log")):
            for line in open(path):
                f = line.strip().split(",")
                out["times"].append((int(f[10]), float(f[9]) / 1000.0))
    finally:
        os.sched_setaffinity(0, mask)
        shutil.rmtree(tmp, ignore_errors=True)
    if placement is not None:
        out["cores"] = None   # the caller's placement, named by `binding`
    elif not out["cores"] or not out["binding"] or out["binding"].startswith("none"):
        out["cores"] = None
    return out


def _spread(rates: list[float]) -> dict:
    return dict(min=round(min(rates), 3), median=round(statistics.median(rates), 3), max=round(max(rates), 3),
                runs=len(rates))


def _placement(r: dict) -> dict:
    return dict(core_list=r["cores"], numa_node=r["numa_node"], binding=r["binding"], leftover_processes=r["leftover"],
                processes_tracked=r["tracked"])


def cpu_baseline(nbytes: int, iters: int, runs: int) -> dict | None:
    """Time the reference on the host: 2 ranks, unidirectional, B bytes;
    each run's rate (runs 1..runs-1; run 0 is the reference's warm-up, never
    recorded) and their min / median / max."""
    sample = f"-u 1 -b {nbytes} -i {iters} -r {runs}, 2 ranks, runs 1..{runs - 1} (run 0 is the reference's warm-up)"
    if reference_available():
        try:
            r = run_reference(2, 1, ["-u", "1", "-b", str(nbytes), "-i", str(iters), "-r", str(runs)], 300)
            times = [t for _, t in r["times"]]
            if r["rc"] == 0 and times:
                t = statistics.median(times)
                return dict(value=round(nbytes * iters / t / 1e9, 3), unit="GB/s", cores=2, kind="reference",
                            sample=f"mpi_perf.c (oracle/_ref) under {MPICH}, " + sample, median_run_s=t,
                            GBps_per_run=_spread([nbytes * iters / x / 1e9 for x in times]), **_placement(r))
            print(f"[bench] reference baseline failed rc={r['rc']}: {r['stderr']}", file=sys.stderr)
        except Exception as e:  # noqa: BLE001
            print(f"[bench] reference baseline unavailable: {e}", file=sys.stderr)
    port = os.path.join(ROOT, "oracle", "oracle_perf")
    if os.path.exists(port):
        p = subprocess.run([port, "-p", "1", "-u", "1", "-b", str(nbytes), "-i", str(iters), "-r", str(runs)],
                           capture_output=True, text=True, timeout=300, env=dict(os.environ, ORACLE_NO_DIGEST="1"))
        rows = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")][1:]
        if rows:
            t = statistics.median(r["max_time_s"] for r in rows)
            return dict(value=round(nbytes * iters / t / 1e9, 3), unit="GB/s", cores=2, kind="port",
                        sample="oracle/oracle_perf (C restatement, 2 threads), " + sample, median_run_s=t)
    return None


def cpu_baseline_pingpong(runs: int = 6) -> dict | None:
    """BASELINE config 1 on the box's own host cores:
    the compiled reference's 2-rank ping-pong (mpi_perf.c:66-83, the default
    loop) under MPICH shm at 8 B (-i 20000) and 4 MiB (-i 500), SURVEY
    §8(d) cfg1's iterations, -r runs; median of runs 1..runs-1 (run 0 is the
    reference's warm-up), with each run's min / max beside it.
    half_rtt_us_8B = time / (2 x iters); GBps_4MiB = 2 x B x iters / time,
    the reference's own formula for this loop (mpi_perf.c:535-542, both
    directions).  ~5 s on the box, before any GPU call."""
    if not reference_available():
        return None
    out = dict(cores=2, kind="reference", loop="ping-pong (mpi_perf.c:66-83)",
               sample=f"mpi_perf.c (oracle/_ref) under {MPICH}, 2 ranks, -b 8 -i 20000 and -b 4194304 "
                      f"-i 500, -r {runs}, median of runs 1..{runs - 1}")
    for nbytes, iters, key in ((8, 20000, "half_rtt_us_8B"), (4 << 20, 500, "GBps_4MiB")):
        try:
            r = run_reference(2, 1, ["-b", str(nbytes), "-i", str(iters), "-r", str(runs)], 120)
            times = [t for _, t in r["times"]]
            if r["rc"] != 0 or not times:
                out[key] = None
                out[key + "_error"] = f"rc {r['rc']}: {r['stderr'][-200:]}"
                continue
            vals = [x / (2 * iters) * 1e6 if nbytes == 8 else 2 * nbytes * iters / x / 1e9 for x in times]
            out[key] = round(statistics.median(vals), 3)
            out[key + "_per_run"] = _spread(vals)
            out.update(_placement(r))
        except Exception as e:  # noqa: BLE001
            out[key] = None
            out[key + "_error"] = f"{type(e).__name__}: {e}"[:200]
    return out


def cpu_baseline_pairs(world: int, nbytes: int, iters: int, runs: int) -> dict | None:
    """The reference itself on the host beside the N >= 2 line: run-hbv3's
    layout (scripts/run-hbv3.sh:22,28: N ranks, ppn = N/2 flows, -u 1) at the
    headline's B and iterations, under MPICH shared memory — N/2 concurrent
    pairs, each a reference process pair on the box's host cores, one bound
    core per rank (reference_cores).  A run's aggregate is the pairs' bytes /
    the slowest sender's time (only group 1 writes records,
    mpi_perf.c:545-554; its time covers its peer's last ack), the reference's
    implied all-pairs figure; median over runs 1..runs-1 (run 0 is the
    reference's own warm-up, never recorded), min / max beside it.  Runs on
    rank 0 before any GPU call."""
    if not reference_available():
        return None
    ppn = world // 2
    try:
        r = run_reference(world, ppn, ["-u", "1", "-b", str(nbytes), "-i", str(iters), "-r", str(runs)], 300)
        per_run = {}
        for k, t in r["times"]:
            per_run.setdefault(k, []).append(t)
        runs_ok = [max(v) for _, v in sorted(per_run.items()) if len(v) == ppn]
        if r["rc"] != 0 or not runs_ok:
            print(f"[bench] reference pairs baseline failed rc={r['rc']}: {r['stderr']}", file=sys.stderr)
            return None
        t = statistics.median(runs_ok)
        return dict(value=round(ppn * nbytes * iters / t / 1e9, 3), unit="GB/s", cores=world, kind="reference",
                    sample=f"mpi_perf.c (oracle/_ref) under {MPICH}, run-hbv3 layout: {world} ranks, "
                           f"-p {ppn} -u 1 -b {nbytes} -i {iters} -r {runs} ({ppn} concurrent pairs, one bound core "
                           f"per rank); aggregate = {ppn} x B x iters / the slowest sender's time per run, median of "
                           f"runs 1..{runs - 1}",
                    per_pair_GBps=round(nbytes * iters / t / 1e9, 3), median_run_s=t,
                    per_pair_GBps_per_run=_spread([nbytes * iters / x / 1e9 for x in runs_ok]), **_placement(r))
    except Exception as e:  # noqa: BLE001
        print(f"[bench] reference pairs baseline unavailable: {e}", file=sys.stderr)
        return None


def traffic_from_profile(workload: str) -> dict | None:
    """Per-launch HBM bytes from the committed PMC summary of this workload
    (profiles/pmc_<workload>.json, written by tools/pmc_summary.py from
    rocprofv3 --pmc passes, corrected per MI355X_MICROARCH.md §HBM)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def counters_skip_reason(args) -> str | None:
    """None when the in-process counters may run; else why not.  A process
    that rocprofv3 already profiles has its own rocprofiler tool (and
    dispatch counting serialises kernels): no second one is added."""
    if args.no_counters:
        return "--no-counters"
    k = under_profiler()
    if k:
        return f"not sampled in-process: the process runs under a profiler ({k} set)"
    return None


COUNTER_STEPS = 3   # untimed re-run of the headline's steps per counter pass (30 launches of 1 GiB)


def copy_traffic(prof, c, src, dst, nbytes: int, iters: int, bus: str) -> dict:
    """HBM bytes per k_copy launch from this process's own counters: the
    headline's step re-run COUNTER_STEPS times, untimed, inside a
    FETCH_SIZE pass and again inside a WRITE_SIZE pass (they cannot share one:
    TCC has 4 slots, FETCH_SIZE uses 3 and WRITE_SIZE 2, MI355X_MICROARCH.md
    "PMC slots"); FETCH_SIZE x 2 per the guide's HBM section (gfx950 tallies
    128-B reads at 64 B), both in KiB."""
    vals, launches, reset = {}, {}, None
    for name in ("FETCH_SIZE", "WRITE_SIZE"):
        n = 0
        with prof.Pass(bus, [name]) as p:
            for _ in range(COUNTER_STEPS):
                n += c.copy(0, dst, src, nbytes, iters).launches
        vals[name], launches[name], reset = p.values[0], n, p.reads_reset
    rd = vals["FETCH_SIZE"] * 1024 * 2 / launches["FETCH_SIZE"]
    wr = vals["WRITE_SIZE"] * 1024 / launches["WRITE_SIZE"]
    return dict(hbm_read_bytes_per_launch=round(rd, 1), hbm_write_bytes_per_launch=round(wr, 1),
                hbm_bytes_per_launch=round(rd + wr, 1), traffic_over_algorithmic=round((rd + wr) / (2 * nbytes), 5),
                launches_per_pass=launches["FETCH_SIZE"], fetch_size_kib=vals["FETCH_SIZE"],
                write_size_kib=vals["WRITE_SIZE"], reads_reset=reset,
                source=f"in-process rocprofiler-sdk device counting service (mpi-perf_amd/lib/libmpxprof.so): "
                       f"FETCH_SIZE x 2 + WRITE_SIZE, separate passes, each over {launches['FETCH_SIZE']} untimed "
                       f"k_copy launches of this run (the headline's step, {COUNTER_STEPS} times)")


def copy_sweep(mpx, c, src, dst, nbytes: int) -> dict:
    """BASELINE config 2's sweep beside the headline: B = 2^k for 1 B ..
    nbytes.  Each size: one mpx_copy call of 10 copies (3 at >= 256 MiB)
    timed with HIP events on the copy's stream, best of 5 such calls; per
    copy = call time / copies.  Up to 16 MiB the call is ONE launch (all
    copies, a grid barrier between them: k_copy_steps to 512 KiB, k_copy_pipe
    above), above it one k_copy launch per copy ("path").  `hbm_GBps` counts 2B per copy; `frac` is that
    over the 8 TB/s HBM peak — below ~256 MiB a repeated copy of the same
    buffer is served from the 4 MB-per-XCD L2 / 256 MB Infinity Cache, not
    HBM, and the small sizes are bound by the barrier or the dispatch, not by
    bytes.  The output of the last size is checked."""
    best = {}
    for _ in range(2):   # two passes over the sizes: a clock transition mid-pass costs one pass only
        b = 1
        while b <= nbytes:
            copies = 10 if b < (256 << 20) else 3
            c.copy(0, dst, src, b, 2)   # warm: first launches of this grid size
            for _ in range(5):
                t = c.copy(0, dst, src, b, copies)
                per = t.device_s / copies
                if b not in best or per < best[b][0]:
                    best[b] = (per, mpx.PROTOCOLS.get(t.protocol, t.protocol))
            b *= 2
    out = {str(k): dict(us=round(v * 1e6, 3), hbm_GBps=round(2 * k / v / 1e9, 1),
                        frac=round(2 * k / v / 1e9 / HBM_PEAK_GBPS, 4), path=p,
                        cache="L2" if k <= (16 << 20) else "MALL" if k <= (128 << 20) else "HBM")
           for k, (v, p) in sorted(best.items())}
    assert c.checksum(dst, b // 2) == c.checksum(src, b // 2), "copy sweep output differs from its input"
    return out


def sustained_copy(c, src, dst, nbytes: int, seconds: float = 10.0) -> dict:
    """The headline copy held for `seconds` of back-to-back launches (calls of
    300 copies, ~0.1 s each at 1 GiB): whether the rate of the short timed
    region holds once clocks and temperature settle.  HBM traffic (2B per
    copy) per call from HIP events; the output is checked at the end."""
    rates, t_end = [], time.perf_counter() + seconds
    while time.perf_counter() < t_end:
        t = c.copy(0, dst, src, nbytes, 300)
        rates.append(2 * nbytes * 300 / t.device_s / 1e9)
    assert c.checksum(dst, nbytes) == c.checksum(src, nbytes), "sustained copy output differs from its input"
    return dict(seconds=seconds, calls=len(rates), copies=300 * len(rates),
                hbm_GBps_median=round(statistics.median(rates), 1), hbm_GBps_min=round(min(rates), 1),
                hbm_GBps_max=round(max(rates), 1), hbm_GBps_last=round(rates[-1], 1),
                frac_median=round(statistics.median(rates) / HBM_PEAK_GBPS, 4))


def hbm_one_direction_ceiling() -> dict | None:
    """Read-only and write-only HBM rates of k_copy's access shape (one 16-B
    nontemporal unit per lane, one step per workgroup), measured by
    tools/copy_lab into profiles/r01_copy_lab_read_write_ceilings.jsonl: what
    HBM delivers in one direction on this part, beside the 8 TB/s spec."""
    path = os.path.join(ROOT, "profiles", "r01_copy_lab_read_write_ceilings.jsonl")
    if not os.path.exists(path):
        return None
    best = {}
    with open(path) as f:
        for line in f:
            d = json.loads(line)
            for key, tag in (("read", "R_read_only"), ("write", "W_write_only")):
                if d["variant"].startswith(tag):   # the lab's column counts 2B per launch
                    best[key] = max(best.get(key, 0.0), round(d["hbm_GBps_best"] / 2, 1))
    return dict(best, source="profiles/r01_copy_lab_read_write_ceilings.jsonl") if best else None


def runtime_copy_rate(torch, nbytes: int, iters: int) -> float:
    """The HIP runtime's own device-to-device copy (torch's copy_ ->
    hipMemcpyAsync) of the same B, for comparison with k_copy: HBM traffic
    (2B per copy) / average time per copy, HIP events on torch's stream."""
    a = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    a.fill_(7)
    b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    per = e0.elapsed_time(e1) * 1e-3 / iters
    del a, b
    torch.cuda.empty_cache()
    return round(2 * nbytes / per / 1e9, 1)


def loopback_pair(mpx, engine: str, mode: int, nbytes: int, iters: int, runs: int = 3, pull: bool = False) -> dict:
    """Two ranks on GPU 0 (one host thread each): per-pair time of the loop
    (pull: the kernel engine's MPX_XFER_PULL form)."""
    with mpx.Context(2, engine) as c:
        bufs = []
        for r in range(2):
            tx, rx = c.alloc(0, max(nbytes, 1)), c.alloc(0, max(nbytes, 1))
            c.fill(tx, nbytes, mpx.FILL_BYTE, ord("b") if r == 0 else ord("a"))
            c.attach(r, 0, tx, rx, nbytes)
            bufs.append((tx, rx))
        res = []
        for _ in range(runs + 1):
            out = {}

            def side(r):
                out[r] = c.xfer(mode, 1 - r, r, 1 - r, iters, bufs[r][0], bufs[r][1], nbytes, pull=pull)

            th = [threading.Thread(target=side, args=(r,)) for r in range(2)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            res.append(max(out[0].wall_s, out[1].wall_s))
        return dict(median_s=statistics.median(res[1:]), per_iter_us=statistics.median(res[1:]) / iters * 1e6)


POST_TIMEOUT_MS = 2000


def start_after_barrier(dist, c, *xfer_args, **xfer_kw):
    """The barrier in front of a timed loop (mpi_perf.c:499), then the
    transfer.  With the spin barrier (SpinBarrierDist) both happen in one C
    call (mpxb_spin_wait_xfer): an armed call starts as the barrier opens,
    with no Python between them — several microseconds that differ from rank
    to rank and showed up as the sender's wait for its peer's start (the
    posted wait).  Otherwise dist.barrier(), then the call."""
    spin = getattr(dist, "spin", None)
    if spin is not None:
        return c.xfer(*xfer_args, after=spin, **xfer_kw)
    dist.barrier()
    return c.xfer(*xfer_args, **xfer_kw)


def safe_wall(c, errs: list, *xfer_args, barrier=None, **xfer_kw) -> float:
    """Wall time of one transfer measured after the headline (latency,
    sweeps); a failure there (a device deadline, a refused transfer, a
    payload checksum mismatch) is recorded in `errs` and returns +inf, so
    this rank still takes part in every collective that follows and the
    headline line is still printed.  barrier: a dist whose barrier goes in
    front of the transfer (start_after_barrier)."""
    try:
        # a 2 s per-wait deadline (the longest wait here is one 4 MiB push):
        # a broken link costs each later partner 2 s, not the default 10
        if barrier is not None:
            return start_after_barrier(barrier, c, *xfer_args, timeout_ms=POST_TIMEOUT_MS, **xfer_kw).wall_s
        return c.xfer(*xfer_args, timeout_ms=POST_TIMEOUT_MS, **xfer_kw).wall_s
    except Exception as e:  # noqa: BLE001
        errs.append(f"{type(e).__name__}: {e}"[:240])
        # a call armed for this transfer whose start never came (the barrier
        # in front of it failed) is cancelled here: left armed, every later
        # arm and transfer of this rank would be refused and its kernel would
        # spin until its go deadline.  A no-op when not armed.
        try:
            c.disarm(xfer_args[2])
        except Exception as e2:  # noqa: BLE001
            errs.append(f"disarm: {type(e2).__name__}: {e2}"[:240])
        return float("inf")


def arm(c, errs: list, *xfer_args, **xfer_kw) -> bool:
    """mpx_xfer_arm ahead of the barrier: the transfer's kernel is launched
    now and started by the xfer call with the same arguments after the
    barrier (MPI's persistent-request split, include/mpx.h), so the ~14 us
    launch is not inside the timed call.  A failure to arm is recorded and
    the call then launches inline."""
    try:
        c.arm(*xfer_args, **xfer_kw)
        return True
    except Exception as e:  # noqa: BLE001
        errs.append(f"arm: {type(e).__name__}: {e}"[:240])
        return False


def finite(x: float, digits: int):
    return round(x, digits) if x != float("inf") and x == x else None


def rate(num: float, wall: float, digits: int):
    """num / wall, or None when the wall time is a failed transfer's +inf"""
    return finite(num / wall, digits) if wall != float("inf") else None


# BASELINE config 3 / SURVEY §8d cfg3: the pair sweep uses config 1's sizes
# (the reference's own CPU sweep) plus the reference's default B = 456131
CFG3_SIZES = (1, 8, 64, 512, 4096, 32768, 262144, 456131, 1 << 20, 4 << 20)
LATENCY_ITERS = 100_000     # cfg3: 8 B latency with I >= 10^5


def round0_sweep(mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, errs) -> dict:
    """Config 3 beside the headline: the pairs of round 0 at every cfg3 size
    <= B, unidirectional (`-u 1`, B per iteration) and bidirectional (`-x 1`
    full duplex, 2B per iteration, mpi_perf.c:538).  Time = max over ranks of
    the loop's wall time; GB/s per pair."""
    g, peer = round_role(rounds, 0, rank)
    rates = {}

    def timed(mode, n, it):
        arm(c, errs, mode, g, rank, peer, it, tx, rx, n, timeout_ms=POST_TIMEOUT_MS)
        w = torch.tensor([safe_wall(c, errs, mode, g, rank, peer, it, tx, rx, n, barrier=dist)], dtype=torch.float64)
        dist.all_reduce(w, op=dist.ReduceOp.MAX)
        return float(w[0])

    for n in sorted(set(x for x in CFG3_SIZES if x <= nbytes) | {nbytes}):
        it = max(20, min(2000, (256 << 20) // n))
        w = timed(mpx.MODE_UNIDIR, n, it)
        rates[f"unidir_{n}"] = dict(us_per_iter=finite(w / it * 1e6, 3), GBps=rate(n * it / 1e9, w, 3))
        w = timed(mpx.MODE_NONBLOCKING, n, it)
        rates[f"nonblocking_{n}"] = dict(us_per_iter=finite(w / it * 1e6, 3), GBps=rate(2 * n * it / 1e9, w, 3))
    return rates


LL_AB_SIZES = (1024, 2048, 4096, 6144, 8192)
LL_AB_ITERS, LL_CHECK_ITERS = 2000, 20
# bytes an LL message writes per payload byte (8-B {tag, 4 B} granules):
# rocprofv3 --pmc WRITE_SIZE over a 1 KiB LL ping-pong, profiles/r02_pmc_xfer.json
LL_BYTES_PER_PAYLOAD_BYTE = 2.0


def choose_ll_max(mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, expect, errs) -> tuple[dict, int]:
    """The node picks its cross-GPU LL threshold (mpx_xfer_opts has none;
    libmpx reads MPX_LL_MAX per call), as it picks the push width.  LL: the
    data is the flag (8-B {tag, 4 B} granules, one link hop, 2 B written per
    payload byte); bulk: the payload, a drain, then a flag (two hops).
    Round 0's pairs ping-pong at each LL_AB_SIZES size with every message LL
    (MPX_LL_MAX = 8192) and every message bulk (MPX_LL_MAX = 0); each form is
    first run in check mode (every payload checksummed against the peer's
    tx), then timed: half round trip, max over ranks.  The threshold is the
    largest size up to which LL is never slower; every rank computes it from
    the same reduced table.  The caller sets MPX_LL_MAX to it (alike on every
    rank, so both ends of each pair agree) for everything after."""
    g, peer = round_role(rounds, 0, rank)
    table = {}
    sizes = [n for n in LL_AB_SIZES if n <= nbytes]
    old = os.environ.get("MPX_LL_MAX")
    try:
        for n in sizes:
            for proto, v in (("ll", "8192"), ("bulk", "0")):
                os.environ["MPX_LL_MAX"] = v
                dist.barrier()
                before = len(errs)
                safe_wall(c, errs, mpx.MODE_PINGPONG, g, rank, peer, LL_CHECK_ITERS, tx, rx, n, check_payload=True,
                          expect=expect[peer][n])
                dist.barrier()
                w = safe_wall(c, errs, mpx.MODE_PINGPONG, g, rank, peer, LL_AB_ITERS, tx, rx, n)
                if len(errs) > before:
                    w = float("inf")
                t = torch.tensor([w], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                table[f"{proto}_{n}"] = finite(float(t[0]) / (2 * LL_AB_ITERS) * 1e6, 3)
    finally:
        if old is None:
            os.environ.pop("MPX_LL_MAX", None)
        else:
            os.environ["MPX_LL_MAX"] = old
    chosen = 512       # LL at <= 512 B is one granule store per lane: never measured slower than bulk
    for n in sizes:
        ll, bulk = table.get(f"ll_{n}"), table.get(f"bulk_{n}")
        if ll is None or bulk is None or ll > bulk:
            break
        chosen = n
    return table, chosen


# bulk push variants tuned on the node's own links: (workgroups per push,
# streaming hint on the payload stores, mpx_xfer_opts.flags MPX_XFER_STREAM)
PUSH_CANDIDATES = tuple((w, st) for w in (16, 32, 64, 128, 256) for st in (False, True))
TUNE_ITERS = 40


def push_name(nwg: int, stream: bool) -> str:
    return f"{nwg}{'+nt' if stream else ''}"


def one_gpu_push_cap(world: int) -> int:
    """MPX_BENCH_ONE_GPU stacks all `world` ranks on GPU 0, and the two
    halves of every pair must have all their workgroups resident at once.
    k_xfer fits 4 workgroups per CU (1024 on 256 CUs); capping each side's
    push width at 512 / world keeps the N/2 concurrent pairs at <= 512 of
    them (N = 8: 64 each), with room for other work on the card.  0 when
    every rank has its own GPU."""
    if not os.environ.get("MPX_BENCH_ONE_GPU"):
        return 0
    return max(16, min(128, 512 // max(world, 1)))


def tune_push_local(mpx, c, rounds, rank, world, tx, rx, nbytes, expect, expect_ack) -> list[float]:
    """Time round 0's unidir loop at B once per bulk push variant (width =
    workgroups per push, mpx_xfer_opts.nwg; streaming store hint), each
    variant's payloads first validated (check mode, 2 iterations).  No
    collectives: each pair synchronises itself inside xfer, so a failure on
    one rank cannot leave the others inside a collective.  Returns this
    rank's wall times (0.0 for a variant that does not apply)."""
    g, peer = round_role(rounds, 0, rank)
    times = []
    max_wg = one_gpu_push_cap(world) or 256
    for nwg, stream in PUSH_CANDIDATES:
        if nbytes <= 8192 or nwg * 16 > nbytes or nwg > max_wg:
            times.append(0.0)
            continue
        c.xfer(mpx.MODE_UNIDIR, g, rank, peer, 2, tx, rx, nbytes, check_payload=True, expect=expect[peer],
               expect_ack=expect_ack[peer], timeout_ms=10000, nwg=nwg, stream=stream)
        times.append(c.xfer(mpx.MODE_UNIDIR, g, rank, peer, TUNE_ITERS, tx, rx, nbytes, nwg=nwg,
                            stream=stream).wall_s)
    return times


def pick_push(torch, dist, times: list[float], nbytes: int) -> tuple[tuple[int, bool], dict]:
    """Max over ranks of every variant's time; every rank then picks the
    same variant (the reduced tensor is identical everywhere)."""
    w = torch.tensor(times, dtype=torch.float64)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    rates = {cand: nbytes * TUNE_ITERS / float(t) / 1e9 for cand, t in zip(PUSH_CANDIDATES, w.tolist()) if t > 0}
    if not rates:
        return (0, False), {}
    best = max(rates, key=rates.get)
    return best, {push_name(*k): round(v, 2) for k, v in rates.items()}


def pair_table(torch, dist, rounds, rank, world, steps, step_dev, step_wall, launch_bytes) -> dict:
    """Every pair the timed steps covered (all N(N-1)/2 once the steps span
    the N-1 rounds): its G1 launch rate, "g1>g0" -> GB/s averaged over the
    steps that ran its round; and each round's aggregate, pairs x bytes /
    the max over ranks of the loop's wall time, averaged over its steps.
    Gathered after the timed region (one gloo all_gather)."""
    mine = torch.tensor(step_dev + step_wall, dtype=torch.float64)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    rates, agg = {}, {}
    for s in range(steps):
        rd = s % len(rounds)
        walls = [float(every[r][steps + s]) for r in range(world)]
        agg.setdefault(rd, []).append((world // 2) * launch_bytes / max(walls) / 1e9)
        for r in range(world):
            g, peer = round_role(rounds, rd, r)
            if g == 1 and float(every[r][s]) > 0:
                rates.setdefault(f"{r}>{peer}", []).append(launch_bytes / float(every[r][s]) / 1e9)
    per_pair = {k: round(statistics.mean(v), 2) for k, v in sorted(rates.items(), key=lambda kv: tuple(
        int(x) for x in kv[0].split(">")))}
    out = {"pair_GBps": per_pair,
           "round_aggregate_GBps": [round(statistics.mean(agg[rd]), 2) for rd in sorted(agg)]}
    if per_pair:
        out["pair_GBps_min_max"] = [min(per_pair.values()), max(per_pair.values())]
    return out


PAIR_LATENCY_ITERS = 10_000
# small messages checked on every link before they are timed: the LL protocol
# (<= 8 KiB across xGMI) and the first bulk size above it; validation of the
# headline covers only B
SMALL_CHECK_SIZES, SMALL_CHECK_ITERS = (1, 8, 4097, 8192, 8193), 20


def small_message_check(mpx, torch, dist, c, rounds, rank, world, tx, rx, nbytes, errs) -> dict:
    """Ping-pong with every received payload checksummed (check mode) at
    SMALL_CHECK_SIZES on every round's pairs, i.e. on every link the steps
    used: the small-message protocol's payloads are verified on the node's
    own links, beside the latency they are timed at."""
    sizes = [n for n in SMALL_CHECK_SIZES if n <= nbytes]
    mine = [c.checksum(tx, n) for n in sizes]
    every = [None] * world
    dist.all_gather_object(every, mine)
    before = len(errs)
    for rd in range(len(rounds)):
        g, peer = round_role(rounds, rd, rank)
        for k, n in enumerate(sizes):
            dist.barrier()
            safe_wall(c, errs, mpx.MODE_PINGPONG, g, rank, peer, SMALL_CHECK_ITERS, tx, rx, n,
                      check_payload=True, expect=every[peer][k])
    bad = torch.tensor([float(len(errs) - before)], dtype=torch.float64)
    dist.all_reduce(bad, op=dist.ReduceOp.SUM)
    return dict(sizes=sizes, iters=SMALL_CHECK_ITERS, rounds=len(rounds),
                payloads_checked=world * len(rounds) * len(sizes) * SMALL_CHECK_ITERS,
                failed_transfers=int(bad[0]))
# BASELINE config 4's other workload, scripts/run-hbv3.sh: -u 1 -b 456131 -i 10
# passes: the median over 11 calls per round (3 read 0.80-0.87 of the long
# loop across boxes; a call is ~35 us, so more passes cost nothing)
HBV3_BYTES, HBV3_ITERS, HBV3_PASSES = 456131, 10, 11


def hbv3_rounds(mpx, torch, dist, c, rounds, rank, world, tx, rx, errs, phases: bool = False) -> dict:
    """run-hbv3's message shape over the all-pairs rounds: every round runs
    the unidir loop at 456131 B x 10 iterations behind a barrier, HBV3_PASSES
    passes; a round's aggregate is pairs x B x iterations / the max over ranks
    of the loop's wall time (the reference's MAX allreduce), median over the
    passes.  At 10 iterations launch and flag latency weigh as much as the
    link: this is the reference's own short-loop measurement.  Each call is
    armed before its barrier (arm), as the timed steps are.  phases (kernel
    engine): every call's mpx_last_phases split, medians per side over all
    calls of all ranks (where the fixed cost per call goes)."""
    walls, ph = [], []
    for _ in range(HBV3_PASSES):
        for rd in range(len(rounds)):
            g, peer = round_role(rounds, rd, rank)
            arm(c, errs, mpx.MODE_UNIDIR, g, rank, peer, HBV3_ITERS, tx, rx, HBV3_BYTES, timeout_ms=POST_TIMEOUT_MS)
            walls.append(safe_wall(c, errs, mpx.MODE_UNIDIR, g, rank, peer, HBV3_ITERS, tx, rx, HBV3_BYTES,
                                   barrier=dist))
            if phases and walls[-1] != float("inf"):
                ph.append((g, c.phases(rank)))
    w = torch.tensor(walls, dtype=torch.float64)
    dist.all_reduce(w, op=dist.ReduceOp.MAX)
    nr = len(rounds)
    per_round = []
    for rd in range(nr):
        t = statistics.median(float(w[p * nr + rd]) for p in range(HBV3_PASSES))
        per_round.append(rate((world // 2) * HBV3_BYTES * HBV3_ITERS / 1e9, t, 2))
    ok = [v for v in per_round if v is not None]
    out = dict(bytes=HBV3_BYTES, iters=HBV3_ITERS, round_aggregate_GBps=per_round,
               mean_aggregate_GBps=round(statistics.mean(ok), 2) if len(ok) == len(per_round) else None)
    if phases:
        every = [None] * world
        dist.all_gather_object(every, ph)
        allp = [x for e in every for x in (e or [])]
        out["phases_us_median"] = {
            side: {k: round(statistics.median(p[k] for gg, p in allp if gg == g) * 1e6, 2) for k in allp[0][1]
                   if k not in ("armed", "resident")}
            for side, g in (("g1", 1), ("g0", 0)) if any(gg == g for gg, _ in allp)} if allp else None
        # armed calls whose whole grid was running when mpx_xfer_arm returned
        out["resident_fraction"] = round(sum(p["resident"] for _, p in allp) / len(allp), 3) if allp else None
    return out


PULL_AB_ITERS = 100


def push_vs_pull(mpx, torch, dist, c, rounds, rank, world, tx, rx, nbytes, nwg, stream, expect, expect_ack,
                 errs) -> dict:
    """Round 0's pairs at B in both directions of data movement of the
    kernel engine ("try pull as well"): push (the
    headline's form and tuned width) and pull (MPX_XFER_PULL: the receiver's
    workgroups load the sender's peer-mapped tx into their own rx, same
    width), each validated first (check mode, 3 iterations), then timed
    unidirectional (-u 1) and full duplex (-x 1), PULL_AB_ITERS iterations;
    GB/s per pair = bytes / the max over ranks of the loop's wall time.
    Reported beside the headline, never chosen for it: that a pulled byte
    crossed the link each iteration (no reuse from this GPU's caches) needs
    the per-launch link counters of tools/node_profile.sh."""
    g, peer = round_role(rounds, 0, rank)
    out = {}
    for name, pull in (("push", False), ("pull", True)):
        for mode, label, mult in ((mpx.MODE_UNIDIR, "unidir", 1), (mpx.MODE_NONBLOCKING, "nonblocking", 2)):
            dist.barrier()
            before = len(errs)
            safe_wall(c, errs, mode, g, rank, peer, 3, tx, rx, nbytes, check_payload=True, expect=expect[peer],
                      expect_ack=expect_ack[peer], nwg=nwg, stream=stream, pull=pull)
            dist.barrier()
            w = safe_wall(c, errs, mode, g, rank, peer, PULL_AB_ITERS, tx, rx, nbytes, nwg=nwg, stream=stream,
                          pull=pull)
            if len(errs) > before:
                w = float("inf")
            t = torch.tensor([w], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            out[f"{name}_{label}_GBps"] = rate(mult * nbytes * PULL_AB_ITERS / 1e9, float(t[0]), 2)
    # the pull's own width: unidir at every tuning width (the push's choice
    # need not be the pull's), within the one-GPU rehearsal's residency cap
    by_width = {}
    max_wg = one_gpu_push_cap(world) or 256
    for w in sorted({x for x, _ in PUSH_CANDIDATES}):
        if w * 16 > nbytes or w > max_wg:
            continue
        dist.barrier()
        wall = safe_wall(c, errs, mpx.MODE_UNIDIR, g, rank, peer, PULL_AB_ITERS, tx, rx, nbytes, nwg=w, pull=True)
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        by_width[str(w)] = rate(nbytes * PULL_AB_ITERS / 1e9, float(t[0]), 2)
    out.update(pull_unidir_GBps_by_width=by_width, bytes=nbytes, iters=PULL_AB_ITERS,
               width=push_name(nwg, stream) if nwg else "default")
    return out


def staged_vs_unstaged(mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, iters, nwg, stream, expect, expect_ack,
                       errs) -> dict:
    """What the headline push reads: each pushing
    workgroup copies its chunk of tx into LDS once per call and every push
    reads LDS (tx is read-only while the loop runs; the reference re-sends
    the same buffer, mpi_perf.c:136).  Round 0's pairs run the headline's
    unidir loop (B x iters, the tuned width) staged and with
    MPX_XFER_NOSTAGE (every push reads tx from HBM), each validated first
    (check mode, 3 iterations); GB/s per pair = B x iters / the max over
    ranks of the loop's wall time.  On links the two should agree: the link,
    not the sender's read, bounds the push."""
    g, peer = round_role(rounds, 0, rank)
    out = {}
    for label, stage in (("staged", True), ("unstaged", False)):
        dist.barrier()
        before = len(errs)
        safe_wall(c, errs, mpx.MODE_UNIDIR, g, rank, peer, 3, tx, rx, nbytes, check_payload=True, expect=expect,
                  expect_ack=expect_ack, nwg=nwg, stream=stream, stage=stage)
        dist.barrier()
        w = safe_wall(c, errs, mpx.MODE_UNIDIR, g, rank, peer, iters, tx, rx, nbytes, nwg=nwg, stream=stream,
                      stage=stage)
        if len(errs) > before:
            w = float("inf")
        t = torch.tensor([w], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        out[f"unidir_{label}_GBps"] = rate(nbytes * iters / 1e9, float(t[0]), 2)
    return out


# xGMI / HBM bytes of the senders, read in-process (mpx/counters.py).  A
# write to a peer GPU leaves the sender's L2 as an EA write request that is
# not destined for local DRAM: link requests = WRREQ - WRREQ_DRAM, 64 B each
# (a bulk push of B bytes makes B / 64 64-B requests: profiles/r02_pmc_xfer_ea.json).
LINK_COUNTERS = ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum", "TCC_EA0_WRREQ_DRAM_sum")
READ_COUNTERS = ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_DRAM_sum")
# where the non-DRAM writes go, in 32-B units (gfx950: "1 64-byte request
# will be counted to 2"): the GMI (inter-die / xGMI) and IO (PCIe) paths
FABRIC_COUNTERS = ("TCC_EA0_WRREQ_WRITE_GMI_32B_sum", "TCC_EA0_WRREQ_WRITE_IO_32B_sum",
                   "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
# the link bytes' self-check: on distinct GPUs the
# subtraction must read the pushed bytes within this band, else the line
# carries no traffic figure (null, with the raw counters and the reason)
LINK_CHECK_BAND = (0.9, 1.1)
COUNTER_SETS = (LINK_COUNTERS, READ_COUNTERS, FABRIC_COUNTERS)
ALL_COUNTERS = LINK_COUNTERS + READ_COUNTERS + FABRIC_COUNTERS
# the candidate link-byte formulas, in order of preference: the EA write
# requests not destined for local DRAM x 64 B, the GMI-path 32-B writes x 32,
# the IO-path 32-B writes x 32
LINK_FORMULAS = ("subtraction", "gmi", "io")
# peer_link_control: known bytes written across one link by k_copy (not the
# pair kernel); a formula reading them within this band is validated
PEER_CONTROL_BYTES, PEER_CONTROL_ITERS, PEER_CONTROL_BAND = 16 << 20, 8, (0.95, 1.1)


def link_formula_bytes(v: dict) -> dict:
    """bytes each candidate link formula reads from one set of counter values
    (a formula whose counters are missing is left out)"""
    out = {}
    if "TCC_EA0_WRREQ_sum" in v and "TCC_EA0_WRREQ_DRAM_sum" in v:
        out["subtraction"] = (v["TCC_EA0_WRREQ_sum"] - v["TCC_EA0_WRREQ_DRAM_sum"]) * 64
    if "TCC_EA0_WRREQ_WRITE_GMI_32B_sum" in v:
        out["gmi"] = v["TCC_EA0_WRREQ_WRITE_GMI_32B_sum"] * 32
    if "TCC_EA0_WRREQ_WRITE_IO_32B_sum" in v:
        out["io"] = v["TCC_EA0_WRREQ_WRITE_IO_32B_sum"] * 32
    return out


def peer_link_control(mpx, prof, bus: str, dev: int, peer_dev: int) -> dict:
    """Positive control of the link-byte counters ON the node, independent
    of the pair kernel (one GPU can only show host and
    local destinations: tools/link_counter_control.py).  In this process, a
    second context with one rank on `dev` and one on `peer_dev` (peer access
    both ways): k_copy on `dev` writes B x iters known bytes into `peer_dev`'s
    memory, then the pair kernel pushes B x iters (unidir, threads) the same
    way; this GPU's counters (LINK_COUNTERS, FABRIC_COUNTERS) are read around
    each.  The first formula whose copy reading lies in PEER_CONTROL_BAND is
    the validated one; None if none does."""
    import threading
    B, IT = PEER_CONTROL_BYTES, PEER_CONTROL_ITERS
    out = dict(bytes=B * IT, gpus=[dev, peer_dev], band=list(PEER_CONTROL_BAND),
               writers="copy: k_copy on gpus[0] into gpus[1]'s HBM; push: k_xfer unidir gpus[0] -> gpus[1]")
    c = mpx.Context(2, "kernel")
    try:
        tx0, rx0, tx1, rx1 = c.alloc(dev, B), c.alloc(dev, B), c.alloc(peer_dev, B), c.alloc(peer_dev, B)
        c.fill(tx0, B, mpx.FILL_SPLITMIX, 0x11)
        c.fill(tx1, B, mpx.FILL_SPLITMIX, 0x22)
        c.attach(0, dev, tx0, rx0, B)
        c.attach(1, peer_dev, tx1, rx1, B)
        errs = []

        def copy():
            # a launch per copy: every byte crosses once per launch, and each
            # launch's end-of-kernel release writes back what the L2 holds —
            # one launch of IT copies lets a write-back-cached destination
            # absorb the rewrites in the L2 (tools/link_counter_control.py:
            # coherent host memory reads 0.39 x that way)
            for _ in range(IT):
                c.copy(dev, rx1, tx0, B, 1)

        def side(r):
            try:
                c.xfer(mpx.MODE_UNIDIR, 1 - r, r, 1 - r, IT, (tx0, tx1)[r], (rx0, rx1)[r], B, timeout_ms=5000)
            except Exception as e:  # noqa: BLE001
                errs.append(f"{type(e).__name__}: {e}"[:160])

        def push():
            th = [threading.Thread(target=side, args=(r,)) for r in (0, 1)]
            for t in th:
                t.start()
            for t in th:
                t.join()

        for name, work in (("copy", copy), ("push", push)):
            # rx1 poisoned before each phase and checked right after it, so
            # the copy's check sees the copy's bytes, not the push's
            c.fill(rx1, B, mpx.FILL_BYTE, 0)
            work()
            out[f"{name}_checked"] = c.checksum(rx1, B) == c.checksum(tx0, B)
            vals = {}
            for names in (LINK_COUNTERS, FABRIC_COUNTERS):
                try:
                    with prof.Pass(bus, list(names)) as p:
                        work()
                    vals.update(zip(names, p.values))
                except Exception as e:  # noqa: BLE001
                    if names is LINK_COUNTERS:
                        raise
                    out[f"{name}_fabric_error"] = f"{type(e).__name__}: {e}"[:160]   # optional set
            fb = link_formula_bytes(vals)
            dram32 = vals.get("TCC_EA0_WRREQ_WRITE_DRAM_32B_sum")
            out[name] = dict({f"{k}_over_bytes": round(v / (B * IT), 5) for k, v in fb.items()},
                             dram_over_bytes=None if dram32 is None else round(dram32 * 32 / (B * IT), 5),
                             raw=vals)
        if errs:
            out["push_errors"] = errs
    finally:
        c.close()
    lo, hi = PEER_CONTROL_BAND
    out["validated_formula"] = next((f for f in LINK_FORMULAS if out["copy_checked"] and f"{f}_over_bytes" in
                                     out["copy"] and lo <= out["copy"][f"{f}_over_bytes"] <= hi), None)
    return out


def link_counters(mpx, prof, torch, dist, c, rounds, rank, world, tx, rx, nbytes, iters, nwg, stream, buses,
                  errs) -> dict:
    """Counters of the timed steps' own work: every round runs once more,
    untimed (the same loop, width and hint, a barrier per round as in the
    steps), inside one counter pass per counter set.  The counters are
    agent-wide, so exactly one rank per GPU samples (the lowest rank on its
    bus id); on a one-GPU rehearsal that rank sees every pair.  Per G1 launch
    (N/2 pairs x N-1 rounds launches per pass): link bytes, local-DRAM bytes,
    EA read requests; rates against the passes' own average G1 launch time."""
    sampler = rank == min(r for r in range(world) if buses[r] == buses[rank])
    vals = {}
    g1_s, g1_n = 0.0, 0
    notes = []
    for names in COUNTER_SETS:
        p = None
        if sampler:
            try:
                p = prof.Pass(buses[rank], list(names)).__enter__()
            except Exception as e:  # noqa: BLE001
                notes.append(f"rank {rank}: {type(e).__name__}: {e}"[:200])
        for rd in range(len(rounds)):
            g, peer = round_role(rounds, rd, rank)
            dist.barrier()
            try:
                t = c.xfer(mpx.MODE_UNIDIR, g, rank, peer, iters, tx, rx, nbytes, nwg=nwg, stream=stream)
                if g == 1 and names is LINK_COUNTERS:
                    g1_s += t.device_s
                    g1_n += 1
            except Exception as e:  # noqa: BLE001
                errs.append(f"counters: {type(e).__name__}: {e}"[:240])
        if p is not None:
            try:
                p.__exit__(None, None, None)
                vals.update(zip(names, p.values))
                vals["reads_reset"] = p.reads_reset
            except Exception as e:  # noqa: BLE001
                notes.append(f"rank {rank}: {type(e).__name__}: {e}"[:200])
    # sampled = the link and read sets were read; the fabric set is optional
    # (one GMI/IO counter unavailable nulls only its own figures)
    required = LINK_COUNTERS + READ_COUNTERS
    mine = [1.0 if (sampler and all(k in vals for k in required)) else 0.0,
            1.0 if (sampler and all(k in vals for k in FABRIC_COUNTERS)) else 0.0]
    mine += [float(vals.get(k, 0.0)) for k in ALL_COUNTERS] + [g1_s, float(g1_n)]
    every = [torch.zeros(len(mine), dtype=torch.float64) for _ in range(world)]
    dist.all_gather(every, torch.tensor(mine, dtype=torch.float64))
    all_notes = [None] * world
    dist.all_gather_object(all_notes, notes)
    notes = [n for x in all_notes for n in (x or [])]
    want = sum(1 for r in range(world) if r == min(q for q in range(world) if buses[q] == buses[r]))
    got = [e for e in every if float(e[0]) == 1.0]
    if len(got) != want:
        return {"error": "; ".join(notes) or "not every GPU was sampled", "samplers": want, "sampled": len(got)}
    tot = [sum(float(e[2 + k]) for e in got) for k in range(len(ALL_COUNTERS))]
    fabric = all(float(e[1]) == 1.0 for e in got)
    wr, w64, dram, rd, rd_dram, gmi32, io32, dram32 = tot
    launches = (world // 2) * len(rounds)
    alg = nbytes * iters * launches
    distinct = len(set(buses)) == world
    g1_avg = sum(float(e[-2]) for e in every) / max(sum(float(e[-1]) for e in every), 1.0)
    link = (wr - dram) * 64
    formulas = link_formula_bytes(dict(zip(ALL_COUNTERS, tot)))
    if not fabric:
        formulas = {k: v for k, v in formulas.items() if k == "subtraction"}
        notes.append("fabric counters (GMI / IO 32-B writes) not read on every sampler: their figures are null")

    def fab(v, digits):
        return round(v, digits) if fabric else None
    out = dict(
        source="in-process rocprofiler-sdk device counting service (mpi-perf_amd/lib/libmpxprof.so), one pass per "
               "counter set over an untimed re-run of every round (the timed steps' loop, width and hint), one "
               "sampling rank per GPU",
        counters=list(ALL_COUNTERS), samplers=want, g1_launches_per_pass=launches,
        raw=dict(zip(ALL_COUNTERS, tot)), ranks_on_distinct_gpus=distinct,
        algorithmic_bytes_per_launch=nbytes * iters,
        link_bytes_per_launch=round(link / launches, 1),
        local_dram_write_bytes_per_launch=round(dram * 64 / launches, 1),
        link_over_algorithmic=round(link / alg, 5), local_dram_over_algorithmic=round(dram * 64 / alg, 5),
        write_requests_64B_fraction=round(w64 / wr, 5) if wr else None,
        read_requests_per_launch=round(rd / launches, 1), read_dram_requests_per_launch=round(rd_dram / launches, 1),
        gmi_write_bytes_per_launch=fab(gmi32 * 32 / launches, 1), io_write_bytes_per_launch=fab(io32 * 32 / launches, 1),
        gmi_over_algorithmic=fab(gmi32 * 32 / alg, 5), io_over_algorithmic=fab(io32 * 32 / alg, 5),
        fabric_counters_read=fabric,
        g1_avg_launch_us=round(g1_avg * 1e6, 2),
        achieved_link_GBps_per_pair=round(link / launches / g1_avg / 1e9, 2) if g1_avg > 0 else None,
        achieved_local_dram_GBps_per_pair=round(dram * 64 / launches / g1_avg / 1e9, 2) if g1_avg > 0 else None,
        reads_reset=vals.get("reads_reset"),
        link_formula_bytes_per_launch={k: round(v / launches, 1) for k, v in formulas.items()},
        link_formula_over_algorithmic={k: round(v / alg, 5) for k, v in formulas.items()})
    if notes:
        out["notes"] = notes
    # MPX_BENCH_PEER_CONTROL=1 runs the control on a one-GPU rehearsal too
    # (GPU 0 -> GPU 0: the integration on hardware; it validates nothing)
    if distinct or os.environ.get("MPX_BENCH_PEER_CONTROL") == "1":
        # rank 0 validates the formulas on this node with known bytes across
        # its round-0 link, while the other ranks wait (untimed)
        if rank == 0:
            peer = round_role(rounds, 0, 0)[1]
            try:
                peer_dev = next(d for d in range(mpx.device_count()) if mpx.bus_id(d) == buses[peer])
                my_dev = next(d for d in range(mpx.device_count()) if mpx.bus_id(d) == buses[rank])
                out["peer_control"] = peer_link_control(mpx, prof, buses[rank], my_dev, peer_dev)
            except Exception as e:  # noqa: BLE001
                out["peer_control"] = {"error": f"{type(e).__name__}: {e}"[:240]}
        dist.barrier()
    return out


def link_traffic(cnt: dict) -> dict:
    """roofline fields from link_counters' result, with the self-check
    (VERDICT r04, next 2).  On distinct GPUs every pushed byte crosses a
    link, so (WRREQ - WRREQ_DRAM) x 64 must read the pushed bytes: outside
    LINK_CHECK_BAND the line prints NO traffic figure (null), with the raw
    counters and the reason — a counter that cannot see the path's link
    writes (e.g. if peer-HBM writes were classified as DRAM at the sender)
    must not pass for a measurement of ~0.  When the ranks share a GPU
    (the one-GPU rehearsal) the pushes are local and ~0 is the right
    reading: no check applies."""
    lo, hi = LINK_CHECK_BAND
    r = cnt["link_over_algorithmic"]
    src = ("xGMI link bytes per G1 launch: (TCC_EA0_WRREQ - TCC_EA0_WRREQ_DRAM) x 64 B of every GPU, summed; "
           + cnt["source"])
    if not cnt.get("ranks_on_distinct_gpus"):
        return dict(traffic=cnt["link_bytes_per_launch"], traffic_local_dram=cnt["local_dram_write_bytes_per_launch"],
                    traffic_source=src, traffic_check="not applicable: ranks share a GPU (local pushes, ~0 expected)")
    pc = cnt.get("peer_control") or {}
    f = pc.get("validated_formula")
    if f and f in cnt["link_formula_over_algorithmic"]:
        # a formula validated on THIS node by known bytes across a link (an
        # independent writer): it measures the pushes, whatever they read
        fr = cnt["link_formula_over_algorithmic"][f]
        return dict(traffic=cnt["link_formula_bytes_per_launch"][f],
                    traffic_local_dram=cnt["local_dram_write_bytes_per_launch"],
                    traffic_source=f"xGMI link bytes per G1 launch by the '{f}' formula, validated on this node: "
                                   f"{pc['copy'][f + '_over_bytes']} x the bytes k_copy wrote across a link "
                                   f"(extras.counters.peer_control); " + cnt["source"],
                    traffic_check=(f"validated ({f}); the pushes read {fr} x the pushed bytes" +
                                   ("" if lo <= fr <= hi else f" — outside {lo}-{hi}: link bytes differ from the "
                                                              f"pushed bytes")))
    if lo <= r <= hi:
        return dict(traffic=cnt["link_bytes_per_launch"], traffic_local_dram=cnt["local_dram_write_bytes_per_launch"],
                    traffic_source=src, traffic_check=f"passed: link bytes {r} x the pushed bytes (band {lo}-{hi})")
    return dict(traffic=None, traffic_local_dram=cnt["local_dram_write_bytes_per_launch"], traffic_source=src,
                traffic_check="failed",
                traffic_reason=(f"link-byte self-check failed: (WRREQ - WRREQ_DRAM) x 64 read {r} x the pushed bytes "
                                f"(band {lo}-{hi}); the GMI 32-B write counter reads {cnt.get('gmi_over_algorithmic')}, "
                                f"IO {cnt.get('io_over_algorithmic')}, local DRAM "
                                f"{cnt.get('local_dram_over_algorithmic')} x; the peer control validated no formula "
                                f"({(cnt.get('peer_control') or {}).get('error') or 'see extras.counters.peer_control'})"
                                f": the counters do not see this path's link bytes as the formula assumes, so no "
                                f"traffic figure is printed"),
                traffic_raw=cnt.get("raw"))


def link_table(mpx, rounds, devs) -> dict:
    """mpx_link_info for EVERY pair the rounds cover:
    "g1>g0" -> {type, hops, gpus}; pairs that are not one xGMI hop are listed
    under "not_one_xgmi_hop" (their rate is not a single link's)."""
    table, odd = {}, []
    for rd in range(len(rounds)):
        for r in range(len(devs)):
            g, peer = round_role(rounds, rd, r)
            if g != 1:
                continue
            key = f"{r}>{peer}"
            try:
                info = dict(mpx.link_info(devs[r], devs[peer]), gpus=[devs[r], devs[peer]], round=rd)
            except Exception as e:  # noqa: BLE001
                info = dict(error=f"{type(e).__name__}: {e}"[:160], gpus=[devs[r], devs[peer]], round=rd)
            table[key] = info
            if info.get("type") != "xgmi" or info.get("hops") != 1:
                odd.append(key)
    return dict(pairs=dict(sorted(table.items(), key=lambda kv: tuple(int(x) for x in kv[0].split(">")))),
                not_one_xgmi_hop=odd)


def pair_latency(mpx, torch, dist, c, rounds, rank, world, tx, rx, errs) -> dict:
    """8 B ping-pong half round trip of every pair, round by round
    (PAIR_LATENCY_ITERS iterations each): "g1>g0" -> us, the pair's slower
    side's wall time / (2 x iterations)."""
    walls = []
    for rd in range(len(rounds)):
        g, peer = round_role(rounds, rd, rank)
        dist.barrier()
        walls.append(safe_wall(c, errs, mpx.MODE_PINGPONG, g, rank, peer, PAIR_LATENCY_ITERS, tx, rx, 8))
    mine = torch.tensor(walls, dtype=torch.float64)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    out = {}
    for rd in range(len(rounds)):
        for r in range(world):
            g, peer = round_role(rounds, rd, r)
            if g == 1:
                w = max(float(every[r][rd]), float(every[peer][rd]))
                out[f"{r}>{peer}"] = finite(w / (2 * PAIR_LATENCY_ITERS) * 1e6, 3)
    return dict(sorted(out.items(), key=lambda kv: tuple(int(x) for x in kv[0].split(">"))))


def pairs_bench(mpx, torch, dist, engine, rank, world, dev, nbytes, iters, steps, warmup, barrier_sync,
                latency=True, tune=True, pull=False, prof=None, count: bool = False) -> dict:
    """All-pairs rounds on `engine` (one process per GPU, IPC-mapped peers;
    pull: the engine's MPX_XFER_PULL form, validation and steps alike).
    Every round's payloads are validated once (check mode, seeded per-rank
    patterns) before anything is timed.  prof (mpx/counters.py, registered):
    the steps' link / DRAM bytes are counted after them.  Returns a dict;
    "error" is set (on every rank) if any rank failed."""
    rounds = all_pairs_rounds(world)
    out = {}
    c = None
    pkw = {"pull": True} if pull else {}   # (the keyword only when set: the default call stays as it was)

    def agree(err: str) -> str:
        """every rank learns the first error of any rank (one gloo collective)"""
        flags = [None] * world
        dist.all_gather_object(flags, err)
        return next((f for f in flags if f), "")

    # phase 1: local setup (no collectives inside the try)
    mine, err, tune_times = None, "", None
    try:
        c = mpx.Context(world, engine)
        tx, rx = c.alloc(dev, nbytes), c.alloc(dev, nbytes)
        c.fill(tx, nbytes, mpx.FILL_SPLITMIX, mpx.pattern_key(mpx.PATTERN_SEED, rank, 0, 0))
        c.attach(rank, dev, tx, rx, nbytes)
        # (descriptor, checksums of tx[0:B] and tx[0:1], bus id, checksums of
        # the small-message and LL-threshold sizes' prefixes)
        mine = (c.export(rank), c.checksum(tx, nbytes), c.checksum(tx, 1), mpx.bus_id(dev),
                {n: c.checksum(tx, n) for n in set(SMALL_CHECK_SIZES) | set(LL_AB_SIZES) if n <= nbytes})
    except Exception as e:  # noqa: BLE001
        err = f"rank {rank}: {type(e).__name__}: {e}"[:300]
    descs = [None] * world
    dist.all_gather_object(descs, mine)
    err = agree(err)
    if engine == "rccl" and not err:
        # RCCL needs one rank per device; two ranks on one GPU (the one-GPU
        # rehearsal) are refused here, before ncclCommInitRank: its refused
        # init left every process of round 3's rehearsal slowed for the rest
        # of the run (profiles/r03_pull_rounds_diag.jsonl)
        buses = [d[3] for d in descs]
        dup = [(a, b) for a in range(world) for b in range(a + 1, world) if buses[a] == buses[b]]
        if dup:
            err = (f"RCCL not initialised: ranks {dup[0][0]} and {dup[0][1]} share GPU {buses[dup[0][0]]} "
                   f"(RCCL needs one rank per device)")
    uid = [None]
    if engine == "rccl" and not err:
        uid = [mpx.rccl_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
    # phase 2: map the peers, then validate every round once, each round
    # behind a barrier like a reference run (mpi_perf.c:499); a rank whose
    # transfer failed keeps joining the barriers, so no rank is left inside a
    # collective; the push tuning has no collectives (each pair synchronises
    # itself inside xfer)
    if not err:
        try:
            for r in range(world):
                if r != rank and engine != "rccl":   # RCCL maps its own buffers
                    c.import_rank(r, descs[r][0])
            if engine == "rccl":
                c.rccl_init_rank(rank, world, uid[0])
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: {type(e).__name__}: {e}"[:300]
        err = agree(err)
    if not err:
        for r in range(len(rounds)):
            g, peer = round_role(rounds, r, rank)
            dist.barrier()
            if err:
                continue
            try:
                c.xfer(mpx.MODE_UNIDIR, g, rank, peer, 3, tx, rx, nbytes, check_payload=True,
                       expect=descs[peer][1], expect_ack=descs[peer][2], timeout_ms=10000, **pkw)
            except Exception as e:  # noqa: BLE001
                err = f"rank {rank}: round {r}: {type(e).__name__}: {e}"[:300]
        err = agree(err)
    if not err and engine == "kernel" and tune:
        try:
            tune_times = tune_push_local(mpx, c, rounds, rank, world, tx, rx, nbytes, [d[1] for d in descs],
                                         [d[2] for d in descs])
        except Exception as e:  # noqa: BLE001
            err = f"rank {rank}: push tuning: {type(e).__name__}: {e}"[:300]
        err = agree(err)
    if err:
        if c is not None:
            try:
                c.close()
            except Exception:  # noqa: BLE001
                pass
        # every rank's imports of the others' buffers are closed before any
        # rank allocates again: a block still imported by a peer cannot be
        # re-exported (hipIpcGetMemHandle: invalid argument, seen on gfx950)
        dist.barrier()
        return {"error": err}
    out["validated_rounds"] = len(rounds)
    nwg, stream = 0, False
    if tune_times is not None:
        (nwg, stream), out["push_tune"] = pick_push(torch, dist, tune_times, nbytes)
    out["push"] = push_name(nwg, stream) if nwg else "default"

    step_err = []
    timed_armed = []   # per timed G1 step: started from an armed launch (kernel-span clock)

    def step(s: int):
        g, peer = round_role(rounds, s % len(rounds), rank)
        # the step's kernel is launched ahead of the barrier and started after
        # it (mpx_xfer_arm; a no-op on the SDMA and RCCL engines)
        armed = not step_err and arm(c, step_err, mpx.MODE_UNIDIR, g, rank, peer, iters, tx, rx, nbytes, nwg=nwg,
                                     stream=stream, **pkw)
        if step_err:                                 # keep joining the barriers, transfer nothing
            dist.barrier()                           # MPI_Barrier, mpi_perf.c:499
            if armed:
                c.disarm(rank)
            return g, None
        try:
            # MPI_Barrier (mpi_perf.c:499), then the loop: one C call with
            # the spin barrier (start_after_barrier)
            t = start_after_barrier(dist, c, mpx.MODE_UNIDIR, g, rank, peer, iters, tx, rx, nbytes, nwg=nwg,
                                    stream=stream, **pkw)
            step.armed = armed and engine == "kernel"
            return g, t
        except Exception as e:  # noqa: BLE001
            step_err.append(f"rank {rank}: step {s}: {type(e).__name__}: {e}"[:300])
            if armed:   # the start never came (a failed barrier): cancel the armed kernel now
                try:
                    c.disarm(rank)
                except Exception:  # noqa: BLE001
                    pass
            return g, None

    # SDMA engine: its graph-captured chunks are built for every round's
    # (peer, side) before the timed steps (mpx_xfer_prepare), and every round
    # gets an untimed step, so no capture or first-use cost lands inside
    # `elapsed` whatever the warmup count
    if engine == "sdma":
        for r in range(len(rounds)):
            g, peer = round_role(rounds, r, rank)
            c.prepare(mpx.MODE_UNIDIR, g, rank, peer, iters, nbytes, **pkw)
    for s in range(max(warmup, len(rounds))):
        step(s)
    dev_s, n_sends, step_nwg = 0.0, 0, 0
    step_dev, step_wall = [0.0] * steps, [0.0] * steps   # this rank's G1 device time / wall time per step
    barrier_sync()
    t0 = time.perf_counter()
    for s in range(steps):
        g, t = step(s)
        if t is None:
            continue
        step_wall[s] = t.wall_s
        if g == 1:
            dev_s += t.device_s
            n_sends += 1
            step_dev[s] = t.device_s
            step_nwg = t.nwg
            timed_armed.append(step.armed)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    err = agree(step_err[0] if step_err else "")
    if err:   # a timed step failed on some rank: no headline from this engine
        c.close()
        dist.barrier()
        return {"error": err}
    tt = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    out["elapsed"] = float(tt[0])
    out["total"] = (world // 2) * nbytes * iters * steps
    st = torch.tensor([dev_s, float(n_sends)], dtype=torch.float64)
    dist.all_reduce(st, op=dist.ReduceOp.SUM)
    out["per_launch_s"] = float(st[0]) / max(float(st[1]), 1.0)
    out["per_pair_GBps"] = nbytes * iters / out["per_launch_s"] / 1e9
    # which clock per_launch_s is on: an armed kernel-engine
    # call's device time is the kernel's own span, from the moment workgroup 0
    # sees the go word to the last workgroup's end (s_memrealtime); an
    # unarmed call's (and the stream engines') is the HIP-event span, launch
    # included.  Rounds 1-3 were all "events".
    na = torch.tensor([float(sum(timed_armed)), float(len(timed_armed))], dtype=torch.float64)
    dist.all_reduce(na, op=dist.ReduceOp.SUM)
    out["device_clock"] = ("kernel-span (armed: go seen -> last workgroup end, s_memrealtime)" if na[0] == na[1] and na[1]
                           else "events (HIP events around the launch)" if na[0] == 0
                           else f"mixed: {int(na[0])} of {int(na[1])} G1 launches armed (kernel span), the rest events")
    out.update(pair_table(torch, dist, rounds, rank, world, steps, step_dev, step_wall, nbytes * iters))
    nw = torch.tensor([float(step_nwg)], dtype=torch.float64)
    dist.all_reduce(nw, op=dist.ReduceOp.MAX)
    out["push_nwg"] = int(nw[0])
    if count and engine == "kernel":
        # every rank joins the passes' rounds; the sampling ranks (the lowest
        # on each bus id) must hold the tool, or no rank runs them
        buses = [d[3] for d in descs]
        samplers = [r for r in range(world) if r == min(q for q in range(world) if buses[q] == buses[r])]
        have = [None] * world
        dist.all_gather_object(have, prof is not None)
        missing = [r for r in samplers if not have[r]]
        if missing:
            out["counters"] = {"error": f"the counter tool is not running on sampling rank(s) {missing}"}
        else:
            errs = []
            out["counters"] = link_counters(mpx, prof, torch, dist, c, rounds, rank, world, tx, rx, nbytes, iters,
                                            nwg, stream, buses, errs)
            if errs:
                out["counters"]["transfer_errors"] = errs[:3]
    ll_old = os.environ.get("MPX_LL_MAX")
    if latency:
        # after the headline: a failure here costs its own numbers only
        errs = []
        if engine == "kernel":
            # the node's own LL threshold first: everything below runs with it
            out["ll_vs_bulk_half_rtt_us"], out["ll_max"] = choose_ll_max(
                mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, [d[4] for d in descs], errs)
            os.environ["MPX_LL_MAX"] = str(out["ll_max"])
        out["small_message_check"] = small_message_check(mpx, torch, dist, c, rounds, rank, world, tx, rx, nbytes,
                                                         errs)
        g, peer = round_role(rounds, 0, rank)
        dist.barrier()
        lat = torch.tensor([safe_wall(c, errs, mpx.MODE_PINGPONG, g, rank, peer, LATENCY_ITERS, tx, rx, 8)],
                           dtype=torch.float64)
        dist.all_reduce(lat, op=dist.ReduceOp.MAX)
        out["pingpong_8B_half_rtt_us"] = finite(float(lat[0]) / (2 * LATENCY_ITERS) * 1e6, 3)
        out["pair_pingpong_8B_half_rtt_us"] = pair_latency(mpx, torch, dist, c, rounds, rank, world, tx, rx, errs)
        out["round0_sweep"] = round0_sweep(mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, errs)
        if nbytes >= HBV3_BYTES:
            out["hbv3_rounds"] = hbv3_rounds(mpx, torch, dist, c, rounds, rank, world, tx, rx, errs,
                                             phases=engine == "kernel")
        if engine == "kernel":
            out["stage"] = staged_vs_unstaged(mpx, torch, dist, c, rounds, rank, tx, rx, nbytes, iters, nwg, stream,
                                              descs[round_role(rounds, 0, rank)[1]][1],
                                              descs[round_role(rounds, 0, rank)[1]][2], errs)
            # last: a pull failure (e.g. a peer's tx not mapped) breaks only
            # what comes after it on this context
            out["push_vs_pull"] = push_vs_pull(mpx, torch, dist, c, rounds, rank, world, tx, rx, nbytes, nwg, stream,
                                               [d[1] for d in descs], [d[2] for d in descs], errs)
        every = [None] * world
        dist.all_gather_object(every, errs[:3])
        if any(every):
            out["extras_errors"] = {str(r): e for r, e in enumerate(every) if e}
    if ll_old is None:
        os.environ.pop("MPX_LL_MAX", None)
    else:
        os.environ["MPX_LL_MAX"] = ll_old
    dist.barrier()
    c.close()
    dist.barrier()   # see above: all imports closed before the next allocation
    return out


def pairs_with_fallback(mpx, torch, dist, engine, rank, world, dev, nbytes, iters, steps, warmup, barrier_sync,
                        extras: dict, latency: bool = True, prof=None, count: bool = False) -> tuple[dict, str]:
    """pairs_bench on `engine`; if the kernel engine fails (payload
    validation, or a device timeout on any rank in validation or in the timed
    steps), measure the SDMA engine instead and say so: an explicit, labelled
    fallback, never a silent one."""
    res = pairs_bench(mpx, torch, dist, engine, rank, world, dev, nbytes, iters, steps, warmup, barrier_sync,
                      latency=latency, prof=prof, count=count)
    engine_used = engine
    if res.get("error") and engine == "kernel":
        extras["kernel_engine_error"] = res["error"]
        # SDMA needs the same IPC mappings as the kernel engine; RCCL maps its
        # own buffers, so it is the last resort when IPC itself failed
        for fb_engine in ("sdma", "rccl"):
            fb = pairs_bench(mpx, torch, dist, fb_engine, rank, world, dev, nbytes, iters, steps, warmup,
                             barrier_sync, latency=latency)
            if not fb.get("error"):
                res, engine_used = fb, f"{fb_engine} (fallback: kernel engine failed, extras.kernel_engine_error)"
                break
            extras[f"{fb_engine}_engine_error"] = fb["error"]
    if res.get("error"):
        errs = [f"{engine}: {res['error']}"] + [f"{k[:-len('_engine_error')]}: {v}" for k, v in extras.items()
                                               if k.endswith("_engine_error") and not k.startswith(engine)]
        raise SystemExit("pairs bench failed: " + "; ".join(errs))
    return res, engine_used


class SpinBarrierDist:
    """torch.distributed as the pairs path uses it, with barrier() replaced
    by the node-local spin barrier (mpx/spin.py): the barrier in front of
    every timed loop (mpi_perf.c:499) then lets the ranks leave within about
    a microsecond, as MPI's intra-node barrier does, instead of a gloo TCP
    round trip apart.  Collectives that carry data stay gloo's."""

    def __init__(self, dist, spin):
        self._dist, self._spin = dist, spin

    def barrier(self):
        self._spin.wait()

    @property
    def spin(self):
        """the spin barrier itself (start_after_barrier waits on it from C)"""
        return self._spin

    def __getattr__(self, k):
        return getattr(self._dist, k)


def spin_barrier_dist(dist, rank: int, world: int):
    """(SpinBarrierDist, spin) when every rank opened the shm barrier, else
    (dist, None): every rank decides alike."""
    from mpx import spin as sp
    # one name per job on this node: its rendezvous address, port and size
    # (ranks started by hand, as tools/node_profile.sh does, have different
    # parents, so the launcher's pid cannot name it)
    name = "/mpxbar-bench-{}-{}-{}".format(os.environ.get("MASTER_ADDR", "x").replace("/", "_"),
                                           os.environ.get("MASTER_PORT", "0"), world)
    s, err = None, ""
    try:
        if rank == 0:
            sp.unlink(name)                       # a stale one from a killed run
            s = sp.SpinBarrier(name, world, True)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    dist.barrier()
    try:
        if rank != 0:
            s = sp.SpinBarrier(name, world, False)
    except Exception as e:  # noqa: BLE001
        err = str(e)
    flags = [None] * world
    dist.all_gather_object(flags, err)
    if rank == 0:
        sp.unlink(name)                           # every rank has it mapped (or gave up)
    if any(flags):
        print(f"[bench] spin barrier unavailable, gloo barriers: {[f for f in flags if f][0]}", file=sys.stderr)
        if s is not None:
            s.close()
        return dist, None
    return SpinBarrierDist(dist, s), s


def quiet_stdout() -> int:
    """Route fd 1 to stderr for the rest of the run and return a duplicate
    of the real stdout: libraries print banners there (RCCL's version block
    at communicator init, HIP / RCCL debug output), and the driver reads
    stdout for the ONE JSON line, which emit() writes to the duplicate."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return real


def emit(fd: int, line: dict) -> None:
    os.write(fd, (json.dumps(line) + "\n").encode())


def main() -> None:
    out_fd = quiet_stdout()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--engine", default="kernel", choices=["kernel", "sdma", "rccl"])
    ap.add_argument("--bytes", type=int, default=0, help="message bytes (default: 1 GiB at N=1, 4 MiB at N>1)")
    ap.add_argument("--iters", type=int, default=0, help="transfers per step (default 10 at N=1, 500 at N>1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true")
    ap.add_argument("--no-counters", action="store_true", help="no in-process hardware counters (mpx/counters.py)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")

    one = world == 1
    nbytes = args.bytes or ((1 << 30) if one else (4 << 20))
    iters = args.iters or (10 if one else 500)

    if os.environ.get("MPX_BENCH_ONE_GPU") and world > 1:
        # All ranks on one card: every process's HW queues share the card's
        # queue slots.  At N = 8 the default (4 per process, plus each rank's
        # CU-masked stream) oversubscribes them; a queue the scheduler has
        # not mapped cannot run the half of a pair its peer is waiting on,
        # and the peer's device deadline fires.  One queue per process (the
        # CU-masked rank stream keeps its own) fits.  Set before HIP starts.
        os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
    # CPU baseline first, before this process touches the GPU: N = 1, two
    # bound ranks at 1 GiB x 40 (~1.7 s per run on the box, 6 runs: ~10 s,
    # ~20 s of CPU work on the two cores); N >= 2,
    # the reference in run-hbv3's layout at the headline's B and iterations
    # (the other ranks wait in the process-group init meanwhile)
    cpu = None
    prof_var = under_profiler()
    if rank == 0 and not args.no_cpu_baseline and prof_var:
        # Under rocprofv3 the profiler's preload and ROCP_* variables would
        # pass through mpiexec to oracle/ref_wrap.sh, whose `exec` would then
        # follow a GPU initialisation (with --pmc the preload initialises the
        # GPU): the reference legs are not started
        cpu = dict(value=None, unit="GB/s", cores=0, kind="reference",
                   sample=f"not run: this process runs under a profiler ({prof_var} set)")
    elif rank == 0 and not args.no_cpu_baseline:
        _ref_deadline[0] = time.monotonic() + REF_BUDGET_S
        cpu = cpu_baseline(nbytes, CPU_BASELINE_ITERS, 6) if one else cpu_baseline_pairs(world, nbytes, iters, 6)
        # BASELINE config 1 itself (the reference's 2-rank ping-pong at 8 B
        # and 4 MiB) beside every line, whatever the workload
        pp = cpu_baseline_pingpong()
        if cpu is not None and pp is not None:
            cpu["config1_pingpong"] = pp
        # no process of the reference legs may outlive them (run_reference
        # kills their groups): the census says so before any GPU call
        cpu_left = descendants()
        if cpu is not None:
            cpu["processes_left_by_baseline"] = cpu_left

    import torch
    import mpx
    from mpx import counters

    # In-process counters (roofline.traffic): the tool registers before the
    # first HIP call of this process (torch is imported, HIP not started yet)
    prof, prof_note = None, counters_skip_reason(args)
    if prof_note is None and os.environ.get("MPX_BENCH_ONE_GPU") and world > 2:
        # One-GPU rehearsal beyond a single pair: not sampled.  The device
        # counting service reads the counters of ITS process's work here
        # (rank 0 alone read 0.25 x the card's pushes at N = 8 = its own
        # share, profiles/r04_bench_n8_onegpu_rehearsal_rank0_tool.json), and
        # the tool in every process cost the card's shared queue slots a 5x
        # slowdown (r04_bench_n8_onegpu_rehearsal_tool_everywhere.json).  On
        # a node, each GPU's one process is its sampler; at N = 2 here the
        # sampler (rank 0) is the side that pushes.
        prof_note = "one-GPU rehearsal with more than one pair: not sampled (per-process counters, shared queues)"
    count = prof_note is None            # agreed across ranks below (environments may differ)
    if prof_note is None:
        try:
            counters.register()
            prof = counters
        except counters.CounterError as e:
            prof_note = f"counters not registered: {e}"

    # MPX_BENCH_ONE_GPU=1: rehearse the N>1 path with every rank on GPU 0
    # (two processes on one card share it; the IPC + mailbox path is the same)
    # A launcher that gives each process only its own GPU (HIP_VISIBLE_DEVICES
    # per rank) leaves device 0 as that GPU.
    dev = 0 if os.environ.get("MPX_BENCH_ONE_GPU") or torch.cuda.device_count() <= local else local
    if one_gpu_push_cap(world) and "MPX_PUSH_WG" not in os.environ:
        # the default push width too (validation, steps, sweep), before the
        # library first reads it
        os.environ["MPX_PUSH_WG"] = str(one_gpu_push_cap(world))
    torch.cuda.set_device(dev)
    torch.cuda.synchronize()                 # HIP (and the counter tool) started
    if prof is not None and not prof.ready():
        prof_note = f"counter tool not initialised: {prof.error()}"
        prof = None
    dist = None
    if not one:
        import datetime

        import torch.distributed as dist
        # a rank that dies must not leave the others in a 30-minute gloo wait
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=180))
        # the counter passes need every rank (they re-run every round): only
        # when every rank can take part — ranks started by hand may differ,
        # e.g. tools/node_profile.sh runs some under rocprofv3 and some not
        flags = [None] * world
        dist.all_gather_object(flags, count)
        if count and not all(flags):
            prof_note = "not sampled: another rank runs without the in-process counters (under a profiler or --no-counters)"
        count = all(flags)

    def barrier_sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # N > 1: the per-round barriers of the pairs path spin in shared memory
    pdist, spin = (spin_barrier_dist(dist, rank, world) if dist is not None else (None, None))

    extras = {}
    if one:
        workload = "local_d2d_copy"
        c = mpx.Context(1, args.engine)
        src, dst = c.alloc(0, nbytes), c.alloc(0, nbytes)
        key = mpx.pattern_key(mpx.PATTERN_SEED, 0, 0, 0)
        c.fill(src, nbytes, mpx.FILL_SPLITMIX, key)
        for _ in range(args.warmup):
            c.copy(0, dst, src, nbytes, iters)
        dev_s, launches = 0.0, 0
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            t = c.copy(0, dst, src, nbytes, iters)
            dev_s += t.device_s
            launches += t.launches
        barrier_sync()
        elapsed = time.perf_counter() - t0
        assert c.checksum(dst, nbytes) == c.checksum(src, nbytes), "copy output differs from its input"
        total = nbytes * iters * args.steps
        per_launch = dev_s / max(launches, 1)
        algo = 2 * nbytes   # read B + write B per launch
        achieved = algo / per_launch / 1e9
        roof = dict(bound="hbm", achieved=round(achieved, 1), peak=HBM_PEAK_GBPS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBPS, 4), traffic=None, kernel="k_copy<1,nt,nt> (one 16-B unit per lane, n/4 KiB blocks)",
                    avg_launch_us=round(per_launch * 1e6, 2), algorithmic_bytes_per_launch=algo)
        if prof is not None:
            try:
                tr = copy_traffic(prof, c, src, dst, nbytes, iters, mpx.bus_id(0))
                roof["traffic"] = tr["hbm_bytes_per_launch"]
                roof["traffic_source"] = tr["source"]
                roof["traffic_detail"] = tr
            except Exception as e:  # noqa: BLE001
                prof_note = f"counter pass failed: {type(e).__name__}: {e}"[:300]
        committed = traffic_from_profile(workload)
        if committed and committed.get("bytes") == nbytes:
            # the rocprofv3 --pmc passes of the same command, committed: the
            # cross-check of the in-run figure (and the figure when it is off)
            roof["traffic_rocprofv3"] = dict(hbm_bytes_per_launch=committed.get("hbm_bytes_per_launch"),
                                             source=committed.get("source"))
            if roof["traffic"] is None:
                roof["traffic"] = committed.get("hbm_bytes_per_launch")
                roof["traffic_source"] = committed.get("source")
        if prof_note:
            roof["traffic_note"] = prof_note
        config = dict(workload=workload, bytes=nbytes, iters_per_step=iters, engine="kernel (k_copy)",
                      parallelism="single GPU")
        metric_unit = "GB/s"
        if not args.no_extras:
            extras["copy_sweep"] = copy_sweep(mpx, c, src, dst, nbytes)
            extras["sustained_copy"] = sustained_copy(c, src, dst, nbytes)
            lat = loopback_pair(mpx, "kernel", mpx.MODE_PINGPONG, 8, 5000)
            extras["loopback_pingpong_8B_half_rtt_us"] = round(lat["per_iter_us"] / 2, 3)
            uni = loopback_pair(mpx, "kernel", mpx.MODE_UNIDIR, 4 << 20, 200)
            extras["loopback_unidir_4MiB_GBps"] = round((4 << 20) / (uni["per_iter_us"] * 1e-6) / 1e9, 2)
            uni = loopback_pair(mpx, "kernel", mpx.MODE_UNIDIR, 4 << 20, 200, pull=True)
            extras["loopback_pull_unidir_4MiB_GBps"] = round((4 << 20) / (uni["per_iter_us"] * 1e-6) / 1e9, 2)
            extras["runtime_copy_hbm_GBps"] = runtime_copy_rate(torch, nbytes, iters)
        ceil = hbm_one_direction_ceiling()
        if ceil:
            extras["hbm_one_direction_ceiling_GBps"] = ceil
        c.close()
    else:
        workload = "all_pairs_rounds_unidir"
        metric_unit = "GB/s"
        # --no-extras: nothing after the timed steps (profiling runs select
        # the timed launches as the last ones)
        res, engine_used = pairs_with_fallback(mpx, torch, pdist, args.engine, rank, world, dev, nbytes, iters,
                                               args.steps, args.warmup, barrier_sync, extras,
                                               latency=not args.no_extras, prof=prof, count=count)
        elapsed, total = res["elapsed"], res["total"]
        achieved = res["per_pair_GBps"]
        roof = dict(bound="xgmi", achieved=round(achieved, 2), peak=XGMI_LINK_PEAK_GBPS, unit="GB/s",
                    frac=round(achieved / XGMI_LINK_PEAK_GBPS, 4), traffic=None,
                    peak_note=("one direction of one xGMI link under the per-direction reading (153.6 GB/s as both "
                               "directions summed, DESIGN.md §7, unsourced); frac_of_bidirectional_link is against "
                               "153.6, the per-direction figure SURVEY.md:361 states and extras.targets judges by"),
                    frac_of_bidirectional_link=round(achieved / XGMI_LINK_PEAK_BIDIR_GBPS, 4),
                    kernel="k_xfer (G1 side)" if engine_used == "kernel" else engine_used,
                    avg_launch_us=round(res["per_launch_s"] * 1e6, 2), algorithmic_bytes_per_launch=nbytes * iters,
                    device_clock=res.get("device_clock"))
        if os.environ.get("MPX_BENCH_ONE_GPU"):
            roof["rehearsal_note"] = ("one-GPU rehearsal: every rank on one card, so achieved is a loopback (HBM) "
                                      "rate and frac against the link peak says nothing about a link")
        # Link bytes of THIS run's sender launches, read in-process
        # (link_counters): per G1 launch, EA write requests not destined for
        # local DRAM x 64 B.  On the one-GPU rehearsal they are ~0 and the
        # local-DRAM figure carries the pushes.
        cnt = res.get("counters")
        if cnt and "error" not in cnt:
            roof.update(link_traffic(cnt))
            extras["counters"] = cnt
        else:
            roof["traffic_source"] = "not measured: " + ((cnt or {}).get("error") or prof_note or "no counter pass")
        nwg_used = res.get("push_nwg") or 0
        chunk = ((-(-nbytes // nwg_used)) + 15) // 16 * 16 if nwg_used else 0
        config = dict(workload=workload, bytes=nbytes, iters_per_step=iters, engine=engine_used,
                      rounds=world - 1, pairs_per_round=world // 2, parallelism=f"pairs{world // 2}",
                      validated_rounds=res["validated_rounds"], push=res.get("push", "default"),
                      push_nwg=nwg_used,
                      barrier=("node-local spin barrier in shared memory before every loop (mpx/spin.py)"
                               if spin is not None else "gloo"),
                      launch=("armed: each loop's kernel launched before its barrier, started by a host-memory "
                              "word after it (mpx_xfer_arm)" if engine_used == "kernel" else "inline"),
                      # bytes of tx each pushing workgroup holds in LDS (read once per call; 0 = tx read from HBM)
                      stage=chunk if (engine_used == "kernel" and 0 < chunk <= 60 << 10) else 0)
        if "ll_max" in res:
            config["ll_max"] = res["ll_max"]
            extras["ll_choice"] = dict(chosen_ll_max=res["ll_max"], half_rtt_us=res.get("ll_vs_bulk_half_rtt_us"),
                                       ll_bytes_written_per_payload_byte=LL_BYTES_PER_PAYLOAD_BYTE,
                                       rule="largest size up to which LL's half round trip is never above bulk's")
        if "stage" in res:
            extras["unidir_staged_vs_unstaged"] = dict(res["stage"], bytes=nbytes, iters=iters)
            extras["unidir_4MiB_unstaged_GBps"] = res["stage"].get("unidir_unstaged_GBps")
        if res.get("push_tune"):
            extras["push_tune_GBps_per_pair"] = res["push_tune"]
        extras["per_pair_unidir_GBps"] = round(achieved, 2)
        extras["pairs_covered"] = len(res.get("pair_GBps", {}))
        extras["pair_unidir_GBps"] = res.get("pair_GBps")
        extras["pair_unidir_GBps_min_max"] = res.get("pair_GBps_min_max")
        extras["round_aggregate_GBps"] = res.get("round_aggregate_GBps")
        if rank == 0 and not os.environ.get("MPX_BENCH_ONE_GPU") and torch.cuda.device_count() >= world:
            # the path every pair of the steps takes (one process per GPU:
            # local rank = GPU), so the first node run describes itself
            extras["link_table"] = link_table(mpx, all_pairs_rounds(world), list(range(world)))
        if "pingpong_8B_half_rtt_us" in res:
            extras["pingpong_8B_half_rtt_us"] = res["pingpong_8B_half_rtt_us"]
            extras["pair_pingpong_8B_half_rtt_us"] = res["pair_pingpong_8B_half_rtt_us"]
        if "extras_errors" in res:
            extras["pair_extras_errors"] = res["extras_errors"]
        if "small_message_check" in res:
            extras["small_message_check"] = res["small_message_check"]
        if "hbv3_rounds" in res:
            extras["hbv3_rounds_unidir"] = res["hbv3_rounds"]
        if "push_vs_pull" in res:
            extras["push_vs_pull"] = res["push_vs_pull"]
        if "round0_sweep" in res:
            extras["round0_sweep"] = res["round0_sweep"]
            bidir = res["round0_sweep"].get(f"nonblocking_{nbytes}")
            if bidir:   # -x 1 at B: both directions of the pair's link (2B per iteration)
                extras["per_pair_bidir_GBps"] = bidir["GBps"]

    value = total / elapsed / 1e9
    if not one:
        # each north_star target beside the number it judges (extras.targets)
        tg = {}
        if nbytes >= (4 << 20):
            tg["per_pair_unidir_GBps"] = link_target(achieved, nbytes)
        if extras.get("pingpong_8B_half_rtt_us") is not None:
            v = extras["pingpong_8B_half_rtt_us"]
            tg["pingpong_8B_half_rtt_us"] = dict(value=v, target=f"< {TARGET_HALF_RTT_US} us",
                                                 meets=v < TARGET_HALF_RTT_US)
        tg["all_pairs_aggregate_GBps"] = dict(value=round(value, 3), n_gpus=world, target="reported at 2/4/8 GPUs")
        lt = extras.get("link_table")
        if lt is not None:
            # the targets are per link: a pair that is not one xGMI hop is
            # named, and its rate is not a single link's
            tg["pairs_not_one_xgmi_hop"] = lt["not_one_xgmi_hop"]
        if os.environ.get("MPX_BENCH_ONE_GPU"):
            # every rank on GPU 0: loopback pairs, no xGMI link was measured
            for t in tg.values():
                for k in ("meets", "meets_per_direction_reading"):
                    if k in t:
                        t[k] = None
            tg["note"] = "MPX_BENCH_ONE_GPU rehearsal: loopback pairs on one GPU, not an xGMI measurement"
        extras["targets"] = tg
    line = {
        "metric": "per-pair xGMI GB/s at 4 MB + 8 B latency us; all-pairs aggregate GB/s at 2/4/8 GPUs",
        "value": round(value, 3),
        "unit": metric_unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": config,
        "roofline": roof,
        "cpu_baseline": cpu,
        "extras": extras,
    }
    if not one and not args.no_extras:
        # The comparison engines (BASELINE config 4: kernel vs SDMA vs RCCL)
        # run after the headline is measured, under a watchdog: should one of
        # them hang (an RCCL bootstrap cannot be interrupted), every rank
        # still ends and rank 0 still prints its line, without those numbers.
        done, lock = threading.Event(), threading.Lock()

        def on_deadline():
            with lock:
                if done.is_set():          # the extras finished in time
                    return
                if rank == 0:
                    extras["comparison_engines"] = f"abandoned after {EXTRAS_DEADLINE_S} s"
                    emit(out_fd, line)
                os._exit(0)

        dog = threading.Timer(EXTRAS_DEADLINE_S, on_deadline)
        dog.daemon = True
        dog.start()
        if config["engine"] == "kernel":
            # the same rounds at 64 MiB: the per-iteration protocol cost
            # (drain, flag, 1-byte ack) is then ~0.5 % of a push, so this is
            # the link rate the kernel engine reaches with B out of the
            # picture, the reference point for the 4 MiB headline's fraction
            r3 = pairs_bench(mpx, torch, pdist, "kernel", rank, world, dev, CEILING_BYTES, CEILING_ITERS, world - 1, 1,
                             barrier_sync, latency=False, tune=False)
            if r3.get("error"):
                extras["unidir_64MiB_per_pair_GBps"] = r3["error"]
            else:
                extras["unidir_64MiB_per_pair_GBps"] = round(r3["per_pair_GBps"], 2)
                extras["unidir_64MiB_pair_GBps_min_max"] = r3.get("pair_GBps_min_max")
                extras["headline_over_64MiB"] = round(achieved / r3["per_pair_GBps"], 4)
        # RCCL first: pairs_bench refuses it before ncclCommInitRank when two
        # ranks share a GPU (the one-GPU rehearsal), so no refused init can
        # slow what follows (round 3 had to run it last:
        # profiles/r03_pull_rounds_diag.jsonl)
        try:
            extras["rccl"] = mpx.rccl_version()   # the RCCL this process runs (torch's, when torch loaded it first)
        except Exception as e:  # noqa: BLE001
            extras["rccl"] = f"{type(e).__name__}: {e}"[:200]
        for eng, pull in (("rccl", False), ("sdma", False), ("kernel", True), ("sdma", True)):
            if not pull and config["engine"].startswith(eng):
                continue
            # 512 iterations: two graph-replayed SDMA chunks (run_sdma), no host-bound tail
            r2 = pairs_bench(mpx, torch, pdist, eng, rank, world, dev, nbytes, 512, world - 1, 1, barrier_sync,
                             latency=False, tune=False, pull=pull) if pull else \
                pairs_bench(mpx, torch, pdist, eng, rank, world, dev, nbytes, 512, world - 1, 1, barrier_sync,
                            latency=False)
            # every round's payloads checksummed on this engine before timing
            # it (BASELINE config 5); pull: the engine's MPX_XFER_PULL form
            # (the receiver loads / its stream copies the sender's tx)
            key = f"{eng}_pull" if pull else eng
            extras[f"{key}_aggregate_GBps"] = r2.get("error") or round(r2["total"] / r2["elapsed"] / 1e9, 3)
            extras[f"{key}_validated_rounds"] = r2.get("validated_rounds", 0)
        with lock:
            done.set()
        dog.cancel()
    if rank == 0:
        # exit census: this process's live descendants
        # as the line goes out (none expected: every reference leg's process
        # group was killed, and libmpx starts no process)
        extras["processes_at_line"] = descendants()
        emit(out_fd, line)
    if dist is not None:
        dist.barrier()
        if spin is not None:
            spin.close()
        dist.destroy_process_group()
    # Every context is finalized and the line is out: the pooled rank streams
    # are destroyed here, in the program's own flow, and the process then
    # ends through its normal exit (the HIP runtime's and any profiler's or
    # counter tool's exit-time teardown included).  Round 4 ended here with
    # os._exit(0): the teardown had faulted inside rocprofiler-sdk's
    # finalizer while rank streams were alive (profiles/r04_exit_segv_stack.txt),
    # and the destroy had stalled 1 processes-mode exit in 4 — root-caused in
    # round 5 (DESIGN.md §5 "Exit") and closed by mpx_shutdown's fence.
    # the marker tools/node_profile.sh tells an exit-time stall by (a rank
    # that printed it and then ran out of time finished its transfers)
    print(f"[bench] rank {rank}: done, shutting down", file=sys.stderr)
    sys.stdout.flush()
    sys.stderr.flush()
    mpx.shutdown()
    left = descendants()
    print(f"[bench] rank {rank}: processes left at exit: {left if left else 'none'}", file=sys.stderr)


if __name__ == "__main__":
    main()
