"""bench.py's transfer helpers on CPU, with stand-in objects (no GPU, no
libmpx calls): the failure paths the advisor flagged in round 4."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import bench  # noqa: E402


class Ctx:
    """records the calls bench.safe_wall makes on an mpx context"""

    def __init__(self, fail_xfer=None):
        self.log, self.fail_xfer = [], fail_xfer

    def xfer(self, mode, group, me, peer, iters, tx, rx, n, **kw):
        self.log.append(("xfer", me))
        if self.fail_xfer:
            raise self.fail_xfer

        class T:
            wall_s = 0.5
        return T()

    def disarm(self, r):
        self.log.append(("disarm", r))


class Dist:
    def __init__(self, fail=None):
        self.fail = fail

    def barrier(self):
        if self.fail:
            raise self.fail


def test_safe_wall_disarms_when_the_start_never_came():
    """The barrier in front of an armed transfer fails (a spin-barrier
    TimeoutError): the call is cancelled, so the rank is not left armed."""
    c, errs = Ctx(), []
    w = bench.safe_wall(c, errs, 2, 1, 3, 4, 10, None, None, 4096, barrier=Dist(TimeoutError("spin barrier")))
    assert w == float("inf") and ("disarm", 3) in c.log and ("xfer", 3) not in c.log
    assert errs and "TimeoutError" in errs[0]


def test_safe_wall_disarm_after_a_failed_transfer_is_harmless():
    """The transfer itself fails (the call was started: libmpx already
    dropped it): disarm is still issued and is a no-op there."""
    c, errs = Ctx(fail_xfer=RuntimeError("device wait timed out")), []
    assert bench.safe_wall(c, errs, 2, 1, 0, 1, 10, None, None, 8) == float("inf")
    assert c.log == [("xfer", 0), ("disarm", 0)]


def test_safe_wall_success_does_not_disarm():
    c, errs = Ctx(), []
    assert bench.safe_wall(c, errs, 2, 1, 0, 1, 10, None, None, 8, barrier=Dist()) == 0.5
    assert c.log == [("xfer", 0)] and not errs


def test_config1_pingpong_baseline_shape():
    """The compiled reference's 2-rank ping-pong (BASELINE config 1) that
    bench.py puts beside its N = 1 and N >= 2 lines: 8 B half round trip and
    4 MiB rate, two cores, median of runs 1..5."""
    pp = bench.cpu_baseline_pingpong()
    assert pp is not None, "oracle/_ref not built (python -c 'import __graft_entry__ as g; g.build()')"
    assert pp["cores"] == 2 and pp["kind"] == "reference" and pp["loop"].startswith("ping-pong")
    assert 0 < pp["half_rtt_us_8B"] < 100 and 0 < pp["GBps_4MiB"] < 1000, pp


def test_config1_pingpong_binds_like_the_launchers_and_leaves_no_process():
    """the reference's ranks run bound, one physical
    core each on one NUMA node (`-bind-to user:<cores> -membind bind:<node>`,
    as scripts/run-1-pair.sh:62 and run-hbv3.sh:23 bind them), each run's
    spread is in the line, and nothing of mpiexec's process group outlives
    the leg (no descendant of this process, none named as left over)."""
    pp = bench.cpu_baseline_pingpong()
    assert pp is not None
    assert pp["binding"].startswith("-bind-to user:") and "-membind bind:" in pp["binding"], pp["binding"]
    assert len(pp["core_list"]) == 2 and len(set(pp["core_list"])) == 2
    assert pp["leftover_processes"] == [] and bench.descendants() == []
    for key in ("half_rtt_us_8B", "GBps_4MiB"):
        s = pp[key + "_per_run"]
        assert s["runs"] == 5 and s["min"] <= pp[key] == s["median"] <= s["max"], (key, s)


def _fake_sysfs(root, nodes, siblings):
    for n, cpus in nodes.items():
        d = root / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cpus + "\n")
    for c, sib in siblings.items():
        d = root / "cpu" / f"cpu{c}" / "topology"
        d.mkdir(parents=True)
        (d / "thread_siblings_list").write_text(sib + "\n")


def test_reference_cores_one_node_one_thread_per_core(tmp_path, monkeypatch):
    """Two nodes of 12 cores with SMT siblings 24..47: node 0's physical
    cores, siblings dropped, the first 8 skipped when the node has 8 + n
    (run-hbv3.sh:23's `--cpu-list 8..17`), else from its first core; only
    CPUs in the affinity mask count."""
    nodes = {0: "0-11,24-35", 1: "12-23,36-47"}
    sib = {c: f"{c % 24},{c % 24 + 24}" for c in range(48)}
    _fake_sysfs(tmp_path, nodes, sib)
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(48)))
    r = bench.reference_cores(2, str(tmp_path))
    assert r["numa_node"] == 0 and r["cores"] == [8, 9] and r["complete"], r
    r = bench.reference_cores(8, str(tmp_path))
    assert r["cores"] == list(range(8)) and r["skipped_first"] == 0, r
    # node 0 outside the mask: the node with the most allowed physical cores
    monkeypatch.setattr(bench.os, "sched_getaffinity", lambda pid: set(range(12, 24)) | set(range(36, 48)))
    r = bench.reference_cores(4, str(tmp_path))
    assert r["numa_node"] == 1 and r["cores"] == [20, 21, 22, 23] and r["complete"], r   # 12 >= 8 + 4: skip 8


def test_reference_legs_not_started_under_a_profiler(monkeypatch):
    """under rocprofv3 the reference's mpiexec chain would
    exec ref_wrap.sh after the profiler's preload initialised the GPU; bench
    names the profiler variable and starts no reference leg."""
    monkeypatch.setenv("ROCP_TOOL_LIBRARIES", "/x/librocprofiler-sdk-tool.so")
    assert bench.under_profiler() == "ROCP_TOOL_LIBRARIES"
    src = open(bench.__file__).read()
    main = src[src.index("def main()"):]
    assert main.index("prof_var = under_profiler()") < main.index("cpu_baseline(nbytes")


def test_run_reference_with_an_explicit_placement():
    """tools/ref_placement.py's A/B: run_reference with a caller's placement
    runs that one form (here mpiexec's default), names it, and leaves no
    process behind."""
    r = bench.run_reference(2, 1, ["-u", "1", "-b", "65536", "-i", "50", "-r", "3"], 60, placement=[])
    assert r["rc"] == 0 and r["binding"].startswith("none") and r["cores"] is None, r
    assert len(r["times"]) == 2 and r["leftover"] == [] and bench.descendants() == []


def test_run_tracked_names_and_kills_an_orphan_in_its_own_session():
    """hydra puts every proxy and rank in a session of its own (setsid), so
    bench.run_tracked follows the parent tree while the command runs: a
    process that outlives the command in a new session is named and
    killed."""
    r = bench.run_tracked(["bash", "-c", "setsid sleep 30 & sleep 0.6; exit 0"], 20)
    assert r["rc"] == 0 and not r["timed_out"] and r["tracked"] >= 1
    assert [q["name"] for q in r["leftover"]] == ["sleep"], r
    import time
    time.sleep(0.2)
    procs = bench._procs()
    pid = r["leftover"][0]["pid"]
    assert pid not in procs or procs[pid]["state"] == "Z" or procs[pid]["name"] != "sleep"


def test_run_tracked_time_limit_kills_the_tree():
    r = bench.run_tracked(["bash", "-c", "sleep 30 & sleep 30"], 0.6)
    assert r["timed_out"] and r["rc"] != 0 and "timed out" in r["stderr"] and r["leftover"] == [], r


def test_reference_legs_share_one_time_budget(monkeypatch):
    """At N >= 2 the other ranks wait in the process-group init (180 s) while
    rank 0 runs the reference legs: they share REF_BUDGET_S, and a leg that
    finds the budget spent runs nothing and says so."""
    import time
    assert bench.REF_BUDGET_S < 180
    monkeypatch.setattr(bench, "_ref_deadline", [time.monotonic()])
    r = bench.run_reference(2, 1, ["-u", "1", "-b", "64", "-i", "5", "-r", "2"], 60)
    assert r["rc"] is None and "budget is spent" in r["stderr"] and r["times"] == [], r
    assert bench.cpu_baseline_pingpong()["GBps_4MiB"] is None
