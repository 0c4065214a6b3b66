"""bench.py main() at N = 2 on CPU over gloo (tests/bench_main_worker.py):
rank 0 prints exactly one JSON line carrying the contract's keys; when a
comparison engine hangs (an RCCL bootstrap that never returns) the watchdog
still ends every rank with status 0 and rank 0 still prints its line."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "extras"}


def run(scenario, world=2, extra_env=None):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ps = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **(extra_env or {}))
        ps.append(subprocess.Popen([sys.executable, os.path.join(HERE, "bench_main_worker.py"), scenario, "--gpus",
                                    str(world), "--steps", "3", "--warmup", "1"], stdout=subprocess.PIPE,
                                   stderr=subprocess.PIPE, text=True, env=env))
    outs = [p.communicate(timeout=120) for p in ps]
    return [p.returncode for p in ps], outs


def lines(stdout):
    return [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]


def test_one_json_line_with_the_contract_keys():
    rcs, outs = run("ok")
    assert rcs == [0, 0], [o[1][-600:] for o in outs]
    got = lines(outs[0][0])
    assert len(got) == 1 and not lines(outs[1][0])
    # library output on fd 1 (the stand-in's RCCL banner) goes to stderr:
    # stdout holds the JSON line and nothing else
    assert outs[0][0].count("\n") == 1 and outs[1][0] == ""
    assert "RCCL version" in outs[0][1]
    d = got[0]
    assert KEYS <= set(d)
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak" and d["unit"] == "GB/s"
    assert d["config"]["workload"] == "all_pairs_rounds_unidir" and d["config"]["engine"] == "kernel"
    assert d["roofline"]["bound"] == "xgmi" and d["roofline"]["peak"] == 76.8
    assert "frac_of_bidirectional_link" in d["roofline"]
    # the target's primary verdict is against the stated 153.6 GB/s per
    # direction (SURVEY.md:361); the per-direction reading beside it
    tg = d["extras"]["targets"]["per_pair_unidir_GBps"]
    assert tg["meets"] == (tg["value"] >= 0.85 * 153.6) and "SURVEY.md:361" in tg["target"]
    assert tg["meets_per_direction_reading"] == (tg["value"] >= 0.85 * 76.8)
    assert isinstance(d["extras"]["sdma_aggregate_GBps"], float)
    # the pulled forms of the kernel and SDMA engines over the same rounds
    assert isinstance(d["extras"]["kernel_pull_aggregate_GBps"], float), d["extras"]
    assert isinstance(d["extras"]["sdma_pull_aggregate_GBps"], float)
    assert isinstance(d["extras"]["rccl_aggregate_GBps"], float)
    # the comparison engines checksum every round before timing it (config 5)
    assert d["extras"]["sdma_validated_rounds"] == 1 and d["extras"]["rccl_validated_rounds"] == 1
    assert d["extras"]["rccl"]["release"] == "2.27.7"
    # the reference itself beside the N >= 2 line: run-hbv3's layout (N ranks,
    # -p N/2 -u 1) at the headline's B and iterations, under MPICH shm
    cb = d["cpu_baseline"]
    assert cb["kind"] == "reference" and cb["cores"] == 2 and cb["value"] > 0, cb
    assert "-p 1 -u 1 -b 4194304 -i 500" in cb["sample"]
    # BASELINE config 1 beside it: the reference's ping-pong at 8 B and 4 MiB
    pp = cb["config1_pingpong"]
    assert pp["cores"] == 2 and pp["kind"] == "reference" and "-b 8 -i 20000" in pp["sample"]
    assert 0 < pp["half_rtt_us_8B"] < 100 and 0 < pp["GBps_4MiB"] < 1000, pp
    # link bytes from the in-process counters (the stand-in's counts: 990
    # link requests of 64 B per sampling rank and pass, 2 samplers, 1 launch)
    # are 6e-5 x the pushed 4 MiB x 500 on two distinct GPUs: the self-check
    # prints no traffic figure, with the raw counters and the reason
    cnt = d["extras"]["counters"]
    assert cnt["link_bytes_per_launch"] == 2 * 990 * 64 and cnt["samplers"] == 2
    assert d["roofline"]["traffic"] is None and d["roofline"]["traffic_check"] == "failed"
    assert d["roofline"]["traffic_raw"]["TCC_EA0_WRREQ_sum"] == 2000.0
    assert d["config"]["ll_max"] == 8192 and d["extras"]["ll_choice"]["chosen_ll_max"] == 8192
    assert d["extras"]["unidir_4MiB_unstaged_GBps"] is not None
    assert d["extras"]["hbv3_rounds_unidir"]["phases_us_median"]["g1"]["kernel_s"] == 1.0
    assert d["config"]["barrier"].startswith("node-local spin barrier") and d["config"]["launch"].startswith("armed")
    assert d["roofline"]["device_clock"].startswith("kernel-span (armed")


def test_exit_path_with_and_without_a_profiler():
    """Every rank destroys its rank streams (mpx_shutdown) after its line and
    returns through the normal exit, profiled or not (round 5: the
    os._exit(0) of round 4 is gone, DESIGN.md §5 "Exit").  Under rocprofv3
    (one of its variables set; ROCPROF_COUNTERS here — the tool-library
    variable would make the SDK in this process try to load that library)
    the in-process counters stand aside (one rocprofiler tool per process)."""
    for env in (None, {"ROCPROF_COUNTERS": "FETCH_SIZE"}):
        rcs, outs = run("ok", extra_env=env)
        assert rcs == [0, 0], [o[1][-600:] for o in outs]
        assert all("MAIN_RETURNED shutdown=True" in o[1] for o in outs), [o[1][-300:] for o in outs]
    d = lines(outs[0][0])[0]
    assert d["roofline"]["traffic"] is None and "under a profiler" in d["roofline"]["traffic_source"]


def test_hung_comparison_engine_cannot_cost_the_line():
    rcs, outs = run("rccl_hangs")
    assert rcs == [0, 0], [o[1][-600:] for o in outs]
    got = lines(outs[0][0])
    assert len(got) == 1
    d = got[0]
    assert d["extras"]["comparison_engines"] == "abandoned after 5 s"
    # RCCL runs first among the comparison engines: nothing after it ran, but
    # the headline and everything measured before the watchdog are in the line
    assert "rccl_aggregate_GBps" not in d["extras"] and "sdma_aggregate_GBps" not in d["extras"]
    assert d["value"] > 0 and d["extras"]["counters"]["samplers"] == 2


def test_every_pair_of_four_ranks_has_a_rate():
    """N = 4, 3 steps = the 3 rounds: all 6 pairs get a G1 launch rate
    (bytes x iters / that rank's device time) and every round an aggregate;
    every pair's link is described (mpx_link_info, the stand-in's GPUs 1-2
    are two hops apart and named in the targets)."""
    rcs, outs = run("ok", world=4)
    assert rcs == [0] * 4, [o[1][-600:] for o in outs]
    d = lines(outs[0][0])[0]
    e = d["extras"]
    lt = e["link_table"]
    assert len(lt["pairs"]) == 6 and {tuple(sorted(v["gpus"])) for v in lt["pairs"].values()} == {
        (a, b) for a in range(4) for b in range(a + 1, 4)}
    bad = [k for k, v in lt["pairs"].items() if sorted(v["gpus"]) == [1, 2]]
    assert lt["not_one_xgmi_hop"] == bad and len(bad) == 1
    assert e["targets"]["pairs_not_one_xgmi_hop"] == bad
    assert e["pairs_covered"] == 6 and len(e["round_aggregate_GBps"]) == 3
    pairs = {tuple(sorted(map(int, k.split(">")))) for k in e["pair_unidir_GBps"]}
    assert pairs == {(a, b) for a in range(4) for b in range(a + 1, 4)}
    launch = d["config"]["bytes"] * d["config"]["iters_per_step"]
    for k, v in e["pair_unidir_GBps"].items():
        g1 = int(k.split(">")[0])
        assert abs(v - launch / (0.001 * (1 + g1)) / 1e9) < 0.01     # the stand-in's device time
    assert e["pair_unidir_GBps_min_max"] == [min(e["pair_unidir_GBps"].values()),
                                             max(e["pair_unidir_GBps"].values())]


def test_every_pair_has_a_latency():
    rcs, outs = run("ok", world=4)
    assert rcs == [0] * 4, [o[1][-600:] for o in outs]
    lat = lines(outs[0][0])[0]["extras"]["pair_pingpong_8B_half_rtt_us"]
    assert {tuple(sorted(map(int, k.split(">")))) for k in lat} == {(a, b) for a in range(4) for b in range(a + 1, 4)}
    assert all(v == round(0.002 / (2 * 10_000) * 1e6, 3) for v in lat.values())    # the stand-in's wall time


def test_hbv3_shaped_rounds():
    """run-hbv3's -u 1 -b 456131 -i 10 over every round (config 4's short
    loop): one aggregate per round, median of the passes."""
    rcs, outs = run("ok", world=4)
    assert rcs == [0] * 4, [o[1][-600:] for o in outs]
    h = lines(outs[0][0])[0]["extras"]["hbv3_rounds_unidir"]
    assert h["bytes"] == 456131 and h["iters"] == 10 and len(h["round_aggregate_GBps"]) == 3
    # the stand-in's wall time is 2 ms: 2 pairs x 456131 B x 10 / 2 ms
    assert all(abs(v - 2 * 456131 * 10 / 0.002 / 1e9) < 0.05 for v in h["round_aggregate_GBps"])


def test_failure_after_the_headline_keeps_the_line():
    """Rank 1's 8 B ping-pong fails (a device deadline) after the timed steps:
    every rank still runs every later collective, the headline and the other
    extras stand, and the failed numbers are null with the error reported."""
    rcs, outs = run("latency_fails")
    assert rcs == [0, 0], [o[1][-600:] for o in outs]
    d = lines(outs[0][0])[0]
    e = d["extras"]
    assert d["value"] > 0 and d["config"]["engine"] == "kernel"
    assert e["pingpong_8B_half_rtt_us"] is None
    assert all(v is None for v in e["pair_pingpong_8B_half_rtt_us"].values())
    assert "LL ping-pong" in e["pair_extras_errors"]["1"][0]
    assert e["round0_sweep"]["unidir_4194304"]["GBps"] > 0
    assert isinstance(e["sdma_aggregate_GBps"], float)
    json.dumps(d, allow_nan=False)          # strict JSON: no Infinity / NaN


def test_failed_timed_step_falls_back_to_sdma_with_a_label():
    """Rank 1's kernel-engine transfer fails inside the timed steps: rank 0
    keeps joining the step barriers, both agree on the error afterwards, and
    the SDMA engine carries the line, labelled, with the kernel error kept."""
    rcs, outs = run("kernel_step_fails")
    assert rcs == [0, 0], [o[1][-600:] for o in outs]
    d = lines(outs[0][0])[0]
    assert d["config"]["engine"].startswith("sdma (fallback")
    assert "timed step" in d["extras"]["kernel_engine_error"] and "rank 1" in d["extras"]["kernel_engine_error"]
    assert d["value"] > 0
