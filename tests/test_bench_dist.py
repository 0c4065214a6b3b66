"""bench.py's N > 1 path (one process per GPU) rehearsed on CPU: world size 2
and 4 over gloo, with a test-only stand-in for the libmpx binding
(tests/bench_dist_worker.py).  Checks what the GPU run relies on but cannot
show on a one-GPU box: every rank follows the same circle-method round each
step and its peer follows the mirror role; each rank maps every other rank's
descriptor; the expected checksums handed to each validation transfer are the
PEER's tx checksums; an error on one rank reaches every rank (no hang); the
kernel engine's failure falls back to SDMA with a label; timing is the max
over ranks."""
import json
import os
import socket
import subprocess
import sys

import pytest

import bench

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mpi-perf_amd"))
from mpx.schedule import all_pairs_rounds, round_role  # noqa: E402

SEED = 0x6D70695F70657266


def key(r):
    return (SEED ^ (r << 56)) & 0xFFFFFFFFFFFFFFFF


def run(world, scenario, tmp_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    ps = [subprocess.Popen([sys.executable, os.path.join(HERE, "bench_dist_worker.py"), str(r), str(world), str(port),
                            scenario, str(tmp_path)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                           env=env) for r in range(world)]
    outs = [p.communicate(timeout=240)[0] for p in ps]
    assert all(p.returncode == 0 for p in ps), [o[-800:] for o in outs]
    return [json.load(open(tmp_path / f"rank{r}.json")) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_rounds_peers_and_expected_checksums(world, tmp_path):
    res = run(world, "ok", tmp_path)
    assert all(d["spin"] for d in res)       # the shared-memory spin barrier carried every per-round barrier
    rounds = all_pairs_rounds(world)
    n, iters, steps, warmup = 4096, 7, 5, 2
    warmup = max(warmup, world - 1)          # pairs_bench warms every round up at least once
    for d in res:
        r = d["rank"]
        assert d["engine_used"] == "kernel"
        assert d["res"]["validated_rounds"] == world - 1
        assert d["res"]["total"] == (world // 2) * n * iters * steps
        imports = sorted(x[1] for x in d["log"] if x[0] == "import")
        assert imports == [q for q in range(world) if q != r]
        xf = [x for x in d["log"] if x[0] == "xfer" and x[1] == "kernel"]
        checked = [x for x in xf if x[8] and x[2] == 2]
        timed = [x for x in xf if not x[8] and x[2] == 2][:warmup + steps]
        # validation: one checked transfer per round, against the PEER's tx
        # (then, after the headline, the staged / unstaged pair and
        # push_vs_pull's two checked unidir loops)
        assert len(checked) == world - 1 + 2 + 2
        assert [x[15] for x in checked[world - 1:world + 1]] == [True, False]   # staged, then MPX_XFER_NOSTAGE
        checked = checked[:world - 1]
        for rd, x in enumerate(checked):
            g, peer = round_role(rounds, rd, r)
            assert (x[3], x[4], x[5], x[6], x[7]) == (g, r, peer, 3, n)
            assert x[9] == (key(peer) * 31 + n) & 0xFFFFFFFFFFFFFFFF
            assert x[10] == (key(peer) * 31 + 1) & 0xFFFFFFFFFFFFFFFF
        # after the headline: checked ping-pong at the small sizes <= B on
        # every round, each against the peer's tx prefix of that size
        small = [x for x in xf if x[8] and x[2] == 0 and x[7] in (1, 8)]
        sizes = [1, 8]                                        # SMALL_CHECK_SIZES <= B = 4096
        assert len(small) == (world - 1) * len(sizes)
        for i, x in enumerate(small):
            g, peer = round_role(rounds, i // len(sizes), r)
            m = sizes[i % len(sizes)]
            assert (x[3], x[5], x[6], x[7]) == (g, peer, 20, m)
            assert x[9] == (key(peer) * 31 + m) & 0xFFFFFFFFFFFFFFFF
        assert d["res"]["small_message_check"]["failed_transfers"] == 0
        # the small messages run with the node's chosen LL threshold (the
        # fake times LL and bulk alike: LL is never slower, so 4 KiB = B)
        assert d["res"]["ll_max"] == 4096 and all(x[13] == "4096" for x in small)
        # warmup + timed steps: step s runs round s mod (N-1)
        assert len(timed) == warmup + steps
        for s, x in enumerate(timed):
            g, peer = round_role(rounds, (s if s < warmup else s - warmup) % (world - 1), r)
            assert (x[3], x[5], x[6], x[7]) == (g, peer, iters, n)
    # every rank reports the same max-over-ranks elapsed time and per-launch time
    assert len({d["res"]["elapsed"] for d in res}) == 1
    assert len({d["res"]["per_launch_s"] for d in res}) == 1
    # per_launch_s averages the G1 launches: G1 rank r reports 0.001*(1+r)
    g1 = [round_role(rounds, s % (world - 1), r)[0] for r in range(world) for s in range(steps)]
    assert sum(g1) == (world // 2) * steps
    # after the headline: LL against bulk on round 0 (the node's LL threshold),
    # then the ping-pong latency probe on round 0 with 10^5 iterations of 8 B,
    # then every round's pairs with 10^4, then the round-0 size sweep (config 3: unidir and full-duplex -x 1)
    for d in res:
        r = d["rank"]
        pp_all = [x for x in d["log"] if x[0] == "xfer" and x[2] == 0 and not x[8]]
        nll = 2 * 3                                           # LL_AB_SIZES <= B: 1, 2, 4 KiB, LL and bulk
        llab, pp = pp_all[:nll], pp_all[nll:nll + world]
        assert len(pp) == world and pp[0][6] == 100_000 and pp[0][7] == 8
        # then 10^4 iterations of 8 B on every round: every pair's latency
        for rd, x in enumerate(pp[1:]):
            assert (x[3], x[5], x[6], x[7]) == (*round_role(rounds, rd, r), 10_000, 8)
        g, peer = round_role(rounds, 0, r)
        sizes = [1, 8, 64, 512, 4096]                        # config 3's sizes <= B (B = 4096 here)
        sweep = [x for x in d["log"] if x[0] == "xfer" and x[1] == "kernel" and not x[8]][
            warmup + steps + nll + world:warmup + steps + nll + world + 2 * len(sizes)]
        assert [x[7] for x in sweep] == [m for m in sizes for _ in (0, 1)]
        assert [x[2] for x in sweep] == [2, 1] * len(sizes)  # -u 1 then -x 1 at every size
        assert all((x[3], x[5]) == (g, peer) for x in sweep)
        assert set(d["res"]["round0_sweep"]) == {f"{m}_{k}" for k in sizes for m in ("unidir", "nonblocking")}
        # LL against bulk on round 0: ping-pong at 1/2/4 KiB (<= B), MPX_LL_MAX set alike on every rank per
        # loop, each form first run in check mode against the peer's tx prefix
        assert [(x[7], x[13]) for x in llab] == [(m, v) for m in (1024, 2048, 4096) for v in ("8192", "0")]
        assert all((x[3], x[5], x[6]) == (g, peer, 2000) for x in llab)
        llchk = [x for x in d["log"] if x[0] == "xfer" and x[2] == 0 and x[8] and x[7] >= 1024]
        assert [(x[7], x[13], x[6]) for x in llchk] == [(m, v, 20) for m in (1024, 2048, 4096) for v in ("8192", "0")]
        assert all(x[9] == (key(peer) * 31 + x[7]) & 0xFFFFFFFFFFFFFFFF for x in llchk)
        assert set(d["res"]["ll_vs_bulk_half_rtt_us"]) == {f"{p}_{m}" for m in (1024, 2048, 4096) for p in ("ll", "bulk")}
        assert d["ll_max_after"] is None                     # the worker's environment is restored
        # last: push against pull on round 0 at B, each validated (check
        # mode, the peer's expected checksum) before it is timed
        byw = [x for x in d["log"] if x[0] == "xfer" and x[14] and x[7] == n][-5:]
        assert [(x[2], x[11], x[8]) for x in byw] == [(2, w, False) for w in (16, 32, 64, 128, 256)]
        assert set(d["res"]["push_vs_pull"]["pull_unidir_GBps_by_width"]) == {"16", "32", "64", "128", "256"}
        pv = [x for x in d["log"] if x[0] == "xfer" and x[7] == n and x[6] in (3, bench.PULL_AB_ITERS)][-13:-5]
        assert [(x[14], x[2], x[8], x[6]) for x in pv] == [
            (p, m, chk, it) for p in (False, True) for m in (2, 1) for chk, it in ((True, 3), (False, 100))]
        assert all((x[3], x[5]) == (g, peer) for x in pv)
        assert all(x[9] == (key(peer) * 31 + n) & 0xFFFFFFFFFFFFFFFF for x in pv if x[8])
        assert all(v is not None for v in d["res"]["push_vs_pull"].values())
        assert all(v is not None for v in d["res"]["push_vs_pull"]["pull_unidir_GBps_by_width"].values())
        assert set(d["res"]["push_vs_pull"]) >= {f"{p}_{m}_GBps" for p in ("push", "pull")
                                                  for m in ("unidir", "nonblocking")}
        assert "extras_errors" not in d["res"], d["res"].get("extras_errors")
        # the armed loops (here: the warm-up and timed steps) start from C as
        # the spin barrier opens (start_after_barrier), each right after its arm
        log = d["log"]
        at = [i for i, x in enumerate(log) if x[0] == "xfer" and x[1] == "kernel" and not x[8] and x[2] == 2
              and x[6] == iters][:warmup + steps]
        assert len(at) == warmup + steps
        assert all(log[i - 1][0] == "after_barrier" and log[i - 2][0] == "arm" for i in at), [
            log[i - 2:i + 1] for i in at[:2]]


def test_ipc_failure_on_one_rank_falls_back_to_rccl_on_every_rank(tmp_path):
    """IPC import fails on rank 1: the kernel and SDMA engines (which write
    into IPC-mapped peer memory) fail on every rank; RCCL maps nothing of
    ours and carries the bench, labelled."""
    res = run(2, "import_fails", tmp_path)
    for d in res:
        assert d["engine_used"].startswith("rccl (fallback")
        for eng in ("kernel", "sdma"):
            assert "rank 1" in d["extras"][f"{eng}_engine_error"] and "cannot map rank 0" in d["extras"][
                f"{eng}_engine_error"]
        assert not any(x[0] == "import" for x in d["log"][[x[0] for x in d["log"]].index("rccl_init"):])


def test_error_on_one_rank_reaches_every_rank(tmp_path):
    res = run(2, "all_fail", tmp_path)
    for d in res:
        # every engine fails on rank 1 -> SystemExit naming every engine's error on all ranks
        assert d["exit"].startswith("pairs bench failed: kernel: rank 1")
        assert "sdma: rank 1: FakeError: cannot map rank 0" in d["exit"]
        assert "rccl: rank 1: FakeError: ncclCommInitRank failed" in d["exit"]


@pytest.mark.parametrize("world", [2, 4])
def test_kernel_validation_failure_falls_back_to_sdma_with_a_label(world, tmp_path):
    res = run(world, "kernel_fails_validation", tmp_path)
    for d in res:
        assert d["engine_used"].startswith("sdma (fallback")
        assert "rank 0" in d["extras"]["kernel_engine_error"]
        assert any(x[0] == "xfer" and x[1] == "sdma" and not x[8] for x in d["log"])
        # the failed kernel context was closed before the SDMA one was opened
        inits = [i for i, x in enumerate(d["log"]) if x[0] == "init"]
        closes = [i for i, x in enumerate(d["log"]) if x[0] == "close" and x[1] == "kernel"]
        assert closes and inits[1] > closes[0]
        # SDMA: every round's graph chunks are built (mpx_xfer_prepare) before
        # the first untimed step, and every round gets a warm-up step, so no
        # capture lands inside the timed steps (bench.py)
        rounds = all_pairs_rounds(world)
        log = d["log"]
        steps_at = [i for i, x in enumerate(log) if x[0] == "xfer" and x[1] == "sdma" and not x[8] and x[6] == 7]
        prep = [(i, x) for i, x in enumerate(log) if x[0] == "prepare" and x[1] == "sdma"]
        assert {(x[3], x[5]) for _, x in prep} == {round_role(rounds, rd, d["rank"]) for rd in range(world - 1)}
        assert all(i < steps_at[0] for i, _ in prep)
        warm = max(2, world - 1)
        assert [(x[3], x[5]) for x in (log[i] for i in steps_at[:warm])] == \
            [round_role(rounds, s % (world - 1), d["rank"]) for s in range(warm)]


@pytest.mark.parametrize("world", [2, 4])
def test_push_tuning_agrees_across_ranks(world, tmp_path):
    """B > the LL landing zone: every push variant (width x streaming hint) is
    validated (check mode, the peer's checksums) and timed on round 0; the
    max over ranks picks one variant for every rank, and every timed step
    uses it."""
    res = run(world, "tune", tmp_path)
    rounds = all_pairs_rounds(world)
    n, warmup, steps = 65536, 2, 5
    warmup = max(warmup, world - 1)          # pairs_bench warms every round up at least once
    ms = {16: 5, 32: 7, 64: 3, 128: 4, 256: 6}
    want = {}
    for w in (16, 32, 64, 128, 256):
        for st in (False, True):
            t = ms[w] + (0 if st and w == 64 else 0.5)
            want[f"{w}{'+nt' if st else ''}"] = round(n * 40 / (t * 1e-3) / 1e9, 2)
    for d in res:
        r = d["rank"]
        g, peer = round_role(rounds, 0, r)
        assert d["res"]["push"] == "64+nt"
        assert d["res"]["push_tune"] == want
        xf = [x for x in d["log"] if x[0] == "xfer" and x[1] == "kernel"]
        tuned = [x for x in xf if x[11]][:20]
        cands = [(w, st) for w in (16, 32, 64, 128, 256) for st in (False, True)]
        for i, (w, st) in enumerate(cands):
            chk, timed = tuned[2 * i], tuned[2 * i + 1]
            assert chk[8] and chk[11] == w and chk[12] == st and (chk[3], chk[5]) == (g, peer)
            assert chk[9] == (key(peer) * 31 + n) & 0xFFFFFFFFFFFFFFFF
            assert not timed[8] and timed[11] == w and timed[12] == st and timed[6] == 40
        # the warm-up and timed steps, then the staged / unstaged pair (the same loop at B x iters)
        steps_run = [x for x in xf if not x[8] and x[2] == 2 and x[6] == 7]
        assert len(steps_run) == warmup + steps + 2 and all(x[11] == 64 and x[12] for x in steps_run)
        assert [x[15] for x in steps_run] == [True] * (warmup + steps + 1) + [False]


def test_rccl_refused_before_init_when_ranks_share_a_gpu(tmp_path):
    """The one-GPU rehearsal puts every rank on one card: the RCCL engine is
    refused from the gathered bus ids, on every rank, before any
    ncclCommInitRank (round 3's refused init slowed every later round of the
    rehearsal: profiles/r03_pull_rounds_diag.jsonl)."""
    res = run(2, "rccl_one_gpu", tmp_path)
    for d in res:
        assert "share GPU 0000:00:00.0" in d["res"]["error"], d["res"]
        assert not any(x[0] == "rccl_init" for x in d["log"])


@pytest.mark.parametrize("world,scenario", [(2, "counters"), (4, "counters"), (4, "one_gpu")])
def test_link_counters_one_sampler_per_gpu(world, scenario, tmp_path):
    """The in-process counter passes (bench.link_counters) after the timed
    steps: one sampling rank per GPU (the lowest rank on each bus id; all
    ranks share one on the one-GPU rehearsal), a write pass and a read pass,
    each around an untimed re-run of every round at the headline's B x iters
    with the tuned width; per G1 launch, link bytes = (WRREQ - WRREQ_DRAM) x
    64 summed over the samplers."""
    res = run(world, scenario, tmp_path)
    samplers = 1 if scenario == "one_gpu" else world
    launches = (world // 2) * (world - 1)
    n, iters = 4096, 7
    for d in res:
        cnt = d["res"]["counters"]
        assert "error" not in cnt, cnt
        assert cnt["samplers"] == samplers and cnt["g1_launches_per_pass"] == launches
        assert cnt["link_bytes_per_launch"] == round(samplers * 990 * 64 / launches, 1)
        assert cnt["local_dram_write_bytes_per_launch"] == round(samplers * 10 * 64 / launches, 1)
        assert cnt["link_over_algorithmic"] == round(samplers * 990 * 64 / (n * iters * launches), 5)
        assert cnt["gmi_write_bytes_per_launch"] == round(samplers * 1980 * 32 / launches, 1)
        assert cnt["ranks_on_distinct_gpus"] == (scenario != "one_gpu")
        assert cnt["raw"]["TCC_EA0_WRREQ_sum"] == samplers * 1000.0
        # the stand-in's 990 link requests are 1.1-4.4 x the pushed bytes here:
        # on distinct GPUs the self-check refuses the figure; sharing a GPU
        # no check applies
        roof = bench.link_traffic(cnt)
        if scenario == "one_gpu":
            assert roof["traffic"] == cnt["link_bytes_per_launch"] and roof["traffic_check"].startswith("not applicable")
        else:
            assert roof["traffic"] is None and roof["traffic_check"] == "failed"
            assert "self-check failed" in roof["traffic_reason"] and roof["traffic_raw"] == cnt["raw"]
        sampled = d["rank"] < samplers
        # rank 0 adds the peer control's passes on distinct GPUs: two writers x
        # two counter sets (its bytes are unrelated to the stand-in's counts, so
        # it validates no formula here)
        extra = 4 if (d["rank"] == 0 and scenario != "one_gpu") else 0
        assert len(d["passes"]) == (3 if sampled else 0) + extra
        if d["rank"] == 0 and scenario != "one_gpu":
            pc = cnt["peer_control"]
            peer = round_role(all_pairs_rounds(world), 0, 0)[1]
            assert pc["gpus"] == [0, peer] and pc["validated_formula"] is None, pc
            copies = [x for x in d["log"] if x[0] == "copy"]
            # warm-up + two passes, a launch per copy
            assert copies == [["copy", 0, peer, 0, bench.PEER_CONTROL_BYTES, 1]] * (3 * bench.PEER_CONTROL_ITERS)
        else:
            assert "peer_control" not in cnt
        # each pass wraps exactly one untimed run of every round, after the timed steps
        log = d["log"]
        if sampled:
            b = [i for i, x in enumerate(log) if x[0] == "pass_begin"][:3]
            e = [i for i, x in enumerate(log) if x[0] == "pass_end"][:3]
            for i, j in zip(b, e):
                inside = [x for x in log[i:j] if x[0] == "xfer"]
                assert len(inside) == world - 1 and all((x[2], x[6], x[7], x[8]) == (2, iters, n, False)
                                                        for x in inside)


def test_link_traffic_self_check_band():
    """bench.link_traffic on distinct GPUs: the subtraction's link bytes
    inside [0.9, 1.1] x the pushed bytes give the traffic figure; outside
    (a counter that sees ~0, or too much) the line prints null with the raw
    counters and the reason; sharing a GPU no check applies."""
    base = dict(link_bytes_per_launch=1000.0, local_dram_write_bytes_per_launch=5.0, source="src",
                gmi_over_algorithmic=1.0, io_over_algorithmic=0.0, local_dram_over_algorithmic=0.005,
                raw={"TCC_EA0_WRREQ_sum": 1.0})
    for r, ok in ((0.9, True), (1.0, True), (1.1, True), (0.0, False), (0.002, False), (0.89, False), (1.2, False)):
        roof = bench.link_traffic(dict(base, link_over_algorithmic=r, ranks_on_distinct_gpus=True))
        if ok:
            assert roof["traffic"] == 1000.0 and roof["traffic_check"].startswith("passed"), r
        else:
            assert roof["traffic"] is None and roof["traffic_check"] == "failed", r
            assert f"read {r} x" in roof["traffic_reason"] and roof["traffic_raw"] == base["raw"]
            assert roof["traffic_local_dram"] == 5.0
    roof = bench.link_traffic(dict(base, link_over_algorithmic=0.0, ranks_on_distinct_gpus=False))
    assert roof["traffic"] == 1000.0 and roof["traffic_check"].startswith("not applicable")


@pytest.mark.parametrize("world", [2, 4])
def test_peer_control_validates_a_formula(world, tmp_path):
    """On distinct GPUs rank 0 writes known bytes across its round-0 link
    (k_copy into the peer GPU's memory, then a threads-mode push) under the
    counters; here the stand-in's GMI counter reads exactly those bytes, so
    the 'gmi' formula is validated and measures the pushes (which, at the
    stand-in's fixed counts, read far more than the pushed bytes: the line
    says so)."""
    res = run(world, "counters_validated", tmp_path)
    d = next(x for x in res if x["rank"] == 0)
    cnt = d["res"]["counters"]
    pc = cnt["peer_control"]
    assert pc["validated_formula"] == "gmi" and pc["copy"]["gmi_over_bytes"] == 1.0, pc
    assert pc["copy"]["subtraction_over_bytes"] < 0.01 and pc["copy_checked"] is True
    roof = bench.link_traffic(cnt)
    assert roof["traffic"] == cnt["link_formula_bytes_per_launch"]["gmi"]
    assert roof["traffic_check"].startswith("validated (gmi)") and "outside" in roof["traffic_check"]


def test_link_traffic_prefers_a_validated_formula():
    cnt = dict(link_bytes_per_launch=0.0, local_dram_write_bytes_per_launch=5.0, source="src",
               link_over_algorithmic=0.0, ranks_on_distinct_gpus=True, gmi_over_algorithmic=1.0,
               io_over_algorithmic=0.0, local_dram_over_algorithmic=0.0, raw={},
               link_formula_bytes_per_launch=dict(subtraction=0.0, gmi=1000.0, io=0.0),
               link_formula_over_algorithmic=dict(subtraction=0.0, gmi=1.001, io=0.0),
               peer_control=dict(validated_formula="gmi", copy=dict(gmi_over_bytes=0.998)))
    roof = bench.link_traffic(cnt)
    assert roof["traffic"] == 1000.0 and roof["traffic_check"] == "validated (gmi); the pushes read 1.001 x the pushed bytes"
    assert "0.998 x the bytes k_copy wrote across a link" in roof["traffic_source"]
    # no validated formula: the subtraction's self-check decides (here: fails)
    cnt["peer_control"] = dict(validated_formula=None)
    roof = bench.link_traffic(cnt)
    assert roof["traffic"] is None and roof["traffic_check"] == "failed"


def test_link_counters_need_the_tool_on_every_sampling_rank(tmp_path):
    """A sampling rank without the counter tool (its registration failed):
    every rank skips the passes alike (no rank left inside a collective the
    others never enter) and the line says which rank lacked it."""
    res = run(4, "counters_missing", tmp_path)
    for d in res:
        assert d["res"]["counters"] == {"error": "the counter tool is not running on sampling rank(s) [1]"}
        assert not d["passes"]
        assert "error" not in d["res"] or d["res"].get("counters")


@pytest.mark.parametrize("world", [2, 4])
def test_cpu_baseline_beside_the_pairs_line(world):
    """The reference itself beside the N >= 2 line:
    run-hbv3's layout (N ranks, -p N/2 -u 1) under MPICH shm at a small B,
    aggregate = N/2 pairs' bytes / the slowest sender's time per run."""
    ref = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "mpi_perf")
    if not os.path.exists(ref):
        pytest.skip("compiled reference not built here (oracle/_ref)")
    cb = bench.cpu_baseline_pairs(world, 1 << 20, 40, 3)
    assert cb and cb["kind"] == "reference" and cb["cores"] == world and cb["unit"] == "GB/s"
    assert cb["value"] > 0 and cb["per_pair_GBps"] == pytest.approx(cb["value"] / (world // 2), rel=1e-2)
    assert f"{world} ranks, -p {world // 2} -u 1 -b {1 << 20} -i 40 -r 3" in cb["sample"]


def test_link_target_primary_verdict_follows_the_stated_bar():
    """extras.targets.per_pair_unidir_GBps: `meets` is
    judged against the stated bar, 0.85 x 153.6 GB/s per direction
    (SURVEY.md:361, BASELINE.md:51); the unsourced per-direction reading
    (0.85 x 76.8) goes beside it as meets_per_direction_reading."""
    assert bench.STATED_LINK_PEAK_GBPS == 153.6 and bench.XGMI_LINK_PEAK_GBPS == 76.8
    for gbps, primary, reading in ((131.0, True, True), (130.0, False, True), (66.0, False, True),
                                   (65.0, False, False)):
        t = bench.link_target(gbps, 4 << 20)
        assert t["meets"] is primary and t["meets_per_direction_reading"] is reading, (gbps, t)
        assert "153.6 GB/s per direction" in t["target"] and "SURVEY.md:361" in t["target"]
        assert "76.8" in t["per_direction_reading"] and "unsourced" in t["per_direction_reading"]
        assert "meets_vs_bidirectional_153_6" not in t


def test_fabric_counters_are_optional(tmp_path):
    """the GMI / IO / DRAM 32-B write counters are an optional
    set.  When their pass fails on a sampler, the link and read figures still
    stand (no error), the fabric figures are null, the 'gmi' / 'io' formulas
    are left out, and the peer control still reports the subtraction."""
    res = run(2, "fabric_missing", tmp_path)
    for d in res:
        cnt = d["res"]["counters"]
        assert "error" not in cnt, cnt
        assert cnt["fabric_counters_read"] is False and cnt["gmi_write_bytes_per_launch"] is None
        assert cnt["link_bytes_per_launch"] == round(2 * 990 * 64 / 1, 1)
        assert set(cnt["link_formula_bytes_per_launch"]) == {"subtraction"}
        assert any("fabric counters" in n for n in cnt["notes"])
        if d["rank"] == 0:
            pc = cnt["peer_control"]
            assert "subtraction_over_bytes" in pc["copy"] and "gmi_over_bytes" not in pc["copy"], pc
            assert "copy_fabric_error" in pc and pc["copy_checked"] is True and pc["push_checked"] is True
        roof = bench.link_traffic(cnt)
        assert roof["traffic_check"] == "failed" and "None" in roof["traffic_reason"]
