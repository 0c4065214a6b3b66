"""One rank of tests/test_bench_dist.py: runs bench.py's N>1 orchestration
(pairs_with_fallback -> pairs_bench) over a gloo process group on CPU, with
a TEST-ONLY stand-in for the mpx binding that records every call.  The stand-in
never replaces libmpx in bench.py or anywhere else: it exists only here, to
check the multi-rank logic (round schedule, peer descriptors, expected
checksums, error agreement, fallback, max-over-ranks timing) without a GPU.

    python bench_dist_worker.py <rank> <world> <port> <scenario> <outdir>
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402

# set by the __main__ block below, or by a worker that imports this module
rank, scenario = 0, "ok"


class Timing:
    def __init__(self, wall_s, device_s, nwg=0):
        self.wall_s, self.device_s, self.nwg = wall_s, device_s, nwg


class FakeError(RuntimeError):
    pass


class FakeMpx:
    """Mirror of the mpx binding's surface that bench.pairs_bench uses."""
    MODE_PINGPONG, MODE_NONBLOCKING, MODE_UNIDIR = 0, 1, 2
    FILL_BYTE, FILL_SPLITMIX = 0, 1
    PATTERN_SEED = 0x6D70695F70657266
    log = []

    @staticmethod
    def pattern_key(seed, src, dst, it):
        return (seed ^ (src << 56) ^ (dst << 48) ^ (it << 24)) & 0xFFFFFFFFFFFFFFFF

    @staticmethod
    def rccl_unique_id():
        return b"uid-from-rank-0"

    @staticmethod
    def bus_id(dev):
        # one GPU per rank, unless the scenario puts every rank on one card;
        # every rank passes dev 0 for its own GPU, and another device index d
        # is GPU d (rank d's card) — rank 0's peer control looks its peer up
        if scenario in ("one_gpu", "rccl_one_gpu"):
            return "0000:00:00.0"
        return f"0000:{(rank if dev == 0 else dev) + 1:02x}:00.0"

    @staticmethod
    def device_count():
        return world

    @staticmethod
    def link_info(a, b):
        # every pair one xGMI hop, except GPUs 1 and 2 (two hops): the table
        # must name it
        FakeMpx.log.append(["link_info", a, b])
        return {"type": "xgmi", "hops": 2 if {a, b} == {1, 2} else 1}

    @staticmethod
    def shutdown():
        FakeMpx.log.append(["shutdown"])

    @staticmethod
    def rccl_version():
        return {"version": 22707, "release": "2.27.7", "library": "fake"}

    class Context:
        def __init__(self, nranks, engine):
            self.engine = engine
            self.nranks = nranks
            self.filled = None
            FakeMpx.log.append(["init", engine, nranks])

        def alloc(self, dev, n):
            return ("buf", dev, n)

        def fill(self, b, n, pattern, key):
            self.filled = key

        def copy(self, dev, dst, src, n, iters):
            FakeMpx.log.append(["copy", dev, dst[1], src[1], n, iters])

        def attach(self, r, dev, tx, rx, n):
            FakeMpx.log.append(["attach", r, dev, n])

        def export(self, r):
            return f"desc-of-{r}".encode()

        def checksum(self, b, n):
            return (self.filled * 31 + n) & 0xFFFFFFFFFFFFFFFF     # a function of this rank's tx

        def import_rank(self, r, desc):
            if scenario in ("import_fails", "all_fail") and rank == 1:
                raise FakeError(f"cannot map rank {r}")
            assert desc == f"desc-of-{r}".encode(), (r, desc)
            FakeMpx.log.append(["import", r])

        def rccl_init_rank(self, r, n, uid):
            assert uid == b"uid-from-rank-0"
            if scenario == "rccl_hangs" and rank == 1:
                time.sleep(600)            # an RCCL bootstrap that never returns
            if scenario == "all_fail" and rank == 1:
                raise FakeError("ncclCommInitRank failed")
            # RCCL prints its version block on stdout at communicator init
            os.write(1, b"RCCL version : 2.x (banner written by the library to fd 1)\n")
            FakeMpx.log.append(["rccl_init", r, n])

        def xfer(self, mode, group, me, peer, iters, tx, rx, n, check_payload=False, expect=0, expect_ack=0,
                 timeout_ms=0, nwg=0, stream=False, pull=False, stage=True, after=None):
            if after is not None:       # the real binding waits on it from C, then starts the call
                FakeMpx.log.append(["after_barrier", self.engine, mode, me, iters])
                after.wait()
            if check_payload and self.engine == "kernel" and scenario == "kernel_fails_validation" and rank == 0:
                raise FakeError("payload checksum mismatch")
            if (scenario == "kernel_step_fails" and self.engine == "kernel" and rank == 1 and mode == 2 and
                    not check_payload and iters == 500):
                raise FakeError("device-side wait timed out (timed step)")
            if scenario == "latency_fails" and rank == 1 and mode == 0 and n == 8:
                raise FakeError("device-side wait timed out (LL ping-pong)")
            FakeMpx.log.append(["xfer", self.engine, mode, group, me, peer, iters, n, bool(check_payload), expect,
                                expect_ack, nwg, stream, os.environ.get("MPX_LL_MAX"), pull, stage])
            time.sleep(0.002)
            if nwg and not check_payload and iters == 40:
                # push tuning: rank 0 is fastest at 32, rank 1 slow at 32; the
                # max over ranks is fastest at 64 with the streaming hint
                ms = {16: 5, 32: 2 if rank != 1 else 7, 64: 3, 128: 4, 256: 6}[nwg] + (0 if stream and nwg == 64
                                                                                       else 0.5)
                return Timing(ms * 1e-3, ms * 1e-3)
            return Timing(0.002, 0.001 * (1 + me))

        def arm(self, mode, group, me, peer, iters, tx, rx, n, check_payload=False, expect=0, expect_ack=0,
                timeout_ms=0, nwg=0, stream=False, pull=False, stage=True):
            FakeMpx.log.append(["arm", self.engine, mode, group, me, peer, iters, n])

        def disarm(self, r):
            FakeMpx.log.append(["disarm", self.engine, r])

        def phases(self, r):
            return dict({k: 1e-6 for k in ("wall_s", "host_prep_s", "launch_to_start_s", "posted_wait_s", "kernel_s",
                                           "done_to_return_s", "first_iter_s", "tail_s")}, armed=1, resident=1)

        def prepare(self, mode, group, me, peer, iters, n, timeout_ms=0, pull=False):
            FakeMpx.log.append(["prepare", self.engine, mode, group, me, peer, iters, n, pull])

        def close(self):
            FakeMpx.log.append(["close", self.engine])


class FakeProf:
    """Stand-in for mpx/counters.py: every pass reports fixed counts per
    counter name (per sampling rank), so the aggregation is checkable."""
    COUNTS = {"TCC_EA0_WRREQ_sum": 1000.0, "TCC_EA0_WRREQ_64B_sum": 1000.0, "TCC_EA0_WRREQ_DRAM_sum": 10.0,
              "TCC_EA0_RDREQ_sum": 50.0, "TCC_EA0_RDREQ_DRAM_sum": 5.0,
              "TCC_EA0_WRREQ_WRITE_GMI_32B_sum": 1980.0, "TCC_EA0_WRREQ_WRITE_IO_32B_sum": 0.0,
              "TCC_EA0_WRREQ_WRITE_DRAM_32B_sum": 20.0}
    passes = []

    class Pass:
        def __init__(self, bus, names):
            self.bus, self.names = bus, names
            self.values, self.reads_reset = None, 0

        def __enter__(self):
            FakeProf.passes.append([self.bus, self.names])
            FakeMpx.log.append(["pass_begin", self.names])
            return self

        def __exit__(self, *exc):
            FakeMpx.log.append(["pass_end", self.names])
            if scenario == "fabric_missing" and "TCC_EA0_WRREQ_WRITE_GMI_32B_sum" in self.names:
                raise RuntimeError("counter TCC_EA0_WRREQ_WRITE_GMI_32B_sum not available on this agent")
            self.values = [FakeProf.COUNTS[n] for n in self.names]
            return False


class FakeCounters:
    """Stand-in for the mpx.counters module (bench.main: register / ready / Pass)."""
    CounterError = RuntimeError
    Pass = FakeProf.Pass

    @staticmethod
    def register():
        pass

    @staticmethod
    def ready():
        return True

    @staticmethod
    def error():
        return ""


FakeMpx.counters = FakeCounters


if __name__ == "__main__":
    rank, world, port, scenario, outdir = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4],
                                           sys.argv[5])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    if scenario == "counters_validated":
        # the GMI counter reads exactly the peer control's known bytes per pass
        FakeProf.COUNTS["TCC_EA0_WRREQ_WRITE_GMI_32B_sum"] = float(bench.PEER_CONTROL_BYTES * bench.PEER_CONTROL_ITERS
                                                                   // 32)
    extras = {}
    out = {"rank": rank}
    try:
        nbytes = 65536 if scenario == "tune" else 4096
        if scenario == "rccl_one_gpu":
            out.update(res=bench.pairs_bench(FakeMpx, torch, dist, "rccl", rank, world, 0, nbytes, 7, 5, 2,
                                             dist.barrier, latency=False))
        else:
            # one_gpu: only rank 0 registers the tool (bench.main's one-GPU
            # rehearsal); counters_missing: sampling rank 1 has none
            prof = FakeProf if (scenario in ("counters", "counters_validated", "fabric_missing")
                                or (scenario == "one_gpu" and rank == 0)
                                or (scenario == "counters_missing" and rank != 1)) else None
            count = scenario in ("counters", "counters_validated", "one_gpu", "counters_missing", "fabric_missing")
            # the per-round barriers spin in shared memory, as in bench.main (world 2 and 4 here)
            d, spin = bench.spin_barrier_dist(dist, rank, world) if scenario == "ok" else (dist, None)
            out["spin"] = spin is not None
            res, used = bench.pairs_with_fallback(FakeMpx, torch, d, "kernel", rank, world, 0, nbytes, 7, 5, 2,
                                                  dist.barrier, extras, prof=prof, count=count)
            out.update(res=res, engine_used=used, extras=extras, passes=FakeProf.passes)
    except SystemExit as e:
        out.update(exit=str(e))
    out["log"] = FakeMpx.log
    out["ll_max_after"] = os.environ.get("MPX_LL_MAX")
    with open(os.path.join(outdir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
