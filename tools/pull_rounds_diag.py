"""Diagnostic: bench.py's all-pairs rounds (pairs_bench) pushed and pulled at
N ranks stacked on one GPU (MPX_BENCH_ONE_GPU's setting), before and after a
failed RCCL communicator init (RCCL refuses two ranks on one device) — the
N = 8 rehearsal's pulled comparison rounds read 0.93 GB/s where round 0's
push_vs_pull read 411.  Launch like bench.py:

    MPX_BENCH_ONE_GPU=1 python -m torch.distributed.run --nproc-per-node 8 ... tools/pull_rounds_diag.py

Rank 0 prints one JSON line per pass: aggregate GB/s (all rounds, 512 x 4 MiB).
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mpi-perf_amd"))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "1")
import bench  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
os.environ["MPX_PUSH_WG"] = str(bench.one_gpu_push_cap(world))
import datetime  # noqa: E402

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mpx  # noqa: E402

torch.cuda.set_device(0)
dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=180))


def barrier_sync():
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()


for label, eng, pull in (("kernel push", "kernel", False), ("kernel pull", "kernel", True),
                         ("rccl (fails on one GPU)", "rccl", False), ("kernel push", "kernel", False),
                         ("kernel pull", "kernel", True)):
    t0 = time.time()
    r = bench.pairs_bench(mpx, torch, dist, eng, rank, world, 0, 4 << 20, 512, world - 1, 1, barrier_sync,
                          latency=False, tune=False, pull=pull)
    if rank == 0:
        agg = r.get("error") or round(r["total"] / r["elapsed"] / 1e9, 3)
        print(json.dumps(dict(n=world, pass_=label, aggregate_GBps=agg, wall_s=round(time.time() - t0, 1))),
              flush=True)
dist.destroy_process_group()
