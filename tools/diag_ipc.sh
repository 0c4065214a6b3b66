#!/bin/bash
# Diagnostic: context lifecycles with IPC imports, 4 processes on one GPU,
# without the post-close barrier; then the N=4 bench rehearsal.
set -o pipefail
export TMPDIR=/tmp MPX_BENCH_ONE_GPU=1
DIAG_BARRIER_AFTER_CLOSE=0 timeout -k 10 120 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29551 tools/diag_ipc_cycle.py > gpurun_out/diag_ipc4_nobar.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --steps 4 --warmup 1 > gpurun_out/diag_n4.json 2> gpurun_out/diag_n4.err
echo rc=$?
