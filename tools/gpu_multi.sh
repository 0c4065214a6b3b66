#!/bin/bash
# Rehearse the N>1 bench path on one GPU (every rank on GPU 0, one process
# per rank, IPC-mapped peers) at N=4, then profile k_xfer of a single-process
# loopback pair (mpx_perf threads host, unidir 4 MiB).  Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
R=${ROUND:-r01}
mkdir -p gpurun_out/prof_xfer_$R gpurun_out/logs_xfer
export TMPDIR=/tmp
echo vm > gpurun_out/group1_xfer
MPX_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 4 --steps 6 --warmup 2 > gpurun_out/bench_n4_onegpu_$R.json 2> gpurun_out/bench_n4_onegpu_$R.err &&
MPX_PROCESSOR_NAMES=vm,runsc timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_xfer_$R -o xfer -- mpi-perf_amd/bin/mpx_perf -w 2 -f gpurun_out/group1_xfer -n 1 -p 1 -u 1 -b 4194304 -i 200 -r 6 -l gpurun_out/logs_xfer > gpurun_out/xfer_prof_$R.log 2>&1
rc=$?
echo "gpu_multi rc=$rc"
exit $rc
