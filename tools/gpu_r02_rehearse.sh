#!/bin/bash
# N=4 and N=8 bench.py paths rehearsed on one GPU (every rank on GPU 0,
# MPX_BENCH_ONE_GPU=1), plus the PMC passes of the 1-GPU copy (traffic of
# the headline kernel).  Each step its own limit; stop at the first failure.
set -o pipefail
R=${ROUND:-r02}
mkdir -p gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
MPX_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 4 --steps 6 --warmup 2 > gpurun_out/bench_n4_onegpu_$R.json 2> gpurun_out/bench_n4_onegpu_$R.err &&
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29548 bench.py --gpus 8 --steps 14 --warmup 2 > gpurun_out/bench_n8_onegpu_$R.json 2> gpurun_out/bench_n8_onegpu_$R.err &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_write.log 2>&1
rc=$?
echo "gpu_r02_rehearse rc=$rc"
exit $rc
