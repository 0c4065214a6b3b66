#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, the 1-GPU bench, the N=2 bench
# path rehearsed on one GPU, then profiles (kernel-trace stats + PMC passes).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${ROUND:-r01}
mkdir -p gpurun_out/prof_$R gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_EXTRA} > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err &&
MPX_BENCH_ONE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/bench_n2_onegpu_$R.json 2> gpurun_out/bench_n2_onegpu_$R.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o bench -- python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof_$R.json 2> gpurun_out/bench_prof_$R.err &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_write.log 2>&1
rc=$?
echo "gpu_check rc=$rc"
exit $rc
