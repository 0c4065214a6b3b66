#!/bin/bash
# Full GPU pass: smoke, the -m gpu suite, the 1-GPU bench (with extras),
# the N=2 path rehearsed on one GPU, and the rocprofv3 kernel-trace summary
# of the 1-GPU bench command.  Each step has its own limit; the chain stops
# at the first failure.
set -o pipefail
R=${ROUND:-r03}
mkdir -p gpurun_out/prof_$R
export TMPDIR=/tmp
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 &&
tools/gpu_pytest.sh all_$R tests &&
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err &&
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 6 --warmup 2 > gpurun_out/bench_n2_onegpu_$R.json 2> gpurun_out/bench_n2_onegpu_$R.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o bench -- python3 -u bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof_$R.json 2> gpurun_out/bench_prof_$R.err
rc=$?
echo "gpu_full rc=$rc"
exit $rc
