#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, the 1-GPU bench, a rocprofv3
# kernel-trace summary of the bench.  Every GPU step has its own time limit
# and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread ${PYTEST_EXTRA} > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python -u bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
rc=$?
echo "gpu_check rc=$rc"
exit $rc
