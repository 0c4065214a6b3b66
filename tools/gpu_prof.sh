#!/bin/bash
# Profiles of the default bench (round N): kernel-trace stats + PMC traffic.
set -o pipefail
R=${ROUND:-r01}
mkdir -p gpurun_out/prof_$R gpurun_out/pmc_fetch gpurun_out/pmc_write
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$R.json 2> gpurun_out/bench_$R.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$R -o bench -- python -u bench.py --no-cpu-baseline --no-extras > gpurun_out/bench_prof_$R.json 2> gpurun_out/bench_prof_$R.err &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o copy -- python -u tools/pmc_copy.py > gpurun_out/pmc_write.log 2>&1
echo "rc=$?"
