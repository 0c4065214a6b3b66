#!/bin/bash
# Round 4, GPU pass o: bench.py under rocprofv3 now exits through its normal
# teardown (mpx_shutdown first) so the profiler writes its output — the
# committed kernel-trace summary and a --pmc pass of the N=1 bench; then the
# N=8 one-GPU rehearsal with the counter tool in rank 0 only, and once more
# without counters (was the tool in all eight processes the r04n slowdown?).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04o}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench \
    -- python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/kt_bench.json 2> $O/kt_bench.err
rc=$?; echo "bench kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench -o x \
    -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_bench.json 2> $O/pmc_bench.err
rc=$?; echo "bench under --pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --steps 14 --warmup 7 > $O/bench_n8.json 2> $O/bench_n8.err
rc=$?; echo "bench n8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 8 --steps 14 --warmup 7 --no-counters --no-cpu-baseline > $O/bench_n8_nocounters.json 2> $O/bench_n8_nocounters.err
rc=$?; echo "bench n8 no counters rc=$rc"; exit $rc
