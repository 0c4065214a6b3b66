#!/bin/bash
# rocprofv3 kernel-trace stats of the N = 2 bench path rehearsed on one GPU:
# two ranks started by hand (no launcher hop under the profiler), each its
# own rocprofv3 process.  Compare k_xfer<2,1>'s average duration with the
# bench line's roofline.avg_launch_us.
set -o pipefail
R=${ROUND:-r01}
export TMPDIR=/tmp MPX_BENCH_ONE_GPU=1 WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=29561
mkdir -p gpurun_out/prof_n2_$R
RANK=0 LOCAL_RANK=0 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n2_$R -o rank0 \
    -- python3 -u bench.py --gpus 2 --steps 6 --warmup 1 --no-extras > gpurun_out/bench_n2_prof_$R.json 2> gpurun_out/bench_n2_prof_$R.err0 &
p0=$!
RANK=1 LOCAL_RANK=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_n2_$R -o rank1 \
    -- python3 -u bench.py --gpus 2 --steps 6 --warmup 1 --no-extras > /dev/null 2> gpurun_out/bench_n2_prof_$R.err1
r1=$?
wait $p0
r0=$?
echo "gpu_prof_n2 rc=$r0/$r1"
[ $r0 -eq 0 ] && [ $r1 -eq 0 ]
