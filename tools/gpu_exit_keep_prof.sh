#!/bin/bash
# Does a process whose pooled rank streams are left to the runtime
# (MPX_POOL_EXIT=keep) exit cleanly under rocprofv3?  (Round 1: SIGSEGV in
# __cxa_finalize after the tool's finalization.)  bench.py N=1 (short) and
# mpx_perf threads mode, each under rocprofv3 --kernel-trace --stats, then
# the same without the knob.  Output: gpurun_out/exit_keep_prof/.
export TMPDIR=/tmp
O=gpurun_out/exit_keep_prof
mkdir -p $O
echo "vm" > $O/group1
for mode in keep default; do
    v=$([ $mode = keep ] && echo keep)
    MPX_POOL_EXIT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench_$mode -o b \
        -- python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > $O/bench_$mode.json 2> $O/bench_$mode.err
    echo "bench under rocprofv3, MPX_POOL_EXIT=$mode: rc=$?" | tee -a $O/summary.txt
    MPX_POOL_EXIT=$v MPX_PROCESSOR_NAMES=vm,runsc MPX_HOSTNAME=localhost timeout -k 10 120 rocprofv3 --kernel-trace --stats \
        --output-format csv -d $O/prof_perf_$mode -o p -- mpi-perf_amd/bin/mpx_perf -w 2 -g 0,0 -e sdma -f $O/group1 -n 1 -p 1 \
        -r 3 -i 300 -b 65536 -l $O/logs_$mode -x 1 -c 1 -t 5000 > $O/perf_$mode.out 2> $O/perf_$mode.err
    echo "mpx_perf under rocprofv3, MPX_POOL_EXIT=$mode: rc=$?" | tee -a $O/summary.txt
done
