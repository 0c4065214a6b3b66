#!/bin/bash
# Counters of the N-GPU bench path ("rocprof counters (achieved
# xGMI and HBM GB/s) ... at 2, 4 and 8 GPUs").  Every rank of bench.py is
# started by hand (no launcher hop under the profiler), each under its own
# rocprofv3:
#   pass 1  --kernel-trace --stats            k_xfer durations per rank
#   pass 2  --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum
#           (three of the four TCC counters one pass may hold); a sender's
#           link traffic is (WRREQ - WRREQ_DRAM) x 64 B per dispatch
#   pass 3  --pmc TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum:
#           which fabric path the non-DRAM writes take (32-B units)
#   pass 4/5 the same timed steps in pull mode (MPX_XFER_PULL=1: the
#           receiver, k_xfer_pull<2, 0>, loads the sender's tx): kernel trace,
#           then --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum
#           TCC_EA0_RDREQ_GMI_32B_sum — a pulling receiver's link reads per
#           launch against B x iters (does every iteration cross the link?)
# then tools/node_profile_summary.py writes gpurun_out/node_prof_n$N/summary.json.
#
#   N=8 tools/node_profile.sh                 on an 8-GPU node (one rank per GPU)
#   N=2 MPX_BENCH_ONE_GPU=1 tools/node_profile.sh   rehearsal on one GPU: only
#       rank 0 is counter-profiled (the GPU's counters are shared), and every
#       write lands in local DRAM, so the link traffic reads 0
# Each rank has its own time limit; the script fails if any rank fails.
# --no-cpu-baseline on every rank: a profiled rank must start no mpiexec chain
# (the profiler's preload would reach oracle/ref_wrap.sh's exec after the GPU
# was initialised; bench.py also refuses the reference legs under a profiler).
set -o pipefail
N=${N:-2}
O=gpurun_out/node_prof_n$N
mkdir -p $O
export TMPDIR=/tmp WORLD_SIZE=$N MASTER_ADDR=127.0.0.1
# one-GPU rehearsal: one HW queue per process, as bench.py sets for itself —
# set here, before the process starts, because the profiler may start HIP
# before bench.py's own line runs
[ -n "$MPX_BENCH_ONE_GPU" ] && export GPU_MAX_HW_QUEUES=1
# Under rocprofv3 bench.py destroys its rank streams (mpx_shutdown) and exits
# normally, so the profiler's exit-time finalizer writes the output and finds
# no live CU-masked queue (profiles/r04_exit_segv_stack.txt)
STEPS=${STEPS:-$((2 * (N - 1)))}
run_pass() {   # pass-name, rocprofv3 options...
    local pass=$1; shift
    export MASTER_PORT=$((29600 + RANDOM % 300))
    local pids=() r
    for r in $(seq 0 $((N - 1))); do
        local prof=("$@")
        if [ -n "$MPX_BENCH_ONE_GPU" ] && [ "${pass%trace}" = "$pass" ] && [ $r -gt 0 ]; then prof=(); fi
        if [ ${#prof[@]} -gt 0 ]; then
            RANK=$r LOCAL_RANK=$r timeout -k 10 300 rocprofv3 "${prof[@]}" --output-format csv -d $O/$pass -o rank$r \
                -- python3 -u bench.py --gpus $N --steps $STEPS --warmup 1 --no-extras --no-cpu-baseline \
                > $O/${pass}_rank$r.json 2> $O/${pass}_rank$r.err &
        else
            RANK=$r LOCAL_RANK=$r timeout -k 10 300 python3 -u bench.py --gpus $N --steps $STEPS --warmup 1 --no-extras \
                --no-cpu-baseline \
                > $O/${pass}_rank$r.json 2> $O/${pass}_rank$r.err &
        fi
        pids+=($!)
    done
    # a rank that timed out after bench.py's "done, shutting down" marker
    # finished its transfers and stalled at exit: reported on its own, so an
    # exit stall is never read as a transfer failure
    local rc=0 i x
    for i in "${!pids[@]}"; do
        wait ${pids[$i]}; x=$?
        [ $x -eq 0 ] && continue
        rc=1
        if { [ $x -eq 124 ] || [ $x -eq 137 ]; } && grep -q "done, shutting down" $O/${pass}_rank$i.err; then
            echo "node_profile N=$N pass $pass rank $i: EXIT STALL (rc $x after its transfers finished)"
        else
            echo "node_profile N=$N pass $pass rank $i: FAILED rc $x"
        fi
    done
    echo "node_profile N=$N pass $pass rc=$rc"
    return $rc
}
run_pass trace --kernel-trace --stats &&
run_pass pmc --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum &&
run_pass fabric --pmc TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_WRREQ_WRITE_IO_32B_sum &&
MPX_XFER_PULL=1 run_pass pull_trace --kernel-trace --stats &&
MPX_XFER_PULL=1 run_pass pull_fabric --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_GMI_32B_sum &&
python3 tools/node_profile_summary.py $O $N
