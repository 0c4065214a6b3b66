#!/bin/bash
# The one GPU recipe (round 5; replaces round 4's gpu_r04*.sh wrappers).
#
#   tools/gpu.sh <out-tag> <step> [<step> ...]
#
# Runs the named steps in order on the gpurun box, each under its own time
# limit, output under gpurun_out/<out-tag>/.  The chain stops at the first
# step that fails; a step that ends with a signal or a time limit stops it
# too (no GPU step runs after a fault or a hang).  Steps:
#   smoke            __graft_entry__.smoke()
#   pytest[:files]   the -m gpu suite (or the given test files, comma-separated)
#   bench1           bench.py at N = 1 (defaults)
#   rehearseN        bench.py at N ranks, every rank on GPU 0 (N = 2, 4, 8)
#   kt               rocprofv3 --kernel-trace --stats of the N = 1 bench
#   pmc              rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of the N = 1 bench
#   stall            tools/exit_stall_repro: fenced vs barrier stream teardown cycles
#   procs_exit       mpx_perf processes mode (2 processes on GPU 0), exit with mpx_shutdown, K runs
#   linkctl          tools/link_counter_control.py: the link-byte counter's positive control
#   soak             tools/soak.py, threads + processes
# Environment: K (procs_exit runs, default 8), STALL_CYCLES (default 2000),
# STALL_RUNS (default 3).
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
O=gpurun_out/$tag
mkdir -p $O
PERF=mpi-perf_amd/bin/mpx_perf

step_ok() {  # name rc
    echo "[$1] rc=$2"
    [ "$2" -eq 0 ] || exit "$2"
}

rehearse() {
    local n=$1
    MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29520 + n + RANDOM % 200)) bench.py --gpus $n \
        > $O/bench_n$n.json 2> $O/bench_n$n.err
    step_ok rehearse$n $?
}

procs_exit() {  # K runs of the processes-mode pingpong; a run whose ranks do not end is SIGUSR1'd (stacks) then killed
    echo vm > $O/group1
    local k stalls=0
    for k in $(seq 1 ${K:-8}); do
        local port=$((29600 + RANDOM % 300)) r
        rm -rf $O/logs_$k; mkdir -p $O/logs_$k
        for r in 0 1; do
            MPX_DEBUG=1 MPX_RANK=$r MPX_SIZE=2 MPX_LOCAL_RANK=$r MPX_PROCESSOR_NAMES=vm,runsc \
                MPX_BOOTSTRAP=127.0.0.1:$port MPX_BOOTSTRAP_TIMEOUT=60 MPX_HOSTNAME=localhost \
                timeout -s USR1 -k 8 40 $PERF -g 0,0 -t 5000 -f $O/group1 -n 1 -p 1 -r 3 -i 3 -b 456131 \
                -l $O/logs_$k -e kernel -c 1 > $O/procs_$k.r$r.out 2> $O/procs_$k.r$r.err &
        done
        local rc=0 pid
        for pid in $(jobs -p); do wait $pid || rc=$?; done
        local recs
        recs=$(cat $O/logs_$k/tcp-* 2>/dev/null | grep -c .)
        echo "{\"run\": $k, \"rc\": $rc, \"records\": $recs}" >> $O/procs_exit.jsonl
        [ $rc -eq 0 ] || stalls=$((stalls + 1))
        # a stall is a host-side wait (no kernel runs at exit): go on counting;
        # any other failure ends the step
        [ $rc -eq 0 ] || [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 138 ] || return $rc
    done
    echo "procs_exit: $stalls of ${K:-8} runs did not exit cleanly"
    return $stalls
}

stall() {
    make -s -C tools exit_stall_repro >/dev/null || return 1
    local k how rc
    for k in $(seq 1 ${STALL_RUNS:-3}); do
        for how in cycle_fence cycle_barrier; do
            timeout -k 5 120 tools/exit_stall_repro $how ${STALL_CYCLES:-2000} > $O/stall_$how.$k.txt 2>&1
            rc=$?
            echo "{\"run\": $k, \"teardown\": \"$how\", \"cycles\": ${STALL_CYCLES:-2000}, \"rc\": $rc, \"out\": \"$(tail -1 $O/stall_$how.$k.txt)\"}" \
                >> $O/stall.jsonl
            [ $rc -eq 0 ] || [ $rc -eq 3 ] || return $rc
        done
    done
    cat $O/stall.jsonl
}

for s in "$@"; do
    case $s in
    smoke)
        timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1
        step_ok smoke $? ;;
    pytest)
        timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
        rc=$?; tail -3 $O/pytest_gpu.log; step_ok pytest $rc ;;
    pytest:*)
        files=${s#pytest:}
        timeout -k 10 900 python3 -u -m pytest ${files//,/ } -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_sel.log 2>&1
        rc=$?; tail -3 $O/pytest_sel.log; step_ok "$s" $rc ;;
    bench1)
        timeout -k 10 400 python3 -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
        step_ok bench1 $? ;;
    rehearse2) rehearse 2 ;;
    rehearse4) rehearse 4 ;;
    rehearse8) rehearse 8 ;;
    kt)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench \
            -- python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/kt_bench.json 2> $O/kt_bench.err
        step_ok kt $? ;;
    pmc)
        for c in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/pmc_$c -o x \
                -- python3 -u bench.py --no-extras --no-cpu-baseline --no-counters --steps 3 --warmup 1 \
                > $O/pmc_$c.json 2> $O/pmc_$c.err
            step_ok "pmc $c" $?
        done ;;
    stall)
        stall; step_ok stall $? ;;
    procs_exit)
        procs_exit; step_ok procs_exit $? ;;
    linkctl)
        timeout -k 10 200 python3 -u tools/link_counter_control.py > $O/link_counter_control.json 2> $O/link_counter_control.err
        step_ok linkctl $? ;;
    soak)
        timeout -k 10 300 python3 -u tools/soak.py threads 20000 61 > $O/soak_threads.json 2> $O/soak_threads.err
        step_ok "soak threads" $?
        timeout -k 10 300 python3 -u tools/soak.py procs 10000 62 > $O/soak_procs.json 2> $O/soak_procs.err
        step_ok "soak procs" $? ;;
    *)
        echo "unknown step $s"; exit 2 ;;
    esac
done
