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
#   refplace         tools/ref_placement.py: the reference's host rate under each rank placement (CPU only)
#   soak             tools/soak.py: threads + processes + SDMA, then the two negative controls
#   fuzz             the live-reference parity fuzz tests (MPX_FUZZ_EXAMPLES, default 150)
#   multi_rehearse   tests/test_gpu_multi.py with every rank on GPU 0 (MPX_MULTI_REHEARSE)
#   stale_l2         tools/stale_l2_probe at 1, 4, 64 MiB
#   validate         mpx_perf with every payload checked, kernel + SDMA, 1 pair and 4 pairs
#   pmc_xfer         FETCH/WRITE_SIZE + EA passes of the pair kernel (tools/pmc_xfer.py), push and pull
#   prof_sdma        kernel + memory-copy trace of the SDMA engine
#   node_profileN    tools/node_profile.sh at N ranks on one GPU (N = 2)
#   node             the FIRST run on a multi-GPU node (refuses with fewer than 8
#                    GPUs): the link-counter control across GPU 0 -> 1, the
#                    multi-GPU suite on distinct GPUs, bench.py at N = 2, 4, 8
#                    (one rank per GPU), then tools/node_profile.sh at N = 8
#   node_rehearse    the same recipe on one GPU (every rank on GPU 0)
# Environment: K (procs_exit runs, default 8), STALL_CYCLES (default 2000),
# STALL_RUNS (default 3).
# Round 4's per-pass wrappers (gpu_r04*.sh) and the older single-purpose
# ones (gpu_full, gpu_pytest, gpu_soak, gpu_fuzz_deep, gpu_multi_rehearse,
# gpu_stale_l2, gpu_validate, gpu_pmc_*, gpu_prof_*, gpu_exit_stall) are these
# steps; profiles/INDEX.md maps each evidence file to its step.
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
    local n=$1 t0=$SECONDS
    MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29520 + n + RANDOM % 200)) bench.py --gpus $n \
        > $O/bench_n$n.json 2> $O/bench_n$n.err
    local rc=$?
    echo "rehearse$n: $((SECONDS - t0)) s"
    step_ok rehearse$n $rc
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

pmc_self() {   # name variant B iters: FETCH_SIZE and WRITE_SIZE passes of a self pair
    local name=$1 v=$2 b=$3 it=$4 ctr
    for ctr in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py self $v $b $it > $O/pmc_${name}_$ctr.log 2>&1 || { echo "$name $ctr failed"; return 1; }
    done
}

pmc_pair() {   # name mode B iters check push|pull: rank 0 profiled, rank 1 beside it
    local name=$1 m=$2 b=$3 it=$4 ck=$5 pl=$6 ctr d p1 r0 r1
    for ctr in FETCH_SIZE WRITE_SIZE; do
        d=$(mktemp -d)
        timeout -s KILL 90 python3 -u tools/pmc_xfer.py pair $d 1 $m $b $it $ck $pl > $O/pmc_${name}_${ctr}_r1.log 2>&1 &
        p1=$!
        timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py pair $d 0 $m $b $it $ck $pl > $O/pmc_${name}_$ctr.log 2>&1
        r0=$?
        wait $p1; r1=$?
        [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { echo "$name $ctr failed $r0/$r1"; return 1; }
    done
}

pmc_xfer() {
    local b
    for b in 4096 456131 4194304; do
        pmc_self nb_$b nb $b 512 && pmc_self nbhbm_$b nb_hbm $b 512 && pmc_self nbcheck_$b nbcheck $b 512 &&
            pmc_self nbpull_$b nbpull $b 256 || return 1
    done
    pmc_pair pp_ll_8 pingpong 8 4000 0 push && pmc_pair pp_llcheck_1024 pingpong 1024 4000 1 push &&
        pmc_pair uni_bulk_456131 unidir 456131 500 0 push && pmc_pair uni_bulk_4194304 unidir 4194304 500 0 push &&
        pmc_pair uni_pull_4194304 unidir 4194304 500 0 pull || return 1
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv \
        -d $O/pmc_EA -o x -- python3 -u tools/pmc_xfer.py self nb 4194304 512 > $O/pmc_EA.log 2>&1 &&
    timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_RDREQ_GMI_32B_sum --output-format csv \
        -d $O/pmc_GMI -o x -- python3 -u tools/pmc_xfer.py self nb 4194304 512 > $O/pmc_GMI.log 2>&1
}

validate() {   # mpx_perf, every payload checked (-c 2), two ranks / eight ranks on GPU 0
    local eng m flag
    echo vm > $O/group1
    for eng in kernel sdma; do
        for m in pp uni nb; do
            flag=""; [ $m = uni ] && flag="-u 1"; [ $m = nb ] && flag="-x 1"
            MPX_PROCESSOR_NAMES=vm,runsc timeout -k 10 240 $PERF -w 2 -g 0,0 -e $eng -c 2 -t 10000 -f $O/group1 -n 1 -p 1 \
                -r 2 -i 7 -S 1:67108864 $flag -l $O/validate_${eng}_$m > $O/validate_${eng}_$m.log 2>&1 || return 1
        done
        MPX_PROCESSOR_NAMES=vm,vm,vm,vm,runsc,runsc,runsc,runsc timeout -k 10 240 $PERF -w 8 -g 0,0,0,0,0,0,0,0 \
            -e $eng -c 2 -t 10000 -f $O/group1 -n 1 -p 4 -u 1 -r 2 -i 7 -S 1024:4194304 \
            -l $O/validate_${eng}_4pairs > $O/validate_${eng}_4pairs.log 2>&1 || return 1
    done
    python3 - $O <<'PY'
import csv, glob, os, sys
rows = []
for d in sorted(glob.glob(sys.argv[1] + "/validate_*/")):
    for f in sorted(glob.glob(d + "gpu-*.csv")):
        rows += [dict(run=os.path.basename(d.rstrip("/")), **r) for r in csv.DictReader(open(f))]
bad = [r for r in rows if r["CheckFailures"] != "0"]
print(f"{len(rows)} transfer records, {sum(int(r['CheckedPayloads']) for r in rows)} payloads checked, {len(bad)} with failures")
sys.exit(1 if bad or not rows else 0)
PY
}

soak() {
    timeout -k 10 300 python3 -u tools/soak.py threads 20000 61 > $O/soak_threads.json 2> $O/soak_threads.err &&
    timeout -k 10 300 python3 -u tools/soak.py procs 10000 62 > $O/soak_procs.json 2> $O/soak_procs.err &&
    timeout -k 10 200 python3 -u tools/soak.py threads 3000 63 sdma > $O/soak_sdma.json 2> $O/soak_sdma.err || return $?
    local rc
    # negative controls: expected to report failures (exit 1)
    MPX_TEST=no_posted,lag_wg=1:-1:2000 timeout -k 10 300 python3 -u tools/soak.py threads 3000 64 \
        > $O/soak_neg_posted.json 2> $O/soak_neg_posted.err
    rc=$?; [ $rc -le 1 ] || return $rc
    MPX_TEST=no_pull_wait,lag_wg=1:-1:2000 timeout -k 10 200 python3 -u tools/soak.py threads 1500 65 \
        > $O/soak_neg_pullwait.json 2> $O/soak_neg_pullwait.err
    rc=$?; [ $rc -le 1 ] || return $rc
    cut -c1-400 $O/soak_*.json
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
    refplace)
        timeout -k 10 600 python3 -u tools/ref_placement.py 3 > $O/ref_placement.json 2> $O/ref_placement.err
        step_ok refplace $? ;;
    soak)
        soak; step_ok soak $? ;;
    fuzz)
        MPX_FUZZ_EXAMPLES=${MPX_FUZZ_EXAMPLES:-150} timeout -k 10 800 python3 -u -m pytest -m gpu -x -v --timeout 700 \
            --timeout-method thread tests/test_integration.py tests/test_gpu_host.py -k random --hypothesis-show-statistics \
            > $O/fuzz.log 2>&1
        rc=$?; grep -E "passing|failing|passed|failed" $O/fuzz.log; step_ok fuzz $rc ;;
    multi_rehearse)
        MPX_MULTI_REHEARSE=1 MPX_LL_MAX=8192 MPX_MULTI_REHEARSE_N=${MPX_MULTI_REHEARSE_N:-4} timeout -k 10 1000 \
            python3 -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py \
            > $O/multi_rehearse.log 2>&1
        rc=$?; tail -3 $O/multi_rehearse.log; step_ok multi_rehearse $rc ;;
    stale_l2)
        make -s -C tools stale_l2_probe >/dev/null || exit 1
        : > $O/stale_l2.jsonl
        for n in 4194304 1048576 67108864; do
            timeout -k 10 120 tools/stale_l2_probe $n 3 >> $O/stale_l2.jsonl
            step_ok "stale_l2 $n" $?
        done ;;
    validate)
        validate; step_ok validate $? ;;
    pmc_xfer)
        pmc_xfer; step_ok pmc_xfer $? ;;
    prof_sdma)
        echo vm > $O/group1
        MPX_PROCESSOR_NAMES=vm,runsc timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
            -d $O/prof_sdma -o sdma -- $PERF -w 2 -e sdma -f $O/group1 -n 1 -p 1 -u 1 -b 4194304 -i 200 -r 3 \
            -l $O/logs_sdma > $O/prof_sdma.log 2>&1
        step_ok prof_sdma $? ;;
    node|node_rehearse)
        # node_rehearse: the same script on ONE GPU (every rank on GPU 0:
        # MPX_BENCH_ONE_GPU for bench.py and node_profile.sh, the multi-GPU
        # suite's own rehearsal), so the node run's recipe itself is proven
        ngpu=$(python3 -c 'import sys; sys.path.insert(0, "mpi-perf_amd"); import mpx; print(mpx.device_count())')
        one=""
        if [ $s = node_rehearse ]; then one=1; else
            [ "$ngpu" -ge 8 ] || { echo "node: $ngpu GPU(s) visible, 8 needed"; exit 2; }
        fi
        timeout -k 10 300 python3 -u tools/link_counter_control.py > $O/link_counter_control.json 2> $O/link_counter_control.err
        step_ok "node linkctl" $?
        timeout -k 10 1200 python3 -u -m pytest tests/test_gpu_multi.py -m gpu -x -v --timeout 300 --timeout-method thread \
            > $O/pytest_multi.log 2>&1
        step_ok "node multi-GPU suite" $?
        for n in 2 4 8; do
            MPX_BENCH_ONE_GPU=$one timeout -k 10 900 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
                --master-addr 127.0.0.1 --master-port $((29700 + n)) bench.py --gpus $n \
                > $O/bench_node_n$n.json 2> $O/bench_node_n$n.err
            step_ok "node bench n$n" $?
        done
        N=8 MPX_BENCH_ONE_GPU=$one tools/node_profile.sh > $O/node_profile_n8.log 2>&1
        step_ok "node profile n8" $? ;;
    node_profile2)
        N=2 MPX_BENCH_ONE_GPU=1 tools/node_profile.sh > $O/node_profile_n2.log 2>&1
        rc=$?; tail -3 $O/node_profile_n2.log; step_ok node_profile2 $rc ;;
    *)
        echo "unknown step $s"; exit 2 ;;
    esac
done
