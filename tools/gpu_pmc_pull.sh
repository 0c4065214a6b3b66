#!/bin/bash
# PMC passes over the pull kernel (k_xfer_pull, MPX_XFER_PULL) beside the
# push kernel on the same box: FETCH_SIZE and WRITE_SIZE in separate runs
# per case (tools/pmc_xfer.py workloads), then where the pull's reads go
# (EA read requests in total / to DRAM).  The question: does every pulled
# iteration read its B bytes from memory (system-scope loads), or are later
# iterations served from the L2?  Outputs under gpurun_out/pmc_pull/.
set -o pipefail
export TMPDIR=/tmp
# Under rocprofv3 --pmc a process that leaves its pooled rank streams to the
# runtime (libmpx's default exit order) segfaults in __cxa_finalize after the
# profiler wrote its output (seen on the first pass of this script): the
# runtime tears the streams down after the tool finalized.  Round 2's exit
# order (drain, 50 ms, destroy in libmpx's exit handler, which runs before
# the tool's) keeps these runs clean.
O=gpurun_out/pmc_pull
mkdir -p $O
run_self() {   # name variant B iters [env]
    local name=$1 v=$2 b=$3 it=$4
    for ctr in FETCH_SIZE WRITE_SIZE; do
        env $5 timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py self $v $b $it > $O/${name}_$ctr.log 2>&1 || { echo "$name $ctr failed"; return 1; }
    done
    echo "$name ok: $(tail -1 $O/${name}_WRITE_SIZE.log)"
}
run_pair() {   # name mode B iters check pull
    local name=$1 m=$2 b=$3 it=$4 ck=$5 pl=$6
    for ctr in FETCH_SIZE WRITE_SIZE; do
        d=$(mktemp -d)
        timeout -s KILL 90 python3 -u tools/pmc_xfer.py pair $d 1 $m $b $it $ck $pl > $O/${name}_${ctr}_r1.log 2>&1 &
        p1=$!
        timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py pair $d 0 $m $b $it $ck $pl > $O/${name}_$ctr.log 2>&1
        r0=$?
        wait $p1; r1=$?
        [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { echo "$name $ctr failed $r0/$r1"; return 1; }
    done
    echo "$name ok: $(tail -1 $O/${name}_WRITE_SIZE.log)"
}
for b in 4096 456131 4194304 67108864; do
    run_self nbpull_$b nbpull $b 256 || exit 1
    run_self nbpush_$b nb_hbm $b 256 || exit 1
done
run_self nbpullcheck_4194304 nbpullcheck 4194304 256 || exit 1
run_pair uni_pull_4194304 unidir 4194304 500 0 pull || exit 1
run_pair uni_push_4194304 unidir 4194304 500 0 push || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv \
    -d $O/nbpull_4194304_EA -o x -- python3 -u tools/pmc_xfer.py self nbpull 4194304 256 > $O/nbpull_4194304_EA.log 2>&1 || exit 1
echo "pmc_pull done"
