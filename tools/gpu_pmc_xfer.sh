#!/bin/bash
# PMC passes over the pair kernel (tools/pmc_xfer.py): FETCH_SIZE and
# WRITE_SIZE in separate runs per case, each under its own time limit; then
# the counter list of this box (xGMI counter names).  Outputs under
# gpurun_out/pmc_xfer/<case>_<counter>/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_xfer
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/rocprofv3_L.txt 2>&1; echo "list rc=$?"
run_self() {   # name variant B iters [env]
    local name=$1 v=$2 b=$3 it=$4
    for ctr in FETCH_SIZE WRITE_SIZE; do
        env $5 timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py self $v $b $it > $O/${name}_$ctr.log 2>&1 || { echo "$name $ctr failed"; return 1; }
    done
    echo "$name ok: $(tail -1 $O/${name}_WRITE_SIZE.log)"
}
run_pair() {   # name mode B iters check
    local name=$1 m=$2 b=$3 it=$4 ck=$5
    for ctr in FETCH_SIZE WRITE_SIZE; do
        d=$(mktemp -d)
        timeout -s KILL 90 python3 -u tools/pmc_xfer.py pair $d 1 $m $b $it $ck > $O/${name}_${ctr}_r1.log 2>&1 &
        p1=$!
        timeout -s KILL 90 rocprofv3 --pmc $ctr --output-format csv -d $O/${name}_$ctr -o x \
            -- python3 -u tools/pmc_xfer.py pair $d 0 $m $b $it $ck > $O/${name}_$ctr.log 2>&1
        r0=$?
        wait $p1; r1=$?
        [ $r0 -eq 0 ] && [ $r1 -eq 0 ] || { echo "$name $ctr failed $r0/$r1"; return 1; }
    done
    echo "$name ok: $(tail -1 $O/${name}_WRITE_SIZE.log)"
}
for b in 4096 456131 4194304; do
    run_self nb_$b nb $b 512 || exit 1
    run_self nbhbm_$b nb_hbm $b 512 || exit 1
    run_self nbcheck_$b nbcheck $b 512 || exit 1
done
run_pair pp_ll_8 pingpong 8 4000 0 || exit 1
run_pair pp_ll_1024 pingpong 1024 4000 0 || exit 1
run_pair pp_llcheck_1024 pingpong 1024 4000 1 || exit 1
run_pair uni_bulk_456131 unidir 456131 500 0 || exit 1
run_pair uni_bulkcheck_456131 unidir 456131 500 1 || exit 1
run_pair uni_bulk_4194304 unidir 4194304 500 0 || exit 1
# where the writes go: EA write requests in total / 64-B ones / to local DRAM
# / to GMI (the inter-die / peer fabric) — on a loopback pair every byte is
# local, so total - DRAM is the recipe's zero point
for c in nb_4194304:nb:4194304 uni_bulk_4194304:unidir:4194304; do
    IFS=: read name m b <<< "$c"
    if [ $m = nb ]; then
        timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv \
            -d $O/${name}_EA -o x -- python3 -u tools/pmc_xfer.py self nb $b 512 > $O/${name}_EA.log 2>&1 || exit 1
        timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_RDREQ_GMI_32B_sum --output-format csv \
            -d $O/${name}_GMI -o x -- python3 -u tools/pmc_xfer.py self nb $b 512 > $O/${name}_GMI.log 2>&1 || exit 1
    fi
done
echo "pmc_xfer done"
