#!/bin/bash
# Round 4, GPU pass d: exit 0 under rocprofv3 --pmc in the default exit
# order (finalize, then mpx_shutdown: VERDICT r03 next 5a), the committed
# kernel-trace and PMC passes of the N=1 bench, and the N=8 one-GPU
# rehearsal with RCCL first among the comparison engines (refused before
# init when ranks share a GPU: VERDICT r03 next 5b).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04d}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_self -o x \
    -- python3 -u tools/pmc_xfer.py self nbpull 4096 256 > $O/pmc_self.log 2>&1
rc=$?; echo "self pair under --pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_bench -o x \
    -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/pmc_bench.json 2> $O/pmc_bench.err
rc=$?; echo "bench under --pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench \
    -- python3 -u bench.py --no-cpu-baseline --no-extras --steps 20 --warmup 5 > $O/kt_bench.json 2> $O/kt_bench.err
rc=$?; echo "bench kernel-trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 8 --steps 14 --warmup 7 > $O/bench_n8.json 2> $O/bench_n8.err
rc=$?; echo "bench n8 rc=$rc"; exit $rc
