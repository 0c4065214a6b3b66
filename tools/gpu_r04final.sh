#!/bin/bash
# Round 4, final GPU pass on the final tree: the whole -m gpu suite, smoke,
# bench N=1 (in-process counters) and the one-GPU rehearsals at N=2, 4, 8
# (cpu_baseline in run-hbv3's layout beside each).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04final}
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench n1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for n in 2 4 8; do
    MPX_BENCH_ONE_GPU=1 timeout -k 10 600 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29520 + n)) bench.py --gpus $n > $O/bench_n$n.json 2> $O/bench_n$n.err
    rc=$?; echo "bench n$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
