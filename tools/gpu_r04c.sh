#!/bin/bash
# Round 4, GPU pass c: armed launches (mpx_xfer_arm) — the armed/disarm GPU
# tests, the phase split armed vs unarmed, then the whole -m gpu suite, the
# N=1 bench with in-process counters and the N=2 one-GPU rehearsal.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04c}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_armed.py -x -v --timeout 120 --timeout-method thread > $O/pytest_armed.log 2>&1
rc=$?; echo "armed tests rc=$rc"; tail -3 $O/pytest_armed.log; [ $rc -eq 0 ] || exit $rc
for a in armed ""; do
    timeout -k 10 150 python3 -u tools/phase_probe.py 40 $a > $O/phases_${a:-unarmed}.jsonl 2> $O/phases_${a:-unarmed}.err
    rc=$?; echo "phases ${a:-unarmed} rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err
rc=$?; echo "bench n1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
rc=$?; echo "bench n2 rc=$rc"; exit $rc
