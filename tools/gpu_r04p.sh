#!/bin/bash
# Round 4, GPU pass p: armed calls post their receives when their kernel runs
# — armed, engine and ordering tests, the protocol soak with armed and
# cancelled calls, and the N=2 rehearsal (posted wait in run-hbv3's phases).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04p}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_armed.py tests/test_gpu_engine.py tests/test_gpu_ordering.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/soak.py threads 20000 61 > $O/soak_threads.json 2> $O/soak_threads.err || exit $?
timeout -k 10 300 python -u tools/soak.py procs 10000 62 > $O/soak_procs.json 2> $O/soak_procs.err || exit $?
cut -c1-300 $O/soak_threads.json $O/soak_procs.json
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
rc=$?; echo "bench n2 rc=$rc"; exit $rc
