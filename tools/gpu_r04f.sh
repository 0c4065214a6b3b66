#!/bin/bash
# Round 4, GPU pass f: the armed start waits for grid residency (Status.ready)
# and the first push stages tx into LDS on the way — the armed tests, the
# engine parity tests (every staged push, check mode), the phase split and
# the N=2 one-GPU rehearsal (hbv3_rounds_unidir vs round0_sweep).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${R04_OUT:-r04f}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_armed.py tests/test_gpu_engine.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 python3 -u tools/phase_probe.py 40 armed > $O/phases_armed.jsonl 2> $O/phases_armed.err
rc=$?; echo "phases rc=$rc"; [ $rc -eq 0 ] || exit $rc
MPX_BENCH_ONE_GPU=1 timeout -k 10 400 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 6 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err
rc=$?; echo "bench n2 rc=$rc"; exit $rc
