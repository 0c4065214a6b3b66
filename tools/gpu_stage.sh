#!/bin/bash
# LDS staging A/B on one GPU: GPU engine tests, then interleaved loopback
# sweeps (ping-pong, -x 1, unidir; 1 B .. 64 MiB) with MPX_STAGE=1 and 0
# (the order flips between the two repetitions).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/stage_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1 || exit 1
for rep in 1 2; do
  order="1 0"; [ $rep = 2 ] && order="0 1"
  for st in $order; do
    MPX_STAGE=$st ENGINES=kernel MODES=0,1,2 MAXLOG=26 timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/stage_tmp.jsonl 2>&1 || exit 1
    sed "s/^{/{\"stage\": $st, \"rep\": $rep, /" gpurun_out/stage_tmp.jsonl >> gpurun_out/stage_ab.jsonl
  done
done
echo "gpu_stage rc=0"
