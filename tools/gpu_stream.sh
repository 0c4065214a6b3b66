#!/bin/bash
# Streaming-hint A/B on one GPU (loopback): bulk payload stores sc0 sc1
# (MPX_PUSH_STREAM=0) against sc0 sc1 nt (=1), 16 KiB .. 64 MiB, order
# flipped between the two repetitions.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/stream_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1 || exit 1
for rep in 1 2; do
  order="1 0"; [ $rep = 2 ] && order="0 1"
  for st in $order; do
    MPX_PUSH_STREAM=$st ENGINES=kernel MODES=0,1,2 MAXLOG=26 timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/stream_tmp.jsonl 2>&1 || exit 1
    sed "s/^{/{\"stream\": $st, \"rep\": $rep, /" gpurun_out/stream_tmp.jsonl >> gpurun_out/stream_ab.jsonl
  done
done
echo "gpu_stream rc=0"
