#!/bin/bash
# LL protocol A/B on one GPU: GPU engine tests, then interleaved loopback
# sweeps of the ping-pong and unidir loops up to 16 KiB with the cross-GPU
# 8 KiB LL threshold forced (MPX_LL_MAX): register-held payload (flags 0)
# against a tx re-read at every send (flags 4).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/ll_ab.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1 || exit 1
for rep in 1 2; do
  for f in ${FLAGS:-0 4}; do
    MPX_LL_FLAGS=$f MPX_LL_MAX=8192 ENGINES=kernel MODES=0,2 MAXLOG=14 timeout -k 10 120 python -u tools/xfer_sweep.py > gpurun_out/ll_tmp.jsonl 2>&1 || exit 1
    sed "s/^{/{\"ll_flags\": $f, \"rep\": $rep, /" gpurun_out/ll_tmp.jsonl >> gpurun_out/ll_ab.jsonl
  done
done
echo "gpu_ll rc=0"
