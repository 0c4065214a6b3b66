#!/bin/bash
# A/B of two libmpx builds on one box: loopback sweeps (ping-pong, -x 1,
# unidir; 1 B .. 4 MiB) with lib/libmpx.so and lib/libmpx_prev.so, order
# flipped between the two repetitions.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/libab.jsonl
for rep in 1 2; do
  order="cur prev"; [ $rep = 2 ] && order="prev cur"
  for v in $order; do
    lib=mpi-perf_amd/lib/libmpx.so; [ $v = prev ] && lib=mpi-perf_amd/lib/libmpx_prev.so
    MPX_LIB=$PWD/$lib ENGINES=${AB_ENGINES:-kernel} MODES=0,1,2 MAXLOG=${AB_MAXLOG:-22} timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/libab_tmp.jsonl 2>&1 || exit 1
    sed "s/^{/{\"lib\": \"$v\", \"rep\": $rep, /" gpurun_out/libab_tmp.jsonl >> gpurun_out/libab.jsonl
  done
done
echo "gpu_libab rc=0"
