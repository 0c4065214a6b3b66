#!/bin/bash
# A/B of one environment knob on one box: loopback sweeps with VAR=A and VAR=B
# (AB_VAR, AB_A, AB_B), order flipped between the two repetitions.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/envab.jsonl
for rep in 1 2; do
  order="$AB_A $AB_B"; [ $rep = 2 ] && order="$AB_B $AB_A"
  for v in $order; do
    env $AB_VAR=$v ENGINES=${AB_ENGINES:-kernel} MODES=${AB_MODES:-0,1,2} MAXLOG=${AB_MAXLOG:-22} timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/envab_tmp.jsonl 2>&1 || exit 1
    sed "s/^{/{\"$AB_VAR\": \"$v\", \"rep\": $rep, /" gpurun_out/envab_tmp.jsonl >> gpurun_out/envab.jsonl
  done
done
echo "gpu_envab rc=0"
