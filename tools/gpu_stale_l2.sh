#!/bin/bash
# tools/stale_l2_probe on the GPU box: does a check read after an acquire see
# bytes a writer outside this XCD's L2 stored mid-kernel (the cross-GPU case,
# DESIGN.md "Cross-GPU visibility")?  Build first (CPU):
#   hipcc --offload-arch=gfx950 -O2 -o tools/stale_l2_probe tools/stale_l2_probe.hip
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/stale_l2.jsonl
for n in 4194304 1048576 67108864; do
    timeout -k 10 120 tools/stale_l2_probe $n 3 >> gpurun_out/stale_l2.jsonl || exit $?
done
grep -c writer gpurun_out/stale_l2.jsonl
