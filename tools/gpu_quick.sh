#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/xfer_ll_ab.jsonl
for f in 0 1 2 3; do
  MPX_LL_FLAGS=$f ENGINES=kernel MODES=0 MAXLOG=14 timeout -k 10 120 python -u tools/xfer_sweep.py | sed "s/^{/{\"ll_flags\": $f, /" >> gpurun_out/xfer_ll_ab.jsonl 2>&1 || exit 1
done
MPX_MAILBOX=fine MPX_LL_FLAGS=0 ENGINES=kernel MODES=0 MAXLOG=14 timeout -k 10 120 python -u tools/xfer_sweep.py | sed 's/^{/{"ll_flags": "fine0", /' >> gpurun_out/xfer_ll_ab.jsonl 2>&1
echo "rc=$?"
