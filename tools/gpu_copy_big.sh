#!/bin/bash
# Cache-policy A/B of the one-step k_copy at the large sizes (512 MiB - 4 GiB),
# two interleaved passes: nontemporal vs plain loads / stores.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/copy_big.jsonl
: > $out
for pass in 1 2; do
    for n in 536870912 1073741824 2147483648 4294967296; do
        for v in 1:1:1:0:0 1:0:1:0:0 1:0:0:0:0 1:1:0:0:0; do
            MPX_COPY_VARIANT=$v timeout -k 10 60 python -u tools/copy_sweep.py one $n >> $out || exit $?
        done
    done
done
echo done
