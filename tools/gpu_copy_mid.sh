#!/bin/bash
# k_copy variants at the mid sizes of config 2's sweep (1 MiB - 256 MiB), where
# the one-step default is below its large-size rate: one process per
# (variant, size), tools/copy_sweep.py's "one" mode (avg of 10 launches, best
# of 5), output checked.  MPX_COPY_VARIANT = U:ldnt:stnt:contig:blocks_per_cu.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/copy_mid.jsonl
: > $out
for v in 1:1:1:0:0 2:1:1:0:0 4:1:1:0:0 1:0:0:0:0 1:1:0:0:0 1:0:1:0:0 2:1:1:1:16 4:1:1:1:8 4:1:1:0:16; do
    for n in 1048576 4194304 8388608 16777216 33554432 67108864 134217728 268435456; do
        MPX_COPY_VARIANT=$v timeout -k 10 60 python -u tools/copy_sweep.py one $n >> $out || exit $?
    done
done
echo done
