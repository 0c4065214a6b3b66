#!/bin/bash
# SDMA engine copy kind A/B: hipMemcpyDeviceToDeviceNoCU (default, SDMA) vs
# hipMemcpyDeviceToDevice (blit kernel on one GPU); two interleaved rounds,
# a process each, then the kernel-trace + memory-copy-trace profile of the
# default.  Each step under its own limit; stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sdma_kind_ab.jsonl
for round in 1 2; do
    for k in nocu blit; do
        if [ $k = blit ]; then export MPX_SDMA_KIND=blit; else unset MPX_SDMA_KIND; fi
        timeout -k 10 150 python3 -u tools/sdma_kind_ab.py >> gpurun_out/sdma_kind_ab.jsonl 2>> gpurun_out/sdma_kind_ab.err || exit 1
    done
done
unset MPX_SDMA_KIND
tools/gpu_prof_sdma.sh
