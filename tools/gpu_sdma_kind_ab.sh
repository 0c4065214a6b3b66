#!/bin/bash
# SDMA engine copy kind A/B on a loopback pair: hipMemcpyDeviceToDeviceNoCU
# (MPX_SDMA_KIND=nocu: SDMA) vs hipMemcpyDeviceToDevice (blit kernel on one
# GPU); two interleaved rounds, a process each, then the kernel-trace +
# memory-copy-trace profiles (tools/gpu_prof_sdma.sh).  The forced NoCU run
# timed out in round 2 (shared SDMA queues), so the loopback default is the
# blit kind (mpx_runtime.hip sdma_kind).  Stop at the first failure.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/sdma_kind_ab.jsonl
for round in 1 2; do
    for k in nocu blit; do
        export MPX_SDMA_KIND=$k
        timeout -k 10 150 python3 -u tools/sdma_kind_ab.py >> gpurun_out/sdma_kind_ab.jsonl 2>> gpurun_out/sdma_kind_ab.err || exit 1
    done
done
unset MPX_SDMA_KIND
tools/gpu_prof_sdma.sh
