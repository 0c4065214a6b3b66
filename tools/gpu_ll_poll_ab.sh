#!/bin/bash
# LL poll A/B: MPX_LL_FLAGS=0 (s_sleep 0 between polls) vs 8 (back to back),
# three interleaved rounds, one process each, each under its own limit.
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ll_poll_ab.jsonl
for round in 1 2 3; do
    for f in 0 8; do
        MPX_LL_FLAGS=$f timeout -k 10 120 python3 -u tools/ll_poll_ab.py >> gpurun_out/ll_poll_ab.jsonl 2>> gpurun_out/ll_poll_ab.err || exit 1
    done
done
cat gpurun_out/ll_poll_ab.jsonl
