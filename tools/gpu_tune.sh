#!/bin/bash
mkdir -p gpurun_out
SWEEP=refine timeout -k 10 300 python -u tools/copy_sweep.py > gpurun_out/copy_refine2.jsonl 2>&1 &&
SWEEP=sizes MPX_COPY_VARIANT=4:1:1:1:256 timeout -k 10 300 python -u tools/copy_sweep.py > gpurun_out/copy_sizes2.jsonl 2>&1 &&
SWEEP=sizes MPX_COPY_VARIANT=2:1:1:1:512 timeout -k 10 300 python -u tools/copy_sweep.py >> gpurun_out/copy_sizes2.jsonl 2>&1
echo "rc=$?"
