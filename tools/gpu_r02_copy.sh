#!/bin/bash
# copy A/B (tools/copy_steps_ab.py) + the profiled N=2 rehearsal
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/copy_steps_ab.py 10 > gpurun_out/copy_steps_ab.jsonl 2> gpurun_out/copy_steps_ab.err
echo "copy_steps_ab rc=$?"
tools/gpu_r02_step3.sh
