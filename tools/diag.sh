#!/bin/bash
mkdir -p gpurun_out
L=gpurun_out/diag5.log
run() { echo "=== $1" >> $L; timeout -k 5 120 python -u -m pytest tests/test_gpu_engine.py -m gpu -q --timeout 60 --timeout-method thread -k "$1" 2>&1 | grep -E 'passed|failed|^FAILED' >> $L; }
run "receive_digest"
run "concurrent"
run "(loopback_pair_every_payload and kernel) or concurrent"
run "(loopback_pair_every_payload and sdma) or concurrent"
run "test_copy_kernel or concurrent"
exit 0
