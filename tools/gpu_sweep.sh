#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/xfer_sweep.py > gpurun_out/xfer_sweep.jsonl 2>&1
MPX_MAILBOX=fine ENGINES=kernel MODES=0 MAXLOG=14 timeout -k 10 120 python -u tools/xfer_sweep.py > gpurun_out/xfer_sweep_fine.jsonl 2>&1
D=$(mktemp -d); (timeout -k 5 60 python -u tools/rccl_probe.py $D 0 > gpurun_out/rccl_probe0.log 2>&1 &); timeout -k 5 60 python -u tools/rccl_probe.py $D 1 > gpurun_out/rccl_probe1.log 2>&1; sleep 2
echo done
