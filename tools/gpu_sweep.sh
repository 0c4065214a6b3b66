#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ref_sweep.py > gpurun_out/ref_sweep.jsonl 2>&1
SWEEP=cfg2 timeout -k 10 300 python -u tools/copy_sweep.py > gpurun_out/cfg2_copy_sweep.jsonl 2>&1

ENGINES=sdma MODES=0,2 MAXLOG=22 timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/sdma_kernel_signal.jsonl 2>&1
MPX_SDMA_SIGNAL=cp ENGINES=sdma MODES=0,2 MAXLOG=22 timeout -k 10 200 python -u tools/xfer_sweep.py > gpurun_out/sdma_cp_signal.jsonl 2>&1
MPX_SDMA_SIGNAL=cp timeout -k 10 200 python -u -m pytest tests/test_gpu_engine.py -m gpu -q -k sdma --timeout 60 --timeout-method thread > gpurun_out/sdma_cp_tests.log 2>&1
echo done2
