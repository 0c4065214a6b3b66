#!/bin/bash
# tests/test_gpu_multi.py (the multi-GPU suite: configs 3/4/5) rehearsed on
# ONE GPU: every rank on GPU 0, the cross-GPU LL threshold forced, RCCL and
# the link-table checks skipped (see the module docstring).  Proves the
# tests' own code before a multi-GPU node runs them for real.
set -o pipefail
mkdir -p gpurun_out
export MPX_MULTI_REHEARSE=1 MPX_LL_MAX=8192 MPX_MULTI_REHEARSE_N=${MPX_MULTI_REHEARSE_N:-4}
timeout -k 10 1000 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests/test_gpu_multi.py \
    > gpurun_out/multi_rehearse.log 2>&1
rc=$?
tail -3 gpurun_out/multi_rehearse.log
exit $rc
