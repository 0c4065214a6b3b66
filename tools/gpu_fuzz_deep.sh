#!/bin/bash
# One deep pass of the GPU parity fuzz tests against the live compiled
# reference: MPX_FUZZ_EXAMPLES random configurations each (not derandomized,
# so every pass draws new ones), one pytest process, generous per-test limit.
set -o pipefail
mkdir -p gpurun_out
export MPX_FUZZ_EXAMPLES=${MPX_FUZZ_EXAMPLES:-150}
timeout -k 10 800 python -u -m pytest -m gpu -x -v --timeout 700 --timeout-method thread \
    tests/test_integration.py tests/test_gpu_host.py -k random --hypothesis-show-statistics \
    > gpurun_out/fuzz_deep.log 2>&1
rc=$?
grep -E "passing|failing|passed|failed" gpurun_out/fuzz_deep.log
exit $rc
