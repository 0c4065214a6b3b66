#!/bin/bash
# full -m gpu suite + smoke + the profiled N=2 rehearsal (exit codes)
tools/gpu_pytest.sh all4 tests && \
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 && \
tools/gpu_r02_step3.sh
