#!/bin/bash
# rocprofv3 kernel + memory-copy trace of the SDMA engine (mpx_perf -e sdma,
# loopback pair on GPU 0, unidir 4 MiB x 200, graph-replayed chunks): which
# work the runtime's copies become on one GPU, and the engine's per-iteration
# kernels (k_signal / k_wait); then a rank paired with itself, whose copies
# are copy-engine (SDMA) transfers even on one GPU (tools/sdma_self_pair.py).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_sdma
echo vm > gpurun_out/group1_sdma
MPX_PROCESSOR_NAMES=vm,runsc timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/prof_sdma -o sdma -- mpi-perf_amd/bin/mpx_perf -w 2 -e sdma -f gpurun_out/group1_sdma -n 1 -p 1 \
    -u 1 -b 4194304 -i 200 -r 3 -l gpurun_out/logs_sdma > gpurun_out/prof_sdma.log 2>&1
rc=$?
[ $rc -eq 0 ] && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv \
    -d gpurun_out/prof_sdma -o self -- python3 -u tools/sdma_self_pair.py > gpurun_out/prof_sdma_self.log 2>&1
rc=$?
echo "gpu_prof_sdma rc=$rc"
exit $rc
