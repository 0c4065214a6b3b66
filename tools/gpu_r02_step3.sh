#!/bin/bash
# rocprofv3 N=2 rehearsal: exit codes of both profiled processes
ROUND=r02 tools/gpu_prof_n2.sh; rc=$?
echo "prof_n2 rc=$rc"
tail -n 3 gpurun_out/bench_n2_prof_r02.err0 gpurun_out/bench_n2_prof_r02.err1
exit $rc
