#!/bin/bash
# Round 4, GPU pass e: which change hangs mpx_perf's processes mode
# (tests/test_gpu_host.py::test_processes_mode_records_match_reference_run
# timed out in r04c): two processes on GPU 0, the test's pingpong case, with
# (a) the defaults (armed, spin barrier, mpx_shutdown), (b) no shutdown,
# (c) not armed; two runs each, bounded; a run that does not end gets
# SIGUSR1 (MPX_DEBUG: every thread's stack) and then SIGKILL.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
PERF=mpi-perf_amd/bin/mpx_perf
echo vm > $O/group1
run() {  # tag, extra env, extra args
    local tag=$1; shift; local envx=$1; shift
    port=$((29600 + RANDOM % 300))
    rm -rf $O/logs_$tag; mkdir -p $O/logs_$tag
    for r in 0 1; do
        env $envx MPX_DEBUG=1 MPX_RANK=$r MPX_SIZE=2 MPX_LOCAL_RANK=$r MPX_PROCESSOR_NAMES=vm,runsc MPX_BOOTSTRAP=127.0.0.1:$port \
            MPX_BOOTSTRAP_TIMEOUT=60 MPX_HOSTNAME=localhost timeout -s USR1 -k 8 40 $PERF -g 0,0 -t 5000 -f $O/group1 -n 1 -p 1 \
            -r 3 -i 3 -b 456131 -l $O/logs_$tag -e kernel -c 1 "$@" > $O/$tag.r$r.out 2> $O/$tag.r$r.err &
    done
    wait; local rc=$?
    echo "$tag: $(grep -c . $O/logs_$tag/tcp-* 2>/dev/null | tail -1) records; rank0 tail: $(tail -1 $O/$tag.r0.err); rank1 tail: $(tail -1 $O/$tag.r1.err)"
}
for k in 1 2; do
    run default_$k ""
    run noshutdown_$k "MPX_PERF_NO_SHUTDOWN=1"
    run unarmed_$k "" -A 0
done
