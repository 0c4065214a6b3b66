#!/bin/bash
# one-workgroup waits: one polling wave (stagger 0) vs four staggered waves
# (6, 12 s_sleep units), interleaved twice, then the engine tests on the default.
# The variants were built on the CPU from an uncommitted experiment on
# csrc/mpx_kernels.hip (four waves polling in wait_ll / wait_bulk of a
# one-workgroup grid, wave k starting k x MPX_POLL_STAGGER s_sleep units
# later, the first to see the message claiming it through LDS), with
# -DMPX_POLL_STAGGER=N, into mpi-perf_amd/lib/variants/libmpx_staggerN.so.
# It lost the A/B (profiles/r04_poll_stagger_ab.jsonl) and was not kept.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/poll_stagger
mkdir -p $O
cp mpi-perf_amd/lib/libmpx.so $O/libmpx_default.so.keep
for pass in 1 2; do
  for v in 0 6 12; do
    cp mpi-perf_amd/lib/variants/libmpx_stagger$v.so mpi-perf_amd/lib/libmpx.so
    timeout -k 10 120 python3 -u tools/poll_stagger_ab.py s$v >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
cp $O/libmpx_default.so.keep mpi-perf_amd/lib/libmpx.so
cat $O/ab.jsonl
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_engine.py tests/test_gpu_armed.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; exit $rc
