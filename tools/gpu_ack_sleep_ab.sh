#!/bin/bash
# The multi-workgroup LL wait (a bulk sender's workgroups waiting for the
# unidir 1-byte ack): s_sleep 0 between polls (shipped) vs 1 and 3 (fewer
# polls of the one word every sending workgroup reads), interleaved; variants
# built on the CPU with -DMPX_ACK_SLEEP=N (an uncommitted experiment on
# wait_ll) into mpi-perf_amd/lib/variants/libmpx_ackN.so.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ack_sleep
mkdir -p $O
cp mpi-perf_amd/lib/libmpx.so $O/libmpx_default.so.keep
for pass in 1 2 3 4; do
  for v in 0 1 3; do
    cp mpi-perf_amd/lib/variants/libmpx_ack$v.so mpi-perf_amd/lib/libmpx.so
    timeout -k 10 120 python3 -u tools/poll_stagger_ab.py ack$v >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
cp $O/libmpx_default.so.keep mpi-perf_amd/lib/libmpx.so
cat $O/ab.jsonl
