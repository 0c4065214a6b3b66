#!/bin/bash
# LL receive polling: one load in flight per lane (the shipped form) vs two
# (the second issued MPX_LL_DUAL = 2 or 5 s_sleep units after the first), for
# messages of one 16-B unit per lane; interleaved twice, measured with
# tools/poll_stagger_ab.py (loopback pair: 8 B / 512 B LL ping-pong, unidir
# per-iteration times, run-hbv3's armed call).  Variants built on the CPU with
# -DMPX_LL_DUAL=N into mpi-perf_amd/lib/variants/libmpx_dualN.so, from an
# uncommitted experiment on wait_ll; it lost (profiles/r04_ll_dual_ab.jsonl).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ll_dual
mkdir -p $O
cp mpi-perf_amd/lib/libmpx.so $O/libmpx_default.so.keep
for pass in ${PASSES:-1 2}; do
  for v in ${VARIANTS:-0 2 5}; do
    cp mpi-perf_amd/lib/variants/libmpx_dual$v.so mpi-perf_amd/lib/libmpx.so
    timeout -k 10 120 python3 -u tools/poll_stagger_ab.py dual$v >> $O/ab.jsonl 2>> $O/ab.err || exit $?
  done
done
cp $O/libmpx_default.so.keep mpi-perf_amd/lib/libmpx.so
cat $O/ab.jsonl
