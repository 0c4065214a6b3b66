#!/bin/bash
# Stream churn: does creating and destroying CU-masked streams over and over
# in one process (the safe order: allocate, create, launch, free, destroy)
# hang by itself?  That is what the -m gpu suite did ~60 contexts in when
# mpx_finalize destroyed its rank streams (profiles/r02_stream_destroy_suite_hang.txt).
# 100 cycles of CU-masked streams, then 100 of ordinary streams as the
# control; each process under a 60 s limit.
mkdir -p gpurun_out
out=gpurun_out/stream_churn.txt
: > $out
cyc() { local kind=$1 n=$2 s=""; for i in $(seq 1 $n); do s="$s a0 ${kind}0 k0.0 f0 d0"; done; echo "$s"; }
for kind in m p; do
    timeout -k 5 60 tools/stream_teardown "$(cyc $kind 100)" > gpurun_out/churn_$kind.txt 2>&1
    rc=$?
    echo "[$kind x100] rc=$rc steps_done=$(tr ' ' '\n' < gpurun_out/churn_$kind.txt | grep -c '^d0') last=$(tail -c 80 gpurun_out/churn_$kind.txt | tr '\n' ' ')" | tee -a $out
done
