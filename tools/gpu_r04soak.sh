#!/bin/bash
# Round 4 soak of the kernel engine's pair protocol on the final tree (armed
# and cancelled calls, workgroup 0 ending every call, the sealed completion
# line): threads and processes (one with a lagging receiver workgroup), the
# SDMA engine, then the receive-posted negative control (expected to report
# failures: exit 1).
set -o pipefail
O=gpurun_out/r04soak
mkdir -p $O
timeout -k 10 300 python -u tools/soak.py threads 20000 51 > $O/soak_threads.json 2> $O/soak_threads.err || exit $?
timeout -k 10 300 python -u tools/soak.py procs 10000 52 > $O/soak_procs.json 2> $O/soak_procs.err || exit $?
MPX_TEST=lag_wg=1:-1:2000 timeout -k 10 300 python -u tools/soak.py threads 5000 53 > $O/soak_threads_lag.json 2> $O/soak_threads_lag.err || exit $?
timeout -k 10 200 python -u tools/soak.py threads 3000 54 sdma > $O/soak_sdma.json 2> $O/soak_sdma.err || exit $?
MPX_TEST=no_posted,lag_wg=1:-1:2000 timeout -k 10 300 python -u tools/soak.py threads 3000 55 > $O/soak_neg_posted.json 2> $O/soak_neg_posted.err
rc=$?; [ $rc -le 1 ] || exit $rc
cut -c1-400 $O/soak_threads.json $O/soak_procs.json $O/soak_threads_lag.json $O/soak_sdma.json $O/soak_neg_posted.json
