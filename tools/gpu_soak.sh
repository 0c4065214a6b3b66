#!/bin/bash
# soak: SDMA engine, then the two negative controls (expected to report failures: exit 1)
set -o pipefail
O=gpurun_out
timeout -k 10 200 python -u tools/soak.py threads 3000 21 sdma > $O/soak_sdma.json 2> $O/soak_sdma.err || exit $?
timeout -k 10 200 python -u tools/soak.py procs 2000 22 sdma > $O/soak_sdma_procs.json 2> $O/soak_sdma_procs.err || exit $?
MPX_TEST=no_posted timeout -k 10 200 python -u tools/soak.py threads 1500 23 > $O/soak_neg_posted.json 2> $O/soak_neg_posted.err
rc=$?; [ $rc -le 1 ] || exit $rc
MPX_TEST=no_pull_wait,lag_wg=1:-1:2000 timeout -k 10 200 python -u tools/soak.py threads 1500 24 > $O/soak_neg_pullwait.json 2> $O/soak_neg_pullwait.err
rc=$?; [ $rc -le 1 ] || exit $rc
cat $O/soak_sdma.json $O/soak_sdma_procs.json $O/soak_neg_posted.json $O/soak_neg_pullwait.json | cut -c1-600
