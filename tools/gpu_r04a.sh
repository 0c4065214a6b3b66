#!/bin/bash
# Round 4, first GPU pass: in-process counters in three load orders, the
# per-call phase split under both completion waits, then the whole -m gpu
# suite and smoke over the changed kernels (last workgroup resets scratch,
# completion word) and knobs.  A probe that ends with a signal / timeout
# ends the script; a Python error (rc 1) does not.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
for ord in no_torch torch_first prof_first; do
    timeout -k 10 150 python3 -u tools/counters_probe.py $ord > $O/counters_$ord.json 2> $O/counters_$ord.err
    rc=$?; echo "counters $ord rc=$rc"; [ $rc -le 1 ] || exit $rc
done
for m in query event; do
    MPX_SYNC=$m timeout -k 10 150 python3 -u tools/phase_probe.py 40 > $O/phases_$m.jsonl 2> $O/phases_$m.err
    rc=$?; echo "phases $m rc=$rc"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; exit $rc
