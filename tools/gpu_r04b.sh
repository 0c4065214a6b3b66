#!/bin/bash
# Round 4, GPU pass b: phases (both completion waits), the whole -m gpu suite
# and smoke over the changed kernels, then the exit-time crash of a process
# that registered the counter tool (r04a: SIGSEGV after the probe's JSON):
# torch-first order with mpx_shutdown, then without rank streams, then the
# failing form with a native stack dump.  Any crash ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
for m in query event; do
    MPX_SYNC=$m timeout -k 10 150 python3 -u tools/phase_probe.py 40 > $O/phases_$m.jsonl 2> $O/phases_$m.err
    rc=$?; echo "phases $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
export MPXPROF_SEGV_DUMP=1
for args in "torch_first shutdown" "no_torch nopair" "no_torch"; do
    tag=${args// /_}
    timeout -k 10 150 python3 -u tools/counters_probe.py $args > $O/counters_$tag.json 2> $O/counters_$tag.err
    rc=$?; echo "counters $args rc=$rc"; [ $rc -le 1 ] || exit $rc
done
