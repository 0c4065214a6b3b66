#!/bin/bash
# HBM traffic of the N = 1 headline kernel (k_copy, 1 GiB) from the bench
# command itself: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate
# passes (MI355X_MICROARCH.md HBM section), summarised by tools/pmc_summary.py
# into gpurun_out/pmc_local_d2d_copy.json (bench.py reads profiles/'s copy as
# roofline.traffic).  The second pass runs only if the first exited cleanly.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_headline
mkdir -p $O
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o x \
    -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/fetch.json 2> $O/fetch.err
rc=$?; echo "fetch pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o x \
    -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/write.json 2> $O/write.err
rc=$?; echo "write pass rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $O/fetch/x_counter_collection.csv $O/write/x_counter_collection.csv \
    gpurun_out/pmc_local_d2d_copy.json 1073741824
