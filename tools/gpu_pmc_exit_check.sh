#!/bin/bash
# rocprofv3 --pmc over libmpx workloads with libmpx's default exit order:
# each must exit 0 (round 3: the default order segfaulted in __cxa_finalize
# under --pmc until destroy_stream_pool switched to round 2's order there).
# The second step runs only if the first exited cleanly.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_exit
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/self -o x \
    -- python3 -u tools/pmc_xfer.py self nbpull 4096 256 > $O/self.log 2>&1
rc=$?; echo "self_pair_pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/bench -o x \
    -- python3 -u bench.py --no-extras --no-cpu-baseline --steps 3 --warmup 1 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench_pmc rc=$rc"; exit $rc
