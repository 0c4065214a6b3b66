#!/bin/bash
# Where the pair kernel's writes go: EA write requests in
# total / 64-B ones / to local DRAM, and the GMI (peer-fabric) request
# counters, over the self-paired non-blocking loop at 4 MiB (tools/pmc_xfer.py).
# On one GPU every byte is local: total - DRAM and the GMI counters are the
# recipe's zero point.  Each pass its own run and time limit.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc_ea
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/rocprofv3_L.txt 2>&1
grep -oE "TCC_EA0_(WR|RD)REQ[A-Z0-9_]*" $O/rocprofv3_L.txt | sort -u > $O/ea_counters.txt || true
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_DRAM_sum --output-format csv \
    -d $O/EA -o x -- python3 -u tools/pmc_xfer.py self nb 4194304 512 > $O/EA.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_WRITE_GMI_32B_sum TCC_EA0_RDREQ_GMI_32B_sum --output-format csv \
    -d $O/GMI -o x -- python3 -u tools/pmc_xfer.py self nb 4194304 512 > $O/GMI.log 2>&1
rc=$?
echo "pmc_ea rc=$rc"
exit $rc
