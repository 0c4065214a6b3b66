#!/bin/bash
# MI355X counterpart of the reference's scripts/run-hbv3.sh: concurrent
# unidirectional flows (-u 1), 456131 B, 10 iterations, runs forever
# (RUNS=-1).  The node's 8 GPUs take the place of two hosts x FLOWS flows:
# with ALL_PAIRS=1 (default) run r is round r mod 7 of the circle-method
# schedule, 4 concurrent pairs per round, so every 7 runs cover all 28 GPU
# pairs; with ALL_PAIRS=0 the pairs are fixed as in the reference
# (--map-by ppr:4:node: rank k <-> rank 4+k).  Every variable below can be
# set from the environment; extra arguments are passed on to mpx_perf.
set -e -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)

ITERS=${ITERS:-10}
RUNS=${RUNS:--1}
FLOWS=${FLOWS:-4}
BUFF_SZ=${BUFF_SZ:-456131}
LOGFOLDER=${LOGFOLDER:-$PWD/tcp-logs}
GPUS=${GPUS:-0,1,2,3,4,5,6,7}     # rank -> GPU (-g)
ENGINE=${ENGINE:-kernel}          # kernel | sdma | rccl
ALL_PAIRS=${ALL_PAIRS:-1}
BINARY=${BINARY:-$HERE/mpi-perf_amd/bin/mpx_perf}

NUM_PROCS=$((2 * FLOWS))
if [ -z "$GROUP1FILE" ]; then
    GROUP1FILE=$(mktemp)
    trap 'rm -f "$GROUP1FILE"' EXIT
    echo "${MPX_HOSTNAME:-$(hostname)}-0" > "$GROUP1FILE"
fi
NUM_GROUP1=${NUM_GROUP1:-1}

"$BINARY" -w ${NUM_PROCS} -g ${GPUS} -e ${ENGINE} -a ${ALL_PAIRS} \
    -f "${GROUP1FILE}" -n ${NUM_GROUP1} -p ${FLOWS} -u 1 -r ${RUNS} -i ${ITERS} -b ${BUFF_SZ} -l "${LOGFOLDER}" "$@"
