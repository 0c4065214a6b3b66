#!/bin/bash
# MI355X counterpart of the reference's scripts/run-1-pair.sh: one pair over
# xGMI (GPU 0 = group 1, GPU 1 = group 0), the full-duplex non-blocking loop
# (-x 1), 4 MiB, 5000 iterations, 10 runs.  The reference's two hosts become
# the two virtual hosts of this node (ranks [0, FLOWS) and [FLOWS, 2 FLOWS));
# mpirun's -np becomes -w.  Every variable below can be set from the
# environment; extra arguments are passed on to mpx_perf (e.g. -c 1).
set -e -o pipefail
HERE=$(cd "$(dirname "$0")/.." && pwd)

ITERS=${ITERS:-5000}
RUNS=${RUNS:-10}
FLOWS=${FLOWS:-1}
BUFF_SZ=${BUFF_SZ:-4194304}
LOGFOLDER=${LOGFOLDER:-$PWD/mpi-perf-logs}
GPUS=${GPUS:-0,1}                 # rank -> GPU (-g)
ENGINE=${ENGINE:-kernel}          # kernel | sdma | rccl
BINARY=${BINARY:-$HERE/mpi-perf_amd/bin/mpx_perf}

NUM_PROCS=$((2 * FLOWS))
if [ -z "$GROUP1FILE" ]; then
    GROUP1FILE=$(mktemp)
    trap 'rm -f "$GROUP1FILE"' EXIT
    # group 1 = virtual host 0, the processor name of ranks [0, FLOWS)
    echo "${MPX_HOSTNAME:-$(hostname)}-0" > "$GROUP1FILE"
fi
NUM_GROUP1=${NUM_GROUP1:-1}

"$BINARY" -w ${NUM_PROCS} -g ${GPUS} -e ${ENGINE} \
    -f "${GROUP1FILE}" -n ${NUM_GROUP1} -p ${FLOWS} -r ${RUNS} -i ${ITERS} -b ${BUFF_SZ} -l "${LOGFOLDER}" -x 1 "$@"
