#!/bin/bash
# ref_wrap.sh — per-rank wrapper for running the compiled reference under
# MPICH's mpiexec: ranks [0,PPN) get FAKE_HOST=$HOST1 (they
# match the -f group1 file), the rest $HOST0; Open MPI's local-rank variable,
# which the reference requires (mpi_perf.c:378-384), is derived from PMI_RANK.
# Usage: mpiexec -np N -genv PPN p ref_wrap.sh <binary> <args...>
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")" && pwd)"
if [ "${PMI_RANK:-0}" -lt "${PPN:-1}" ]; then export FAKE_HOST="${HOST1:-vm}"; else export FAKE_HOST="${HOST0:-runsc}"; fi
export OMPI_COMM_WORLD_LOCAL_RANK=$(( ${PMI_RANK:-0} % ${PPN:-1} ))
export LD_PRELOAD="$HERE/_ref/libshim.so${LD_PRELOAD:+:$LD_PRELOAD}"
exec "$@"
