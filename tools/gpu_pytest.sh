#!/bin/bash
# Run a selection of the -m gpu tests on the GPU box (one process, per-test
# timeout), output to gpurun_out/pytest_<tag>.log.
#   tools/gpu_pytest.sh <tag> <pytest args...>
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${PYTEST_BUDGET:-900} python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "$@" \
    > gpurun_out/pytest_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$tag.log
echo "gpu_pytest $tag rc=$rc"
exit $rc
