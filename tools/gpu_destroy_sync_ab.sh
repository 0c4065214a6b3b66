#!/bin/bash
# Rank streams destroyed at every mpx_finalize (MPX_STREAM_POOL=0) with NO
# delay after the drain: first with a device-wide synchronize before each
# destroy (MPX_STREAM_DESTROY_SYNC=device, a knob removed after this run: it
# stalled too, profiles/r02_stream_destroy_devsync.txt), twice; then the plain form (stream
# drain only), the one that stalled the engine tests inside a later
# mpx_finalize in round 2 (profiles/r02_stream_pool_ab.txt) — last, since it
# may stall; its own limit ends it.
set -o pipefail
export MPX_STREAM_POOL=0 MPX_STREAM_POOL_DELAY_MS=0
MPX_STREAM_DESTROY_SYNC=device PYTEST_BUDGET=300 tools/gpu_pytest.sh devsync1 tests/test_gpu_engine.py &&
MPX_STREAM_DESTROY_SYNC=device PYTEST_BUDGET=300 tools/gpu_pytest.sh devsync2 tests/test_gpu_engine.py &&
{ PYTEST_BUDGET=300 tools/gpu_pytest.sh nosync tests/test_gpu_engine.py; echo "nosync rc=$?"; }
