#!/bin/bash
# GPU-box iteration on the Cholesky: parity tests, a traced bench (FBA_PANEL_TRACE), a timed bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/flow_t1.log 2>&1
rc=$?; tail -3 gpurun_out/flow_t1.log
if [ $rc -gt 1 ]; then exit $rc; fi
FBA_PANEL_TRACE=${TRACE:-1} timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --verbose > gpurun_out/flow_trace.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/flow_bench.log 2>&1 || exit $?
tail -1 gpurun_out/flow_bench.log | cut -c1-300
