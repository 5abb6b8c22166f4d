#!/bin/bash
# k_chol_flow per-record timelines at config 4 (FBA_PANEL_TRACE=3: every record; =2: the diagonal blocks'
# detail) and k_lin_reduce's phase profile; extra environment settings as arguments (e.g. FBA_FLOW_DYN=0)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
env "$@" FBA_PANEL_TRACE=3 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/flow_trace3.log 2>&1 || exit $?
env "$@" FBA_PANEL_TRACE=2 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/flow_trace2.log 2>&1 || exit $?
env "$@" FBA_LR_PROFILE=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/lrprof.log 2>&1 || exit $?
echo traced
