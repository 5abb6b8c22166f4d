#!/bin/bash
# Round 3: kernel trace of fba_covariance at config 4 and the convergent config-4 scene's kernel trace +
# PMC passes (HBM bytes, MFMA busy cycles) -- each GPU step under its own limit, stop at the first failure
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="python bench.py --config 4 --network convergent --steps 2 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/cov_prof" -o run -- python scripts/cov_time.py 4 > gpurun_out/cov_prof.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/conv_prof" -o run -- $B > gpurun_out/conv_prof.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/conv_fetch" -o run -- $B > gpurun_out/conv_fetch.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/conv_write" -o run -- $B > gpurun_out/conv_write.log 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$PWD/gpurun_out/conv_mfma" -o run -- $B > gpurun_out/conv_mfma.log 2>&1 || exit $?
echo done
# k_chol_flow per-record timeline at config 4 (FBA_PANEL_TRACE=2: eager launches, one step traced)
FBA_PANEL_TRACE=2 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu > gpurun_out/flow_trace_c4.log 2>&1 || exit $?
echo traced
