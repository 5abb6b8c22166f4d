#!/bin/bash
# GPU-box: multi-rank parity, the traced bench, then the fused-update split swept (FBA_FLOW_KSPLIT)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T="tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 python -m pytest $T > gpurun_out/flow_t1.log 2>&1; rc=$?; tail -1 gpurun_out/flow_t1.log
[ $rc -gt 1 ] && exit $rc
FBA_PANEL_TRACE=2 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-cpu --verbose > gpurun_out/flow_trace.log 2>&1 || exit $?
for K in 4 0 2 3 5 6; do
  FBA_FLOW_KSPLIT=$K timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/ks$K.log 2>&1 || exit $?
  echo "ksplit $K: $(tail -1 gpurun_out/ks$K.log | grep -o '"value": [0-9.]*')"
done
