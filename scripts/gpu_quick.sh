#!/bin/bash
# GPU-box: parity tests, a quick bench, the k_lin_reduce phase profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh tests benchq || exit $?
FBA_LR_PROFILE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/lrprof.log 2>&1
rc=$?; echo "== lrprof rc=$rc"; grep "k_lin_reduce per chunk" gpurun_out/lrprof.log | tail -2
exit $rc
