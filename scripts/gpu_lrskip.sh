#!/bin/bash
# GPU-box: k_lin_reduce phase profile with image / pair items left out (FBA_LR_SKIP=1 / 2 / 3)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for m in ${LRSKIP_MODES:-0 1 2 3}; do
  FBA_LR_PROFILE=1 FBA_LR_SKIP=$m timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu > gpurun_out/lrskip$m.log 2>&1
  rc=$?; echo "== skip $m rc=$rc"; grep "k_lin_reduce per chunk" gpurun_out/lrskip$m.log | tail -1
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
exit 0
