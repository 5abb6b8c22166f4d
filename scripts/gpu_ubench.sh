#!/bin/bash
# GPU-box: run the calibration micro-benchmarks (prebuilt in scripts/ubench/)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/ubench/chol_ubench > gpurun_out/chol_ubench.log 2>&1
rc=$?; echo "== chol_ubench rc=$rc"; cat gpurun_out/chol_ubench.log
exit $rc
