#!/bin/bash
# GPU-box: parity tests, then bench.py once per environment setting given as arguments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh tests || exit $?
grep -q " passed" gpurun_out/tests.log && ! grep -q "failed" gpurun_out/tests.log || { echo "tests not green"; exit 1; }
bash scripts/sweep_env.sh "$@"
