#!/bin/bash
# GPU-box round check: parity tests, smoke, bench (with the CPU baseline), a rocprofv3 kernel trace
# and the two PMC passes (FETCH_SIZE, WRITE_SIZE) behind bench.py's roofline.traffic
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh tests smoke bench prof pmc
