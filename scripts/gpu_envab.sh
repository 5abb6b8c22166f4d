#!/bin/bash
# A/B of environment settings on one box and one library: bench.py at config 4 under each setting, alternating.
#   bash scripts/gpu_envab.sh <rounds> "<settings A>" "<settings B>" ... [-- extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
rounds=$1; shift
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
[ $# -gt 0 ] && shift
for r in $(seq 1 "$rounds"); do
  k=0
  for e in "${sets[@]}"; do
    k=$((k + 1))
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu "$@" > "gpurun_out/envab_${k}_$r.log" 2>&1 || { echo "bench [$e] rc=$?"; tail -5 "gpurun_out/envab_${k}_$r.log"; exit 3; }
    echo "[$e] $r $(python -c "import json; d=json.loads([l for l in open('gpurun_out/envab_${k}_$r.log') if l.startswith('{')][-1]); print(round(d['value'],1), round(d['roofline']['avg_launch_us'],1))")"
  done
done
