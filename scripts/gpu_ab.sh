#!/bin/bash
# A/B of an environment knob on one box: bench.py alternated between VAR=A and VAR=B (usage: VAR=.. A=.. B=..)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu > gpurun_out/ab.log 2>&1 || exit $?
    echo "$VAR=$v $(tail -1 gpurun_out/ab.log | cut -c1-140 | grep -o '"value": [0-9.]*')"
  done
done
