#!/bin/bash
# As sweep_env.sh with 40 timed steps per setting (less noise): bash scripts/sweep_env40.sh "A=1" "A=2"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for envs in "$@"; do
  echo "== $envs"
  env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 3 --no-cpu > gpurun_out/sweep.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/sweep.log; echo "stopping (rc=$rc)"; exit $rc; fi
  python -c "import json;d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]);print(round(d['value'],2), round(d['phase_ms']['cholesky'],3))"
done
