#!/bin/bash
# Run bench.py (no CPU baseline) once per environment setting given as arguments, e.g.
#   bash scripts/sweep_env.sh "FBA_PRIO=0" "FBA_PRIO=1 FBA_SYRK_CAP=256"
# (BENCH_ARGS: extra bench.py arguments, e.g. "--network convergent")
# Each run under its own time limit; stop at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for envs in "$@"; do
  echo "== $envs"
  env $envs timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS:-} > gpurun_out/sweep.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/sweep.log; echo "stopping (rc=$rc)"; exit $rc; fi
  python -c "import json;d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]);print(round(d['value'],2), {k:round(v,3) for k,v in d['phase_ms'].items()})"
done
