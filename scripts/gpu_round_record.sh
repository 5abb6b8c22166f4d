#!/bin/bash
# GPU-box round record at HEAD: parity tests + smoke, the driver's default bench (config 4 with the CPU
# baseline), then configs 3 and 5 and the convergent scene without it, then the 2-rank torchrun/gloo
# rehearsal of both multi-GPU solves at config 4 (both ranks on the one GPU); each step under its own limit.
#   bash scripts/gpu_round_record.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh tests smoke || exit $?
timeout -k 10 500 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench rc=$?"; tail -5 gpurun_out/bench_default.log; exit 3; }
echo "== bench default"; tail -1 gpurun_out/bench_default.log | cut -c1-400
for args in "--config 3" "--config 5" "--network convergent"; do
  tag=$(echo "$args" | tr -d ' -')
  timeout -k 10 400 python bench.py $args --steps 10 --warmup 2 --no-cpu > "gpurun_out/bench_$tag.log" 2>&1 || { echo "bench $args rc=$?"; exit 3; }
  echo "== bench $args"; tail -1 "gpurun_out/bench_$tag.log" | cut -c1-300
done
bash scripts/gpu_gloo_split.sh 4
