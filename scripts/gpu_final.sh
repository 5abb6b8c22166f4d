#!/bin/bash
# GPU-box round record: parity tests, smoke, bench with the CPU baseline, kernel trace, PMC traffic,
# configs 3 and 5, and a 2-rank torchrun rehearsal of the multi-GPU path (gloo, both ranks on the one GPU)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/gpu_check.sh tests smoke bench prof pmc || exit $?
for cfg in 3 5; do
  timeout -k 10 400 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu > gpurun_out/bench_c$cfg.log 2>&1
  rc=$?; echo "== config $cfg rc=$rc"; tail -1 gpurun_out/bench_c$cfg.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
bash scripts/gpu_gloo2.sh  # both ranks on the one GPU: the flow kernels take their records from start-order tickets
