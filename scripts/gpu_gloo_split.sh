#!/bin/bash
# 2-rank torchrun rehearsal (both ranks on the one GPU of a test box, gloo) of the two multi-GPU solves:
# replicated (observations sharded, the summed reduced system factored on every rank) and subtree split.
#   bash scripts/gpu_gloo_split.sh [config]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cfg=${1:-4}
for solve in replicated subtree; do
  FBA_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 1 --config "$cfg" \
    --solve "$solve" > "gpurun_out/gloo2_${solve}_c$cfg.log" 2>&1
  rc=$?; echo "== gloo 2-rank $solve config $cfg rc=$rc"
  grep '"metric"' "gpurun_out/gloo2_${solve}_c$cfg.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['parallelism'], d['phase_ms'])" || tail -5 "gpurun_out/gloo2_${solve}_c$cfg.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
