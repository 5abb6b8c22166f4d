#!/bin/bash
# torchrun rehearsal (every rank on the one GPU of a test box, gloo) of the two multi-GPU solves:
# replicated (observations sharded, the summed reduced system factored on every rank) and subtree split.
#   bash scripts/gpu_gloo_split.sh [config] [ranks: 2 (default) or 4]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cfg=${1:-4}
n=${2:-2}
[ "$n" -le 4 ] || { echo "at most 4 ranks on one GPU here"; exit 2; }
for solve in replicated subtree; do
  FBA_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus "$n" --steps 5 --warmup 1 --config "$cfg" \
    --solve "$solve" > "gpurun_out/gloo${n}_${solve}_c$cfg.log" 2>&1
  rc=$?; echo "== gloo $n-rank $solve config $cfg rc=$rc"
  grep '"metric"' "gpurun_out/gloo${n}_${solve}_c$cfg.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['parallelism'], d['phase_ms'])" || tail -5 "gpurun_out/gloo${n}_${solve}_c$cfg.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
