#!/bin/bash
# 2-rank torchrun rehearsal of the multi-GPU path with both ranks on the one GPU of a test box (gloo).
# The persistent dataflow kernels (k_chol_flow, k_bwd_flow) take their records from start-order tickets,
# so two processes' launches can share the GPU (default path; the real runs have one rank per GPU).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
FBA_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 1 > gpurun_out/gloo2.log 2>&1
rc=$?; echo "== gloo 2-rank rc=$rc"; grep '"metric"' gpurun_out/gloo2.log | cut -c1-400
exit $rc
