#!/bin/bash
# HEAD counter record of one workload: a kernel trace and three PMC passes (FETCH_SIZE; WRITE_SIZE;
# SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CYCLES + GRBM_GUI_ACTIVE), each its own rocprofv3 run of bench.py
# under its own time limit, then scripts/pmc_summary.py -> gpurun_out/pmc_<tag>.json (stamped with the
# build id; copy it to profiles/ to let bench.py use it).
#   bash scripts/gpu_pmc.sh <config> [grid|convergent]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cfg=$1; net=${2:-grid}
tag="c${cfg}$([ "$net" = grid ] || echo "_$net")"
root=$PWD
cd /tmp && export TMPDIR=/tmp && cd "$root"
args="--config $cfg --network $net --steps 2 --warmup 1 --no-cpu"
# the scene is generated once, outside the profiled runs
timeout -k 10 300 python bench.py $args > "gpurun_out/pmc_${tag}_gen.log" 2>&1 || { echo "scene/bench failed"; tail -5 "gpurun_out/pmc_${tag}_gen.log"; exit 1; }
pass() {
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d "$root/gpurun_out/pmc_${tag}_$name" -o run -- python bench.py $args > "gpurun_out/pmc_${tag}_$name.log" 2>&1
  local rc=$?
  echo "== $tag $name rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "gpurun_out/pmc_${tag}_$name.log"; exit $rc; }
  return 0
}
pass trace --kernel-trace --stats
pass fetch --pmc FETCH_SIZE
pass write --pmc WRITE_SIZE
pass mfma --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
python scripts/pmc_summary.py --fetch "gpurun_out/pmc_${tag}_fetch" --write "gpurun_out/pmc_${tag}_write" \
  --mfma "gpurun_out/pmc_${tag}_mfma" --trace "gpurun_out/pmc_${tag}_trace" --config "$cfg" --network "$net" \
  --out "gpurun_out/pmc_${tag}.json"
