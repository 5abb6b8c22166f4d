#!/bin/bash
# PMC counters for selected kernels (separate passes), bench.py --steps 1:
#   bash scripts/pmc_kernels.sh '<kernel regex>' "CTR1 CTR2 ..." ["CTR3 ..."]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
re=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex "$re" --output-format csv -d "$PWD/gpurun_out/pmck_$i" -o run -- python bench.py --steps 1 --warmup 1 --no-cpu > "gpurun_out/pmck_$i.log" 2>&1
  rc=$?; echo "== pass $i ($ctrs) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "gpurun_out/pmck_$i.log"; exit $rc; }
done
exit 0
