#!/bin/bash
# PMC passes of the convergent-network scene (bench.py --network convergent): HBM traffic (FETCH_SIZE,
# WRITE_SIZE) and MFMA activity (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE), each its own run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d "$PWD/gpurun_out/convpmc_$i" -o run -- python bench.py --network convergent --steps 2 --warmup 1 --no-cpu > "gpurun_out/convpmc_$i.log" 2>&1
  rc=$?; echo "== conv pmc pass $i ($ctrs) rc=$rc"; [ $rc -ne 0 ] && { tail -5 "gpurun_out/convpmc_$i.log"; exit $rc; }
done
exit 0
