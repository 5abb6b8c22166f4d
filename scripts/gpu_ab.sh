#!/bin/bash
# A/B on one box: library variants fish-eye_bundle_adjustment_amd/libfba_<name>.so (built from other
# commits or working trees; "new" = the working tree's libfba.so), alternating, bench.py at config 4,
# then each variant's k_lin_reduce phase profile.
#   bash scripts/gpu_ab.sh <rounds> <name>... [-- extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
P=fish-eye_bundle_adjustment_amd
rounds=$1; shift
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ $# -gt 0 ] && shift
cp $P/libfba.so $P/libfba_new.so
restore() { cp $P/libfba_new.so $P/libfba.so; }
for r in $(seq 1 "$rounds"); do
  for v in "${names[@]}"; do
    cp "$P/libfba_$v.so" $P/libfba.so
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu "$@" > "gpurun_out/ab_${v}_$r.log" 2>&1 || { echo "bench $v rc=$?"; tail -5 "gpurun_out/ab_${v}_$r.log"; restore; exit 3; }
    echo "$v $r $(python -c "import json; d=json.loads([l for l in open('gpurun_out/ab_${v}_$r.log') if l.startswith('{')][-1]); print(round(d['value'],1), round(d['roofline']['avg_launch_us'],1))")"
  done
done
for v in "${names[@]}"; do
  cp "$P/libfba_$v.so" $P/libfba.so
  FBA_LR_PROFILE=1 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu "$@" > "gpurun_out/ab_lrprof_$v.log" 2>&1 || { restore; exit 3; }
  echo "$v $(grep 'k_lin_reduce per chunk' "gpurun_out/ab_lrprof_$v.log" | tail -1)"
done
restore
