#!/bin/bash
# Ablation timing on one box: for each library variant fish-eye_bundle_adjustment_amd/libfba_<name>.so,
# a rocprofv3 kernel trace of scripts/ablate_time.py, then the average duration per kernel side by side.
#   bash scripts/gpu_ablate.sh <config> <name>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
P=fish-eye_bundle_adjustment_amd
cfg=$1; shift
cp $P/libfba.so $P/libfba_keep.so
restore() { cp $P/libfba_keep.so $P/libfba.so; }
timeout -k 10 300 python bench.py --config "$cfg" --steps 1 --warmup 0 --no-cpu > gpurun_out/abl_gen.log 2>&1 || { echo "scene rc=$?"; exit 3; }
for v in "$@"; do
  cp "$P/libfba_$v.so" $P/libfba.so
  rm -rf "gpurun_out/abl_$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/abl_$v" -o run -- \
    python scripts/ablate_time.py "$cfg" 6 > "gpurun_out/abl_$v.log" 2>&1 || { echo "prof $v rc=$?"; restore; exit 3; }
  tail -1 "gpurun_out/abl_$v.log"
done
restore
python - "$@" <<'PY'
import csv, glob, sys
rows = {}
for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/abl_{v}/**/run_kernel_stats.csv", recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        rows.setdefault(r["Name"].split("(")[0][:40], {})[v] = float(r["AverageNs"]) / 1e3
print("kernel".ljust(40), *[v.rjust(9) for v in sys.argv[1:]])
for k, d in sorted(rows.items(), key=lambda kv: -max(kv[1].values()))[:8]:
    print(k.ljust(40), *[f"{d.get(v, float('nan')):9.1f}" for v in sys.argv[1:]])
PY
