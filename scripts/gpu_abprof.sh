#!/bin/bash
# Kernel-level A/B on one box: for each library variant fish-eye_bundle_adjustment_amd/libfba_<name>.so
# ("new" = the working tree's libfba.so), one rocprofv3 kernel trace of bench.py, then the average
# duration per kernel of every variant side by side.
#   bash scripts/gpu_abprof.sh <name>... [-- extra bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
export TMPDIR=/tmp
P=fish-eye_bundle_adjustment_amd
names=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do names+=("$1"); shift; done
[ $# -gt 0 ] && shift
cp $P/libfba.so $P/libfba_new.so
restore() { cp $P/libfba_new.so $P/libfba.so; }
for v in "${names[@]}"; do
  cp "$P/libfba_$v.so" $P/libfba.so
  rm -rf "gpurun_out/abprof_$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/abprof_$v" -o run -- \
    python bench.py --steps 5 --warmup 1 --no-cpu "$@" > "gpurun_out/abprof_$v.log" 2>&1 || { echo "prof $v rc=$?"; restore; exit 3; }
done
restore
python - "${names[@]}" <<'PY'
import csv, glob, sys
rows = {}
for v in sys.argv[1:]:
    f = glob.glob(f"gpurun_out/abprof_{v}/**/run_kernel_stats.csv", recursive=True)
    if not f:
        continue
    for r in csv.DictReader(open(f[0])):
        rows.setdefault(r["Name"].split("(")[0][:48], {})[v] = float(r["AverageNs"]) / 1e3
print("kernel".ljust(48), *[v.rjust(10) for v in sys.argv[1:]])
for k, d in sorted(rows.items(), key=lambda kv: -max(kv[1].values())):
    print(k.ljust(48), *[f"{d.get(v, float('nan')):10.1f}" for v in sys.argv[1:]])
PY
