#!/bin/bash
# rocprofv3 kernel trace of a short bench run under the given environment settings:
#   bash scripts/prof_env.sh <tag> [VAR=value ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1; shift
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for kv in "$@"; do export "$kv"; done
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_$tag" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu > "gpurun_out/prof_$tag.log" 2>&1
rc=$?
echo "== prof $tag rc=$rc"; tail -3 "gpurun_out/prof_$tag.log" | cut -c1-200
exit $rc
