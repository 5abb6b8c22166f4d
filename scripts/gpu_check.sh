#!/bin/bash
# GPU-box check: each GPU step under its own time limit; stop at the first abort / fault / timeout
# (exit codes other than 0 = ok and 1 = test/assert failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  local name=$1 t=$2; shift 2
  # a heartbeat file while the step runs (a long test -- the config-5 oracle passes -- prints nothing for minutes)
  ( while sleep 50; do date >> gpurun_out/heartbeat.log; done ) &
  local hb=$!
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  kill "$hb" 2>/dev/null; wait "$hb" 2>/dev/null
  echo "== $name rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit "$rc"; fi
}
for step in "$@"; do
  case "$step" in
    tests) run tests 1100 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread -p no:cacheprovider ;;
    quick) run tests_quick 800 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -v --timeout 400 --timeout-method thread -p no:cacheprovider ;;
    reftext) run reftext 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -k reference_text -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py --steps 5 --warmup 1 --verbose ;;
    benchq) run bench 600 python bench.py --steps 5 --warmup 1 --no-cpu --verbose ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python bench.py --steps 3 --warmup 1 --no-cpu ;;
    pmc) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_fetch" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu
          run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_write" -o run -- python bench.py --steps 2 --warmup 1 --no-cpu ;;
    pmc5) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run pmc5_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmc5_fetch" -o run -- python bench.py --config 5 --steps 2 --warmup 1 --no-cpu
          run pmc5_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmc5_write" -o run -- python bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    pmcconv) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run pmcc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmcc_fetch" -o run -- python bench.py --network convergent --steps 2 --warmup 1 --no-cpu
          run pmcc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmcc_write" -o run -- python bench.py --network convergent --steps 2 --warmup 1 --no-cpu ;;
    leaf) run leaf 60 ./scripts/ubench/leaf_lat ;;
    conv) run conv 600 python bench.py --network convergent --steps 5 --warmup 1 --no-cpu --verbose ;;
    convprof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run convprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/convprof" -o run -- python bench.py --network convergent --steps 3 --warmup 1 --no-cpu ;;
    covprof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run covprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/covprof" -o run -- python scripts/cov_time.py 4 ;;
    c3) run bench_c3 400 python bench.py --config 3 --steps 10 --warmup 2 --no-cpu ;;
    c5) run bench_c5 400 python bench.py --config 5 --steps 10 --warmup 2 --no-cpu ;;
  esac
done
