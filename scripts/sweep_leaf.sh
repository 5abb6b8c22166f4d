cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --steps 1 --warmup 0 --no-cpu > /dev/null 2>&1
for L in 100 60 80 120 150; do
  FBA_ND_LEAF=$L timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu --verbose > gpurun_out/leaf$L.log 2>&1 || exit $?
  echo "leaf $L: $(grep -o 'camera system: [^,]*, [^,]*, [^,]*' gpurun_out/leaf$L.log) $(tail -1 gpurun_out/leaf$L.log | grep -o '"value": [0-9.]*')"
done
