# closing check at FPER = 8: full GPU suite, the default bench line and its kernel trace,
# then the fine-tile A/B around the new default (4 / 8 / 16 entries per thread)
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4final4
mkdir -p "$O"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o prove -- \
  python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_traced.json" 2> "$O/bench_traced.err" || exit 1
AB=yet-another-halo2-fork_amd/lib_ab
for i in 1 2; do
  for v in base fper4 fper16; do
    if [ $v = base ]; then LIBV=""; else LIBV="$PWD/$AB/libh2g_$v.so"; fi
    H2G_LIB=$LIBV timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_${v}_$i.json" 2> "$O/prove_${v}_$i.err" || exit 1
  done
done
