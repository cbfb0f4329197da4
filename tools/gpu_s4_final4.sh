# closing check at FPER = 8: full GPU suite, the default bench line and its kernel trace
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4final4
mkdir -p "$O"
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 || exit 1
timeout -k 10 600 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o prove -- \
  python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_traced.json" 2> "$O/bench_traced.err" || exit 1
