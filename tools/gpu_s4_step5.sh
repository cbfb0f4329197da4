# counted MSM entries in the bench's modmul rates: the new profiling test, then the
# default bench and the keccak-style bench (no PMC)
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4f
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench.json" 2> "$O/bench.err" || exit 1
timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/bench_keccak.json" 2> "$O/bench_keccak.err" || exit 1
