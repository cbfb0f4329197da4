# keccak-style k=18 proof (BASELINE configs[4] circuit on one GPU): bench line and kernel trace
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4k
mkdir -p "$O"
timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/bench_keccak.json" 2> "$O/bench_keccak.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o keccak -- \
  python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/bench_keccak_traced.json" 2> "$O/bench_keccak_traced.err"
