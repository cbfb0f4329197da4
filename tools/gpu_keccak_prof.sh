set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/keccak
mkdir -p "$O"
timeout -k 10 300 python3 bench.py --workload keccak --no-pmc --steps 5 --warmup 2 > "$O/bench_keccak.json" 2> "$O/bench_keccak.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o kk -- \
  python3 tools/prove_bench.py keccak 18 > "$O/prove_bench.log" 2>&1
