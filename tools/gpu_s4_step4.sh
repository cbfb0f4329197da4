# SHPLONK's lone commitments as two concurrent half MSMs: prover parity, then an
# interleaved A/B of the C3 k=22 proof against H2G_COMMIT_SPLIT_MIN=0 (no split)
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4e
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_prover.py tests/test_gpu_baseline_sizes.py tests/test_gpu_serde.py -x -v --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_split_$i.json" 2> "$O/bench_split_$i.err" || exit 1
  H2G_COMMIT_SPLIT_MIN=0 timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_nosplit_$i.json" 2> "$O/bench_nosplit_$i.err" || exit 1
done
