set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02prof4
mkdir -p "$O"
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_prover.py tests/test_gpu_sharded.py tests/test_gpu_multi_circuit.py > "$O/pytest.log" 2>&1 || exit 1
for ln in 19 20 21 22; do
  timeout -k 10 120 python3 bench.py --workload msm --log-n $ln --no-pmc --steps 10 --warmup 2 > "$O/msm_$ln.json" 2> "$O/msm_$ln.err" || exit 1
done
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 8 --warmup 2 > "$O/prove.json" 2> "$O/prove.err"
