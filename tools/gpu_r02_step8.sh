set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02prof8
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
  tests/test_gpu_sharded.py > "$O/pytest_sharded.log" 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --k 18 --no-pmc --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench_spmd_gloo2.json" 2> "$O/bench_spmd_gloo2.err" || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --k 18 --no-subcosets --no-pmc --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench_spmd_nosub_gloo2.json" 2> "$O/bench_spmd_nosub_gloo2.err" || exit 1
timeout -k 10 300 python3 bench.py --gpus 4 --dist-backend gloo --workload keccak --k 16 --no-pmc --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench_keccak_spmd_gloo4.json" 2> "$O/bench_keccak_spmd_gloo4.err"
