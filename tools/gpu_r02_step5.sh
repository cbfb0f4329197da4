set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02prof5
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_gpu_sharded.py > "$O/pytest_sharded.log" 2>&1 || exit 1
# SPMD bench rehearsal: 2 gloo ranks sharing the one GPU (torch all_gather transport)
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --k 18 --no-pmc --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench_spmd_gloo2.json" 2> "$O/bench_spmd_gloo2.err" || exit 1
timeout -k 10 300 python3 bench.py --gpus 2 --dist-backend gloo --mode shard --transport torch --k 18 --no-pmc --no-cpu-baseline --steps 3 --warmup 1 > "$O/bench_shard_gloo2.json" 2> "$O/bench_shard_gloo2.err" || exit 1
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 8 --warmup 2 > "$O/prove.json" 2> "$O/prove.err"
