set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 250 --timeout-method thread -m gpu \
  tests/test_gpu_pairing_verify.py > gpurun_out/pytest_r02_step7.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 5 --warmup 1 > gpurun_out/bench_r02_step7.json 2> gpurun_out/bench_r02_step7.err
