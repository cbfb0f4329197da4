set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 800 --timeout-method thread -m gpu \
  tests/test_gpu_sharded.py -k spmd > gpurun_out/pytest_sharded9.log 2>&1
