set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_prover.py tests/test_gpu_multi_circuit.py > gpurun_out/pytest_r02_step1.log 2>&1 && \
bash tools/gpu_profile_r02.sh
