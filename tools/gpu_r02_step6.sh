set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread -m gpu \
  tests/test_gpu_keccak_transcript.py tests/test_gpu_prover.py tests/test_gpu_multi_circuit.py > gpurun_out/pytest_r02_step6.log 2>&1
