set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 500 --timeout-method thread -m gpu \
  tests/test_gpu_prover.py tests/test_gpu_multi_circuit.py tests/test_gpu_baseline_sizes.py tests/test_gpu_keccak_transcript.py > gpurun_out/pytest_step10.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 8 --warmup 2 > gpurun_out/bench_step10.json 2> gpurun_out/bench_step10.err
