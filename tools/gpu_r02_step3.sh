set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_prover.py > gpurun_out/pytest_r02_step3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r02prof3/pmc_write -o pmc -- \
  python3 bench.py --pmc-child --workload msm --log-n 22 > gpurun_out/pmc_write3.log 2>&1 && \
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc --steps 8 --warmup 2 > gpurun_out/bench_r02h.json 2> gpurun_out/bench_r02h.err && \
bash tools/gpu_r02_step2.sh
