# accumulation chunk length A/B (H2G_MSM_CHUNK; the default at 2^22 is 52 entries):
# MSM parity at 32, the 2^22 MSM and the C3 k=22 proof at 32 / 40 / 52
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4k3
mkdir -p "$O"
H2G_MSM_CHUNK=32 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_chunk32.log" 2>&1 || exit 1
for i in 1 2; do
  for L in 32 40 52; do
    H2G_MSM_CHUNK=$L timeout -k 10 300 python3 bench.py --workload msm --log-n 22 --no-pmc --steps 10 --warmup 2 > "$O/msm22_L${L}_$i.json" 2>&1 || exit 1
    H2G_MSM_CHUNK=$L timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_L${L}_$i.json" 2> "$O/prove_L${L}_$i.err" || exit 1
  done
done
