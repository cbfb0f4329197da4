# fine-pass fan-out A/B (H2G_MSM_FB = fine bits per coarse bin; 11 is the default): MSM
# parity at FB=9, the 2^22 MSM at FB 8..11 twice interleaved, the C3 k=22 proof at 9/10/11
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4h
mkdir -p "$O"
H2G_MSM_FB=9 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > "$O/pytest_fb9.log" 2>&1 || exit 1
for i in 1 2; do
  for fb in 8 9 10 11; do
    H2G_MSM_FB=$fb timeout -k 10 300 python3 bench.py --workload msm --log-n 22 --no-pmc --steps 10 --warmup 2 > "$O/msm22_fb${fb}_$i.json" 2>&1 || exit 1
  done
done
for fb in 9 10 11; do
  H2G_MSM_FB=$fb timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_fb${fb}.json" 2> "$O/prove_fb${fb}.err" || exit 1
done
