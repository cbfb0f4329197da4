# MSM parity with bit planes for every set size up to 2^17 groups, then interleaved A/B
# against H2G_MSM_RED=group: slab-size MSMs, the C3 k=22 proof, the keccak-style k=18 proof
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4d
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
for L in 19 20 21 22; do
  timeout -k 10 300 python3 bench.py --workload msm --log-n $L --no-pmc --steps 10 --warmup 2 > "$O/msm_plane_$L.json" 2>&1 || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --workload msm --log-n $L --no-pmc --steps 10 --warmup 2 > "$O/msm_group_$L.json" 2>&1 || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_plane_$i.json" 2> "$O/bench_plane_$i.err" || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_group_$i.json" 2> "$O/bench_group_$i.err" || exit 1
  timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/keccak_plane_$i.json" 2> "$O/keccak_plane_$i.err" || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/keccak_group_$i.json" 2> "$O/keccak_group_$i.err" || exit 1
done
