# MSM parity with the bit-plane bucket reduction, then an interleaved A/B of the proof
# bench against the previous rscale scheme (H2G_MSM_RED=group)
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4c
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_plane_$i.json" 2> "$O/bench_plane_$i.err" || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_group_$i.json" 2> "$O/bench_group_$i.err" || exit 1
done
for L in 19 21; do
  timeout -k 10 300 python3 bench.py --workload msm --log-n $L --no-pmc --steps 10 --warmup 2 > "$O/msm_plane_$L.json" 2>&1 || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --workload msm --log-n $L --no-pmc --steps 10 --warmup 2 > "$O/msm_group_$L.json" 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o prove -- \
  python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_traced.json" 2> "$O/bench_traced.err"
