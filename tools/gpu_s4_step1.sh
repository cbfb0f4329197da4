# serde Processed + MSM parity on the device, then an interleaved A/B of the bucket
# reduction (block suffix scans, default, vs H2G_MSM_RED=group) on the default bench
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4a
mkdir -p "$O"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_serde.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_scan_$i.json" 2> "$O/bench_scan_$i.err" || exit 1
  H2G_MSM_RED=group timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_group_$i.json" 2> "$O/bench_group_$i.err" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o prove -- \
  python3 bench.py --no-cpu-baseline --no-pmc > "$O/bench_traced.json" 2> "$O/bench_traced.err"
