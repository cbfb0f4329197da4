# MSM kernel traces at slab sizes and a window-size A/B at 2^22
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02prof2
mkdir -p "$O"
for ln in 19 22; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/msm$ln" -o msm -- \
    python3 bench.py --workload msm --log-n $ln --no-pmc --steps 10 --warmup 2 > "$O/msm_$ln.json" 2> "$O/msm_$ln.err" || exit 1
done
for c in 20 22 21; do
  timeout -k 10 200 python3 bench.py --workload msm --log-n 22 --window-bits $c --no-pmc --steps 20 --warmup 3 > "$O/msm22_c$c.json" 2> "$O/msm22_c$c.err" || exit 1
done
