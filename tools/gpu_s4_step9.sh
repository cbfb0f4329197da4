# after the fine-bits default change: q4 threshold A/B with the plane reduction
# (H2G_MSM_Q4_MAX: sets of at most this many groups use quad-cooperative 64-group planes)
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4j
mkdir -p "$O"
for L in 20 21 22; do
  for q in 16384 32768 65536; do
    H2G_MSM_Q4_MAX=$q timeout -k 10 300 python3 bench.py --workload msm --log-n $L --no-pmc --steps 10 --warmup 2 > "$O/msm${L}_q$q.json" 2>&1 || exit 1
  done
done
for i in 1 2; do
  for q in 32768 65536; do
    H2G_MSM_Q4_MAX=$q timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_q${q}_$i.json" 2> "$O/prove_q${q}_$i.err" || exit 1
  done
done
