set -o pipefail
O=$PWD/gpurun_out/abpart
mkdir -p "$O"
L=$PWD/yet-another-halo2-fork_amd/lib_ab
run() { tag=$1; lib=$2; shift 2; H2G_LIB=$lib timeout -k 10 200 python3 bench.py "$@" > "$O/$tag.json" 2> "$O/$tag.err"; }
for rep in 1 2; do
  run def_$rep "" --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
  run fper32_$rep $L/libh2g_fper32.so --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
  run pt1024_$rep $L/libh2g_pt1024.so --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
  run both_$rep $L/libh2g_both.so --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
done
