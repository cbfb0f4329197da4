# fine-tile size A/B at 10 fine bits (H2G_MSM_FPER entries per thread: 16 default, 8, 32;
# variant libraries from tools/build_variant.py): 2^22 MSM and C3 k=22 proof, interleaved
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4l
mkdir -p "$O"
AB=yet-another-halo2-fork_amd/lib_ab
for i in 1 2; do
  for v in base fper8 fper32; do
    if [ $v = base ]; then LIBV=""; else LIBV="$PWD/$AB/libh2g_$v.so"; fi
    H2G_LIB=$LIBV timeout -k 10 300 python3 bench.py --workload msm --log-n 22 --no-pmc --steps 10 --warmup 2 > "$O/msm22_${v}_$i.json" 2>&1 || exit 1
    H2G_LIB=$LIBV timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_${v}_$i.json" 2> "$O/prove_${v}_$i.err" || exit 1
  done
done
