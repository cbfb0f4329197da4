# per-kernel A/B of prover_kernels.hip variants built by tools/ab_lib.py (lib_ab/libh2g_<tag>.so):
#   bash tools/ab_evpf.sh OUT WORKLOAD tag1 tag2 ...   (rocprofv3 kernel traces of a short bench)
out=$1; wl=$2; shift 2
mkdir -p gpurun_out/$out && export TMPDIR=/tmp || exit 1
for t in "$@"; do
  H2G_LIB=yet-another-halo2-fork_amd/lib_ab/libh2g_$t.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/$out/$wl-$t -o run -- python3 bench.py --workload $wl --steps 2 --warmup 1 --no-cpu-baseline --no-krange --no-pmc > gpurun_out/$out/$wl-$t.log 2>&1 || exit 1
done
