# C3 k=22 proof, fine bits 10 vs 11 (default), three interleaved pairs
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4i
mkdir -p "$O"
for i in 1 2 3; do
  for fb in 10 11; do
    H2G_MSM_FB=$fb timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-pmc > "$O/prove_fb${fb}_$i.json" 2> "$O/prove_fb${fb}_$i.err" || exit 1
  done
done
