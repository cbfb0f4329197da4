# Round-2 profiles: kernel traces of the C3 k=22 and keccak k=18 benches, and FETCH/WRITE
# PMC passes over the 2^22 MSM child workload (partition + accumulation kernels).
# Run on the GPU box from the repo root:  bash tools/gpu_profile_r02.sh
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r02prof
mkdir -p "$O"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prove" -o prove -- \
  python3 bench.py --no-cpu-baseline --no-pmc --steps 3 --warmup 1 > "$O/prove.json" 2> "$O/prove.err" && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/keccak" -o keccak -- \
  python3 bench.py --workload keccak --no-pmc --steps 3 --warmup 1 > "$O/keccak.json" 2> "$O/keccak.err" && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o pmc -- \
  python3 bench.py --pmc-child --workload msm --log-n 22 > "$O/pmc_fetch.log" 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o pmc -- \
  python3 bench.py --pmc-child --workload msm --log-n 22 > "$O/pmc_write.log" 2>&1 || exit 1
# slab MSM times for the multi-GPU model: one GPU, 2^19..2^22 resident points
for ln in 19 20 21 22; do
  timeout -k 10 120 python3 bench.py --workload msm --log-n $ln --no-pmc --steps 10 --warmup 2 > "$O/msm_$ln.json" 2> "$O/msm_$ln.err" || exit 1
done
