# A/B: quad-cooperative bucket reduction for 2^22 MSMs (H2G_MSM_Q4_MAX=65536) vs the
# default threshold (32768 groups): lone 2^22 MSM and the C3 k=22 proof, interleaved.
set -o pipefail
O=$PWD/gpurun_out/abq4
mkdir -p "$O"
run() { tag=$1; q=$2; shift 2; H2G_MSM_Q4_MAX=$q timeout -k 10 200 python3 bench.py "$@" > "$O/$tag.json" 2> "$O/$tag.err"; }
for rep in 1 2; do
  run msm_def_$rep 32768 --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
  run msm_q4_$rep 65536 --workload msm --log-n 22 --no-pmc --steps 20 --warmup 3 || exit 1
  run c3_def_$rep 32768 --no-pmc --no-cpu-baseline --steps 8 --warmup 2 || exit 1
  run c3_q4_$rep 65536 --no-pmc --no-cpu-baseline --steps 8 --warmup 2 || exit 1
done
for f in "$O"/*.json; do echo "$(basename $f) $(python3 -c "import json,sys; a=json.loads(open('$f').read().strip().splitlines()[-1]); print(a['value'], a.get('msm_in_prover',{}).get('phases_ms',{}).get('reduce', a.get('phases_ms',{}).get('reduce')))")"; done
