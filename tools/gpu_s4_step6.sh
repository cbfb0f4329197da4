# lookup permutations on 4 streams: prover parity (lookup / keccak-style circuits, several
# circuits per proof, serde), then an interleaved A/B of the keccak-style k=18 proof
# against H2G_LK_STREAMS=1
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/s4g
mkdir -p "$O"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_prover.py tests/test_gpu_multi_circuit.py tests/test_gpu_baseline_sizes.py tests/test_gpu_serde.py -x -v --timeout 600 --timeout-method thread > "$O/pytest.log" 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/keccak_s4_$i.json" 2> "$O/keccak_s4_$i.err" || exit 1
  H2G_LK_STREAMS=1 timeout -k 10 300 python3 bench.py --workload keccak --k 18 --no-cpu-baseline --no-pmc > "$O/keccak_s1_$i.json" 2> "$O/keccak_s1_$i.err" || exit 1
done
