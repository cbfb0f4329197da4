#!/bin/bash
# round-4 check step: SPMD tests (small), per-rank emulation of C3 k=22 / keccak k=18 at
# N=8 for the current library and an optional A/B library, partition PMC at 2^22.
#   tools/r4_step.sh TAG [AB_LIB_NAME]
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
L=$PWD/yet-another-halo2-fork_amd/lib
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -k "spmd and not at_size and not k18" > $O/tests.log 2>&1 || exit 1
for v in default $2; do
  E=""; [ "$v" != default ] && E="H2G_LIB=$L/$v"
  env $E timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --ranks 0,3,6 --out $O/c3_n8_$v.json > $O/c3_$v.log 2>&1 || exit 1
  env $E timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks 0,4 --out $O/k18_n8_$v.json > $O/k18_$v.log 2>&1 || exit 1
done
[ -n "$3" ] && { python3 tools/pmc_partition.py --log-n 22 --out $O/pmc_partition_2p22.json > $O/pmc.log 2>&1 || exit 1; }
echo ok
