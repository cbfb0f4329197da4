#!/bin/bash
# per-rank emulation of every rank at N = 2, 4, 8 for C3 k=22 and keccak-style k=18
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
for w in 2 4 8; do
  timeout -k 10 280 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world $w --out $O/c3_n$w.json > $O/c3_n$w.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world $w --out $O/k18_n$w.json > $O/k18_n$w.log 2>&1 || exit 1
done
echo ok
