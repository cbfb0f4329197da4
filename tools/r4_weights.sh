#!/bin/bash
# C3 k=22 per-rank emulation with leader-favouring slab weights (row-pieces mode)
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 280 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 4 --weights 21,21,19,19 --out $O/c3_n4_w21.json > $O/a.log 2>&1 || exit 1
timeout -k 10 280 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 4 --weights 11,11,9,9 --out $O/c3_n4_w11.json > $O/b.log 2>&1 || exit 1
timeout -k 10 280 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --weights 7,7,6,6,6,6,6,6 --out $O/c3_n8_w7.json > $O/c.log 2>&1 || exit 1
timeout -k 10 280 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --weights 13,13,12,12,12,12,12,12 --out $O/c3_n8_w13.json > $O/d.log 2>&1 || exit 1
echo ok
