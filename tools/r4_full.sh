#!/bin/bash
# full GPU suite, then the keccak N=8 rank trace and the bench
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks 0,4 --out $O/k18_n8.json > $O/k18.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --ranks 0,3,6 --out $O/c3_n8.json > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || exit 1
echo ok
