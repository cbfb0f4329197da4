#!/bin/bash
# prover parity tests (single GPU, SPMD small), keccak / C3 N=8 emulation, bench
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_prover.py tests/test_gpu_multi_circuit.py tests/test_gpu_sharded.py -k "not at_size and not k18 and not rccl" > $O/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks 0,4 --out $O/k18_n8.json > $O/k18.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --ranks 0,3,6 --out $O/c3_n8.json > $O/c3.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py > $O/bench.log 2>&1 || exit 1
echo ok
[ -n "$2" ] && { cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/tr -o run -- python3 -u $GRAFT_REPO_ROOT/tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks 0 --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$O/tr.log 2>&1 || exit 1; }
echo ok2
