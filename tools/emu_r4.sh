#!/bin/bash
# per-rank SPMD emulation (tools/spmd_emulate.py) of the BASELINE multi-GPU configs:
#   tools/emu_r4.sh TAG [c3|keccak|both] [extra spmd_emulate args]
set -o pipefail
R=$PWD; O=$R/gpurun_out/$1; mkdir -p $O
W=${2:-both}; shift 2
if [ "$W" != keccak ]; then
  timeout -k 10 400 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --ranks 0,2 --owner-weight 0.1 --out $O/c3_n8.json "$@" > $O/c3_n8.log 2>&1 || exit 1
fi
if [ "$W" != c3 ]; then
  timeout -k 10 400 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks 0,4 --owner-weight 0.5 --out $O/k18_n8.json "$@" > $O/k18_n8.log 2>&1 || exit 1
fi
echo ok
