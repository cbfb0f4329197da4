#!/bin/bash
# per-rank SPMD emulation (tools/spmd_emulate.py) of the BASELINE multi-GPU configs:
#   tools/emu_r4.sh TAG [c3|keccak|both] [c3 ranks] [keccak ranks] [extra spmd_emulate args]
set -o pipefail
R=$PWD; O=$R/gpurun_out/$1; mkdir -p $O
W=${2:-both}; CR=${3:-0,2,6}; KR=${4:-0,4}; shift 4
if [ "$W" != keccak ]; then
  timeout -k 10 500 python3 -u tools/spmd_emulate.py --workload c3 --k 22 --world 8 --ranks $CR --out $O/c3_n8.json "$@" > $O/c3_n8.log 2>&1 || exit 1
fi
if [ "$W" != c3 ]; then
  timeout -k 10 500 python3 -u tools/spmd_emulate.py --workload keccak --k 18 --world 8 --ranks $KR --out $O/k18_n8.json "$@" > $O/k18_n8.log 2>&1 || exit 1
fi
echo ok
