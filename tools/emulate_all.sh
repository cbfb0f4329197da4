#!/bin/bash
# Emulated multi-GPU scaling on one GPU (tools/spmd_emulate.py, tools/msm_scale_emulate.py):
# every rank of C3 k = 22 at N = 2 / 4 / 8 and of the keccak-style k = 18 proof at N = 8,
# compute only and with the xGMI communication model, and the 2^24 MSM's point slabs.
#   tools/emulate_all.sh TAG   -> gpurun_out/TAG/*.json
set -o pipefail
O=gpurun_out/$1
mkdir -p "$O"
export TMPDIR=/tmp
run() {  # name, args...
  local nm=$1; shift
  timeout -k 10 300 python3 -u "$@" > "$O/$nm.log" 2>&1 || { echo "$nm failed"; tail -5 "$O/$nm.log"; exit 1; }
  grep -E "^(EMULATE|MSMSCALE)" "$O/$nm.log" | cut -d' ' -f2- > "$O/$nm.json"
  echo "$nm ok"
}
run msm_scale tools/msm_scale_emulate.py --log-n 24 --worlds 2,4,8 --comm-model 50,40
for N in 2 4 8; do
  run c3_n$N tools/spmd_emulate.py --k 22 --world $N
  run c3_n${N}_comm tools/spmd_emulate.py --k 22 --world $N --comm-model 50,40
done
run k18_n8 tools/spmd_emulate.py --k 18 --workload keccak --world 8
run k18_n8_comm tools/spmd_emulate.py --k 18 --workload keccak --world 8 --comm-model 50,40
