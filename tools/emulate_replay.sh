#!/bin/bash
# every rank's collective timeline recorded (compute only) and the ranks replayed against
# each other (tools/spmd_emulate.py --replay): no wire time, and the xGMI model
set -o pipefail
O=gpurun_out/$1; mkdir -p "$O"
run() {
  local nm=$1; shift
  timeout -k 10 300 python3 -u tools/spmd_emulate.py "$@" --replay "1e9,0;50,40" > "$O/$nm.log" 2>&1 || { echo "$nm failed"; tail -5 "$O/$nm.log"; exit 1; }
  grep "^EMULATE" "$O/$nm.log" | cut -d' ' -f2- > "$O/$nm.json"; echo "$nm ok"
}
for N in 2 4 8; do run c3_n$N --k 22 --world $N; done
run k18_n8 --k 18 --workload keccak --world 8
