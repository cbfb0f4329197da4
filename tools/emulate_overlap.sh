#!/bin/bash
# the SPMD emulation with the column exchanges overlapped (default) and completing on return
# (--sync-exchange), under the xGMI communication model; JSON per run under gpurun_out/r5o
set -o pipefail
O=gpurun_out/r5o; mkdir -p $O
for spec in "c3_n4_async --k 22 --world 4 --comm-model 50,40 --ranks 2,3" \
            "c3_n4_sync --k 22 --world 4 --comm-model 50,40 --ranks 2,3 --sync-exchange" \
            "c3_n8_async --k 22 --world 8 --comm-model 50,40 --ranks 6,7" \
            "c3_n4_async_compute --k 22 --world 4 --ranks 2,3" \
            "k18_n8_async --k 18 --workload keccak --world 8 --comm-model 50,40 --ranks 3"; do
  set -- $spec; nm=$1; shift
  timeout -k 10 300 python3 -u tools/spmd_emulate.py "$@" > $O/$nm.log 2>&1 || { echo "$nm failed"; tail -5 $O/$nm.log; exit 1; }
  grep "^EMULATE" $O/$nm.log | cut -d' ' -f2- > $O/$nm.json; echo "$nm ok"
done
