set -o pipefail
O=gpurun_out/r5m; mkdir -p $O
for spec in "c3_n4_comm_noown --k 22 --world 4 --comm-model 50,40 --no-column-owners" "c3_n4_comm --k 22 --world 4 --comm-model 50,40 --ranks 2,3" "c3_n8_comm --k 22 --world 8 --comm-model 50,40 --ranks 6,7" "c3_n8_comm_noown --k 22 --world 8 --comm-model 50,40 --no-column-owners" "k18_n8_comm --k 18 --workload keccak --world 8 --comm-model 50,40 --ranks 3"; do
  set -- $spec; nm=$1; shift
  timeout -k 10 300 python3 -u tools/spmd_emulate.py "$@" > $O/$nm.log 2>&1 || { echo "$nm failed"; tail -3 $O/$nm.log; exit 1; }
  grep "^EMULATE" $O/$nm.log | cut -d' ' -f2- > $O/$nm.json; echo "$nm ok"
done
