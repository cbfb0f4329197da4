set -o pipefail
O=gpurun_out/r5ab; mkdir -p $O
for v in def early; do
  for N in 4 8; do
    if [ $v = early ]; then export H2G_ADV_XFORM_EARLY=1; else unset H2G_ADV_XFORM_EARLY; fi
    timeout -k 10 300 python3 -u tools/spmd_emulate.py --k 22 --world $N --replay "1e9,0;50,40" > $O/${v}_n$N.log 2>&1 || exit 1
    grep "^EMULATE" $O/${v}_n$N.log | cut -d' ' -f2- > $O/${v}_n$N.json
  done
done
unset H2G_ADV_XFORM_EARLY
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_sharded.py -k "row_pieces or diverged_witness or c3_k22_at_size" > $O/tests.log 2>&1
