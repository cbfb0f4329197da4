#!/bin/bash
# The one GPU-box driver script (run through gpurun from the repo root).  Every GPU step has
# its own time limit and the steps stop at the first failure.
#   tools/gpu.sh tests TAG [paths / pytest args]  -m gpu suite (default: tests/) -> gpurun_out/TAG/pytest.log
#   tools/gpu.sh bench TAG [bench args...]    bench.py line                    -> gpurun_out/TAG/bench.json
#   tools/gpu.sh prof  TAG [bench args...]    rocprofv3 --kernel-trace --stats of bench.py
#   tools/gpu.sh pmc   TAG [bench args...]    one rocprofv3 --pmc pass per counter (FETCH_SIZE, WRITE_SIZE)
#   tools/gpu.sh pmcbin TAG binary [args]    a standalone binary under the two --pmc passes
#   tools/gpu.sh py    TAG script.py [args]   any python script (A/B runs, microbenchmarks)
set -o pipefail
CMD=$1; TAG=$2; shift 2
R=$PWD
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
case "$CMD" in
  tests)
    [ $# -eq 0 ] && set -- tests
    timeout -k 10 1500 python3 -u -m pytest -m gpu -x -v --timeout 1200 --timeout-method thread --durations=0 \
      -p no:cacheprovider "$@" > "$O/pytest.log" 2>&1
    rc=$?; tail -5 "$O/pytest.log"; exit $rc ;;
  bench)
    timeout -k 10 900 python3 -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
    rc=$?; tail -c 3000 "$O/bench.json"; exit $rc ;;
  prof)
    cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o prof -- \
      python3 "$R/bench.py" --no-cpu-baseline --no-pmc --no-krange "$@" > "$O/bench_traced.json" 2> "$O/bench_traced.err"
    rc=$?; tail -c 1500 "$O/bench_traced.json"; exit $rc ;;
  pmc)
    cd /tmp
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_$C" -o pmc -- \
        python3 "$R/bench.py" --no-cpu-baseline --no-pmc --no-krange "$@" > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; exit 1; }
    done
    echo pmc ok ;;
  pmcbin)  # a standalone binary under one --pmc pass per counter (tools/microbench/pmc_calib)
    B=$1; shift
    cd /tmp
    for C in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_$C" -o pmc -- "$R/$B" "$@" > "$O/pmc_$C.log" 2>&1 || { echo "pmc $C failed"; exit 1; }
    done
    cat "$O/pmc_FETCH_SIZE.log"; echo pmc ok ;;
  py)
    S=$1; shift
    timeout -k 10 900 python3 -u "$S" "$@" > "$O/out.txt" 2> "$O/err.txt"
    rc=$?; tail -c 3000 "$O/out.txt"; tail -c 1500 "$O/err.txt"; exit $rc ;;
  *) echo "usage: tools/gpu.sh tests|bench|prof|pmc|py TAG ..."; exit 2 ;;
esac
