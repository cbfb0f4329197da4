#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only), per the MI355X guide:
# FETCH_SIZE and WRITE_SIZE cannot share a pass.  usage: tools/pmc_pass.sh TAG [bench args]
TAG=${1:-run}; shift
R=$PWD
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/pmc_${TAG}_$C -o pmc -- python $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
echo pmc ok
