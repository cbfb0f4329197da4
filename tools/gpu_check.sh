#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprof kernel stats.
# usage: tools/gpu_check.sh TAG [bench args...]
TAG=${1:-run}; shift
R=$PWD
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -x > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log
grep -q "passed" gpurun_out/pytest_gpu_$TAG.log && ! grep -q "failed\|error" gpurun_out/pytest_gpu_$TAG.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { echo smoke failed; tail gpurun_out/smoke_$TAG.log; exit 1; }
timeout -k 10 600 python bench.py "$@" > gpurun_out/bench_$TAG.log 2>&1 || { echo bench failed; tail gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o prof -- python $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/bench_prof_$TAG.log 2>&1
echo "prof exit $?"
