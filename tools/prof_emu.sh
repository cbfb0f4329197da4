#!/bin/bash
# kernel trace of one emulated SPMD rank (tools/spmd_emulate.py): tools/prof_emu.sh TAG WORKLOAD K WORLD RANK [args]
set -o pipefail
R=$PWD; O=$R/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
WL=$2; K=$3; WD=$4; RK=$5; shift 5
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o p -- python3 $R/tools/spmd_emulate.py --workload $WL --k $K --world $WD --ranks $RK --steps 3 --warmup 1 "$@" > $O/emu.log 2>&1 || exit 1
echo done
