#!/bin/bash
# kernel traces of tools/ab_env.py's child (lone fixed-base MSMs and/or C3 proofs) for the
# current library and an A/B library:  tools/prof_msm.sh TAG MSM_LOG_NS PROVE_KS [AB_LIB]
set -o pipefail
R=$PWD; O=$R/gpurun_out/$1; mkdir -p $O; export TMPDIR=/tmp
AB=${4:?an A/B library (tools/build_variant.py output copied under yet-another-halo2-fork_amd/lib/)}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o p -- python3 $R/tools/ab_env.py --child --msm "$2" --prove "$3" > $O/new.log 2>&1 || exit 1
H2G_LIB=$AB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o p -- python3 $R/tools/ab_env.py --child --msm "$2" --prove "$3" > $O/old.log 2>&1 || exit 1
echo done
