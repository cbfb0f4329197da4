#!/bin/bash
# interleaved A/B of NTT builds: the current lib and lib_ab/libh2g_<tag>.so for each tag,
# tools/ntt_bench.py at the given sizes, `reps` rounds
#   bash tools/ab_ntt.sh "tw1 tw2" 3 20 22
set -o pipefail
tags=$1; reps=$2; shift 2
for r in $(seq $reps); do
  echo "== round $r base"; timeout -k 10 120 python3 tools/ntt_bench.py "$@" || exit 1
  for t in $tags; do
    echo "== round $r $t"; H2G_LIB=yet-another-halo2-fork_amd/lib_ab/libh2g_$t.so timeout -k 10 120 python3 tools/ntt_bench.py "$@" || exit 1
  done
done
