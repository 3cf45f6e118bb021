#!/bin/bash
# A/B of libmxa variant builds (lib/libmxa_<name>.so) on one GPU box, interleaved:
# tools/ab_run.sh OUT "name1 name2 ..." ROUNDS CMD...   (CMD runs with MXA_LIB set per variant)
set -o pipefail
OUT=$1; NAMES=$2; ROUNDS=$3; shift 3
mkdir -p $(dirname $OUT)
for r in $(seq 1 $ROUNDS); do
  for n in $NAMES; do
    MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$n.so timeout -k 10 300 "$@" >> $OUT 2>&1 || { echo "variant $n failed"; tail -5 $OUT; exit 1; }
  done
done
cat $OUT
