#!/bin/bash
# bench several libmxa builds back to back (parity via smoke hashes first, except *nohash*)
set -o pipefail
mkdir -p gpurun_out
for w in "$@"; do
  echo "== $w"
  case $w in
    *nohash*) ;;
    *) MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$w.so timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
  esac
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$w.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu || exit 1
done
