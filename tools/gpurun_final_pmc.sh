#!/bin/bash
# final PMC records and kernel stats of a list of configurations (no test suite).
# usage: tools/gpurun_final_pmc.sh TAG PART CONFIG:ENVS[:TAPE] ...
set -o pipefail
T=${1:?tag}; P=${2:?part}; shift 2
O=gpurun_out/final_$T; mkdir -p $O
timeout -k 10 1000 bash tools/final_evidence.sh $T "$@" > $O/pmc$P.log 2>&1 || { tail $O/pmc$P.log; exit 1; }
grep profiled $O/pmc$P.log
