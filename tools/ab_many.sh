#!/bin/bash
# A/B runs: "kind:variant:config:envs" ... (kind run = tools/ab_config.py, replay = tools/ab_replay.py)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for spec in "$@"; do
  IFS=: read kind v cfg n <<< "$spec"
  if [ "$kind" = replay ]; then
    MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_replay.py $cfg $n 2 2>>gpurun_out/$TAG/err.log | tee -a gpurun_out/$TAG/ab.txt || exit 1
  else
    MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_config.py $cfg $n 2 2>>gpurun_out/$TAG/err.log | tee -a gpurun_out/$TAG/ab.txt || exit 1
  fi
done
