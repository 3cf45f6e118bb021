#!/bin/bash
# A/B of one configuration's run kernel across single-configuration library variants
# (tools/build_variants.sh NAME:.:-DMXA_ONLY_CFG=<id> ...); usage: tools/ab_cfg.sh TAG CONFIG ENVS VARIANT...
set -o pipefail
TAG=$1; CFG=$2; N=$3; shift 3
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_config.py $CFG $N 2 2>>gpurun_out/$TAG/err.log | tee -a gpurun_out/$TAG/ab.txt || exit 1
done
