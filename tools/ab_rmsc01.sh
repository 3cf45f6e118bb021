#!/bin/bash
# A/B of rmsc01's run kernel across single-configuration library variants (tools/build_variants.sh
# with -DMXA_ONLY_CFG=6), interleaved; usage: tools/ab_rmsc01.sh TAG VARIANT...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 120 python tools/ab_config.py rmsc01 4096 3 2>>gpurun_out/$TAG/err.log | tee -a gpurun_out/$TAG/ab.txt || exit 1
done
