#!/bin/bash
# PMC HBM records and rocprofv3 kernel stats of the final build for several configurations
# (tools/profile_round.sh each), stopping at the first failure.
# usage: tools/final_evidence.sh TAG CONFIG:ENVS[:TAPE] ...  -> gpurun_out/prof_TAG_CONFIG/, profiles/hbm_traffic_CONFIG.json
set -o pipefail
TAG=$1
shift
for c in "$@"; do
  IFS=: read cfg envs tape <<< "$c"
  bash tools/profile_round.sh ${TAG}_$cfg${tape:+_$tape} $cfg $envs $tape || { echo "profile $cfg failed"; exit 1; }
  echo "profiled $cfg x$envs"
done
