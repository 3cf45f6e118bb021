#!/bin/bash
# A/B several configurations across single-configuration variant builds named c<ID><SUFFIX>
# (tools/build_variants.sh): usage tools/ab_sweep.sh TAG "SUFFIX..." CONFIG:ID:ENVS ...
set -o pipefail
TAG=$1; SUF=$2; shift 2
for spec in "$@"; do
  IFS=: read cfg id n <<< "$spec"
  vs=()
  for s in $SUF; do vs+=("c$id$s"); done
  tools/ab_cfg.sh $TAG $cfg $n "${vs[@]}" || exit 1
done
