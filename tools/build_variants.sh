#!/bin/bash
# build rmsc03-only libmxa variants: NAME:SRCROOT:FLAGS...   (SRCROOT "." = working tree)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
pids=()
for spec in "$@"; do
  IFS=: read name root flags <<< "$spec"
  [ "$root" = "." ] && root=$R
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -ffp-contract=off -fno-fast-math -fPIC -shared \
    -Wno-unused-result -Wno-unused-value -mllvm -structurizecfg-skip-uniform-regions -DMXA_ONLY_RMSC03 $flags -I$root/marl-optimal-execution_amd/csrc -I$root/include \
    $root/marl-optimal-execution_amd/csrc/mxa_api.hip -o $R/marl-optimal-execution_amd/lib/libmxa_$name.so &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
