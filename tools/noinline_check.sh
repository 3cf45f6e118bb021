#!/bin/bash
# Parity of the diagnostics builds with every engine helper a real call (-DMXA_DEV_NOINLINE,
# libmxa_c<ID>noinl.so): the configuration's GPU parity tests against its single-config variant.
# usage: tools/noinline_check.sh TAG "ID:TESTFILE:KEXPR" ...   -> gpurun_out/TAG/noinl_<ID>.log
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out/$TAG
for spec in "$@"; do
  IFS=: read id tf kx <<< "$spec"
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_c${id}noinl.so timeout -k 10 400 python -u -m pytest $tf -k "$kx" -m gpu -v \
    --timeout 300 --timeout-method thread > gpurun_out/$TAG/noinl_$id.log 2>&1
  rc=$?
  echo "cfg $id: rc $rc $(tail -1 gpurun_out/$TAG/noinl_$id.log)"
  [ $rc -le 1 ] || exit $rc
done
