#!/bin/bash
# r06 pf: MarketReplayAgent tape look-ahead (MXA_MR_PF_MASK), replay step kernel, same digests
set -o pipefail
O=gpurun_out/r06pf; mkdir -p $O
for r in 1 2; do
  for v in rp0 rpP; do
    MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_replay_many.py IBM_2003-01-14 512 3 >> $O/ibm_many.txt 2>&1 || { echo "$v failed"; tail -5 $O/ibm_many.txt; exit 1; }
  done
done
for v in rp0 rpP; do
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_replay_many.py GOOG_2012-06-21 512 2 >> $O/goog_many.txt 2>&1 || { echo "$v failed"; tail -5 $O/goog_many.txt; exit 1; }
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python tools/ab_replay.py IBM_2003-01-14 512 1 >> $O/ibm_step.txt 2>&1 || { echo "$v failed"; tail -5 $O/ibm_step.txt; exit 1; }
done
cat $O/*.txt
