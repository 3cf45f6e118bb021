#!/bin/bash
# r06 sched: a first launch of FC pops, then the running envs compacted into the next launch's grid
set -o pipefail
O=gpurun_out/r06sched2
mkdir -p $O
t() { local out=$1; shift; timeout -k 10 300 python tools/ab_sched.py "$@" >> $O/$out 2>&1 || { echo "failed: $*"; tail -5 $O/$out; return 1; }; }
t rmsc03.txt rmsc03 4096 "0 2048 4096 6144 8192 16384 0" 3 &&
t sbmmp.txt rmsc03_sbmm_poll 4096 "0 4096 8192" 2 &&
t sbmm.txt rmsc03_sbmm 4096 "0 4096" 2 &&
t z1k.txt sparse_zi_1000 1024 "0 8192" 1 &&
t rmsc01.txt rmsc01 4096 "0 8192" 1 &&
t rmsc02.txt rmsc02 4096 "0 8192" 1 &&
t rfv.txt random_fund_value 2048 "0 8192" 1
cat $O/*.txt
