#!/bin/bash
# r06 ab19: -fno-slp-vectorize per configuration (run / step kernels, same digests)
set -o pipefail
O=gpurun_out/r06ab19
tools/ab_run.sh $O/z1k.txt "z0 zF" 2 python tools/ab_config.py sparse_zi_1000 1024 1 &&
tools/ab_run.sh $O/rmsc01.txt "o0 oF" 1 python tools/ab_config.py rmsc01 4096 1 &&
tools/ab_run.sh $O/rmsc02.txt "m0 mF" 1 python tools/ab_config.py rmsc02 4096 1 &&
tools/ab_run.sh $O/z100.txt "s0 sF" 2 python tools/ab_config.py sparse_zi_100 4096 2 &&
tools/ab_run.sh $O/vn.txt "v0 vF" 2 python tools/ab_config.py value_noise 4096 3 &&
tools/ab_run.sh $O/rfv.txt "f0 fF" 1 python tools/ab_config.py random_fund_value 2048 1 &&
tools/ab_run.sh $O/ibm.txt "rp0 rpF" 2 python tools/ab_replay.py IBM_2003-01-14 512 2
