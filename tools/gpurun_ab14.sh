#!/bin/bash
# r06 ab14: batched agent-stream maintenance and lane-parallel wake times in the build kernel
set -o pipefail
O=gpurun_out/r06ab14
tools/ab_run.sh $O/build_rmsc03.txt "rP rN" 2 python tools/time_build.py rmsc03 4096 &&
tools/ab_run.sh $O/build_z1k.txt "zP zN" 2 python tools/time_build.py sparse_zi_1000 1024 &&
tools/ab_run.sh $O/build_vn.txt "vP vN" 2 python tools/time_build.py value_noise 4096 &&
tools/ab_run.sh $O/build_rfv.txt "fP fN" 2 python tools/time_build.py random_fund_value 2048 &&
tools/ab_run.sh $O/build_rfd.txt "dP dN" 1 python tools/time_build.py random_fund_diverse 2048 &&
tools/ab_run.sh $O/rmsc03.txt "rP rN" 1 python tools/ab_config.py rmsc03 4096 2 &&
tools/ab_run.sh $O/z1k.txt "zP zN" 1 python tools/ab_config.py sparse_zi_1000 1024 1 &&
tools/ab_run.sh $O/vn.txt "vP vN" 1 python tools/ab_config.py value_noise 4096 2 &&
tools/ab_run.sh $O/rfv.txt "fP fN" 1 python tools/ab_config.py random_fund_value 2048 1 &&
tools/ab_run.sh $O/rfd.txt "dP dN" 1 python tools/ab_config.py random_fund_diverse 2048 1
