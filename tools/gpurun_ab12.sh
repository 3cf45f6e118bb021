#!/bin/bash
# r06 ab12: build-kernel changes (LDS RNG windows, one-round-trip MT blocks, LDS-tiled seeding,
# agent look-ahead) A/B: build time per config, run kernel and per-env digests
set -o pipefail
O=gpurun_out/r06ab12
tools/ab_run.sh $O/build_rmsc03.txt "r0 rA" 2 python tools/time_build.py rmsc03 4096 &&
tools/ab_run.sh $O/build_z100.txt "s0 sA" 2 python tools/time_build.py sparse_zi_100 4096 &&
tools/ab_run.sh $O/build_vn.txt "v0 vA" 2 python tools/time_build.py value_noise 4096 &&
tools/ab_run.sh $O/build_z1k.txt "z0 zA zL zS" 1 python tools/time_build.py sparse_zi_1000 1024 &&
tools/ab_run.sh $O/build_rfv.txt "f0 fA fL fS" 1 python tools/time_build.py random_fund_value 2048 &&
tools/ab_run.sh $O/rmsc03.txt "r0 rA" 2 python tools/ab_config.py rmsc03 4096 2 &&
tools/ab_run.sh $O/z100.txt "s0 sA" 1 python tools/ab_config.py sparse_zi_100 4096 2 &&
tools/ab_run.sh $O/vn.txt "v0 vA" 1 python tools/ab_config.py value_noise 4096 2 &&
tools/ab_run.sh $O/z1k.txt "z0 zA" 1 python tools/ab_config.py sparse_zi_1000 1024 1 &&
tools/ab_run.sh $O/rfv.txt "f0 fA" 1 python tools/ab_config.py random_fund_value 2048 1
