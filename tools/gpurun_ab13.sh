#!/bin/bash
# r06 ab13: the ZI / HBL theta draws 64 agents at once in the build kernel: build time, run kernel
# and per-env digests (the digest covers every pop, so a wrong theta shows)
set -o pipefail
O=gpurun_out/r06ab13
tools/ab_run.sh $O/build_z1k.txt "zA zZ" 2 python tools/time_build.py sparse_zi_1000 256 1024 &&
tools/ab_run.sh $O/build_z100.txt "sA sZ" 2 python tools/time_build.py sparse_zi_100 4096 &&
tools/ab_run.sh $O/build_rmsc01.txt "oA oZ" 2 python tools/time_build.py rmsc01 4096 &&
tools/ab_run.sh $O/z1k.txt "zA zZ" 1 python tools/ab_config.py sparse_zi_1000 1024 1 &&
tools/ab_run.sh $O/z100.txt "sA sZ" 1 python tools/ab_config.py sparse_zi_100 4096 2 &&
tools/ab_run.sh $O/rmsc01.txt "oA oZ" 1 python tools/ab_config.py rmsc01 4096 1
