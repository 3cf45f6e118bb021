set -o pipefail
timeout -k 10 300 bash tools/bench_sweep.sh r04fb3 rmsc03_ddqn
