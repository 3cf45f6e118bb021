set -o pipefail
timeout -k 10 300 bash tools/ab_cfg.sh s15 rmsc02 4096 v7so9 v7ser
