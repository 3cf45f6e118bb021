set -o pipefail
for lib in libmxa_old.so libmxa.so; do
  MXA_LIB=$PWD/marl-optimal-execution_amd/lib/$lib timeout -k 10 300 python tools/ab_config.py sparse_zi_1000 1024 3 || exit 1
done
