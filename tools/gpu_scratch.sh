set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
for lib in libmxa_nof.so libmxa.so; do
  MXA_LIB=$PWD/marl-optimal-execution_amd/lib/$lib timeout -k 10 300 python tools/ab_config.py rmsc03 4096 3 || exit 1
done
done
