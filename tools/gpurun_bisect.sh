set -o pipefail
O=gpurun_out/bisect; mkdir -p $O
for v in ${VARIANTS:-v6 v7 v5}; do
  MXA_LIB=marl-optimal-execution_amd/lib/libmxa_$v.so timeout -k 10 200 python -u -m pytest "tests/test_gpu_replay.py::test_gpu_replay_matches_reference_and_oracle" -x -q --timeout 150 --timeout-method thread -m gpu > $O/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc"; tail -2 $O/$v.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
