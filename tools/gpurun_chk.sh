set -o pipefail
O=gpurun_out/chk; mkdir -p $O
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_chk3.so timeout -k 10 300 python -u -m pytest "tests/test_gpu_replay.py::test_gpu_replay_matches_reference_and_oracle" -x -v --timeout 200 --timeout-method thread -m gpu -s > $O/pytest.log 2>&1; rc=$?
grep -a "RPCHK" $O/pytest.log | head -20
tail -5 $O/pytest.log
exit $rc
