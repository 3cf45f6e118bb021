set -o pipefail
O=gpurun_out/rp4
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_replay.log 2>&1 || { tail -30 $O/pytest_replay.log; exit 1; }
tail -8 $O/pytest_replay.log
