set -o pipefail
O=gpurun_out/obi1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_obi.py tests/test_gpu_rmsc02.py tests/test_gpu_booklog.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "obi or rmsc02 or book_log or fundamental" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
