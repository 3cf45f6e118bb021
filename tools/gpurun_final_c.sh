set -o pipefail
timeout -k 10 120 python -u -m pytest tests/test_gpu_records.py -x -v --timeout 100 --timeout-method thread -m gpu > gpurun_out/records.log 2>&1 || { tail -30 gpurun_out/records.log; exit 1; }
tail -2 gpurun_out/records.log
bash tools/gpurun_final_a.sh
