set -o pipefail
rm -rf gpurun_out/sq_r04f
timeout -k 10 900 bash tools/sq_counters.sh r04f sparse_zi_1000 1024 > gpurun_out/sq_z1k.log 2>&1 || { tail gpurun_out/sq_z1k.log; exit 1; }
grep -A22 "mxa_run_kernel" gpurun_out/sq_r04f/summary.txt
