set -o pipefail
bash tools/gpurun_final_bench1.sh && bash tools/gpurun_final_bench2.sh
