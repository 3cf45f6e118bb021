set -o pipefail
mkdir -p gpurun_out/${VTAG:-v1}
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/${VTAG:-v1}/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${VTAG:-v1}/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${VTAG:-v1}/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${VTAG:-v1}/smoke.log 2>&1 || { echo smoke failed; tail gpurun_out/${VTAG:-v1}/smoke.log; exit 1; }
cat gpurun_out/${VTAG:-v1}/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${VTAG:-v1}/bench.json 2> gpurun_out/${VTAG:-v1}/bench.err || { echo bench failed; tail gpurun_out/${VTAG:-v1}/bench.err; exit 1; }
cut -c1-600 gpurun_out/${VTAG:-v1}/bench.json
