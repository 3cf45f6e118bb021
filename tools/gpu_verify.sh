#!/bin/bash
# One GPU verification pass: the -m gpu suite (or the test paths given), smoke(), the default bench.
# usage (on the GPU box, from the repo root): tools/gpu_verify.sh TAG [TEST_PATH...]
#   -> gpurun_out/TAG/{pytest_gpu.log,smoke.log,bench.json}
set -o pipefail
TAG=${1:-v1}
shift
TESTS=${@:-tests}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 1000 python -u -m pytest $TESTS -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
cut -c1-800 $O/bench.json
