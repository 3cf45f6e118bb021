#!/bin/bash
# GPU parity suite, smoke, default bench, then rocprofv3 kernel stats + HBM counters
# (tools/profile_round.sh). usage: tools/gpu_round2.sh TAG
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
cut -c1-300 $OUT/bench.json
bash tools/profile_round.sh $TAG > $OUT/profile.log 2>&1 || { echo profile failed; tail $OUT/profile.log; exit 1; }
tail -30 $OUT/profile.log
