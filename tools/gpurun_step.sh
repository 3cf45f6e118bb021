#!/bin/bash
# One GPU check of a kernel change: selected -m gpu tests, then bench lines without the CPU leg.
# usage (on the GPU box, from the repo root): tools/gpurun_step.sh TAG "TESTS" "CONFIG[:ENVS[:TAPE]] ..."
#   -> gpurun_out/TAG/{pytest.log,bench_<config>.json}
set -o pipefail
TAG=$1; TESTS=$2; BENCH=$3
O=gpurun_out/$TAG; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 \
    || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest.log | head -30; tail -5 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for b in $BENCH; do
  IFS=: read cfg envs tape <<< "$b"
  args="--config $cfg --no-cpu"
  [ -n "$envs" ] && args="$args --envs $envs"
  [ -n "$tape" ] && args="$args --tape $tape"
  name=$cfg${tape:+_$tape}
  timeout -k 10 300 python bench.py $args --steps ${STEPS:-3} > $O/bench_$name.json 2> $O/bench_$name.err \
    || { echo "bench $b failed"; tail $O/bench_$name.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/bench_$name.json').read().strip().splitlines()[-1]); r=d.get('roofline',{}); print('$name', '%.4g' % d['value'], '%.2f ms' % d['ms_per_step'], r.get('kernel'), r.get('avg_launch_ms'))"
done
