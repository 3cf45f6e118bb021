#!/bin/bash
# bench.py for several configurations in one GPU call (each under its own time limit; stops at
# the first failure).  usage: tools/bench_sweep.sh TAG CONFIG[:ENVS] ... [-- EXTRA BENCH ARGS]
#   -> gpurun_out/TAG/bench_CONFIG_ENVS.json
set -o pipefail
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
CFGS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do CFGS+=("$1"); shift; done
[ "$1" = "--" ] && shift
for c in "${CFGS[@]}"; do
  IFS=: read cfg envs <<< "$c"
  E=${envs:+--envs $envs}
  timeout -k 10 400 python bench.py --config $cfg $E "$@" > $O/bench_${cfg}_${envs:-default}.json 2> $O/bench_${cfg}.err \
    || { echo "bench $cfg failed"; tail $O/bench_${cfg}.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], 'ms/step %.1f' % d['ms_per_step'], 'kernel %.2f ms' % d.get('roofline',{}).get('avg_launch_ms',0), 'err', d['config']['env_errors'], 'cpu %.4g' % d.get('cpu_baseline',{}).get('value',0))" $O/bench_${cfg}_${envs:-default}.json $cfg
done
