#!/bin/bash
# the final bench lines of one evidence series (TAG) into profiles/r06/final/bench/, under the
# names tools/bench_table.py reads.  usage: tools/assemble_bench.sh TAG
set -e
T=${1:?tag}
B=profiles/r06/final/bench
mkdir -p $B
for d in gpurun_out/${T}_b1 gpurun_out/${T}_b2 gpurun_out/${T}_cfg; do
  [ -d $d ] && for f in $d/bench_*.json; do cp $f $B/; done
done
[ -f gpurun_out/${T}_e/bench_rmsc03_default.json ] && cp gpurun_out/${T}_e/bench_rmsc03_default.json $B/
[ -f gpurun_out/${T}_goog/bench_marketreplay_default.json ] && cp gpurun_out/${T}_goog/bench_marketreplay_default.json $B/bench_marketreplay_GOOG_2012-06-21.json
[ -f gpurun_out/${T}_shard/bench_rmsc03_ddqn_512.json ] && cp gpurun_out/${T}_shard/bench_rmsc03_ddqn_512.json $B/
[ -f gpurun_out/${T}_shard/bench_marketreplay_64.json ] && cp gpurun_out/${T}_shard/bench_marketreplay_64.json $B/
[ -f gpurun_out/${T}_shard_goog/bench_marketreplay_64.json ] && cp gpurun_out/${T}_shard_goog/bench_marketreplay_64.json $B/bench_marketreplay_64_GOOG_2012-06-21.json
grep -L "\"value\"" $B/*.json || true
