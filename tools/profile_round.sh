#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats of a bench command, then HBM traffic
# counters in their own passes (FETCH_SIZE, WRITE_SIZE; never mixed with traces).
# usage: tools/profile_round.sh TAG [CONFIG] [ENVS] [TAPE]  -> gpurun_out/prof_TAG/...
#   (TAPE: marketreplay on another tape than IBM_2003-01-14; the record is hbm_traffic_CONFIG_TAPE.json)
#   writes gpurun_out/prof_TAG/hbm_traffic_CONFIG.json (stamped with the library's build id);
#   copy it to profiles/ so bench.py reports it as roofline.traffic for this build
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r02}
CFG=${2:-rmsc03}
ENVS=${3:-4096}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
TAPE=${4:-}
B="$R/bench.py --config $CFG --envs $ENVS --no-cpu --no-count --no-latency${TAPE:+ --tape $TAPE}"
export MXA_PROF_TAPE=$TAPE
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $B > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail $OUT/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 $B --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail $OUT/fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 $B --steps 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "write pass failed"; tail $OUT/write.log; exit 1; }
cd $R
python3 tools/hbm_summary.py $OUT --record $CFG $ENVS 0 \
  "tools/profile_round.sh $TAG: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of" \
  "'bench.py --config $CFG --envs $ENVS${TAPE:+ --tape $TAPE} --steps 1 --warmup 0 --no-cpu --no-count' (parity hash off, as bench.py runs);" \
  "reads doubled per MI355X_MICROARCH.md HBM section (gfx950 FETCH_SIZE reports half); L2 memory-side" \
  "requests, Infinity-Cache hits included"
