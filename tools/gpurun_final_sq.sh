# final SQ issue records (on the GPU box): tools/sq_counters.sh per configuration.
# usage: tools/gpurun_final_sq.sh TAG CONFIG:ENVS ...
set -o pipefail
T=${1:?tag}; shift
for c in "$@"; do
  IFS=: read cfg envs <<< "$c"
  rm -rf gpurun_out/sq_${T}_$cfg
  timeout -k 10 400 bash tools/sq_counters.sh ${T}_$cfg $cfg $envs > gpurun_out/sq_${T}_$cfg.log 2>&1 || { tail gpurun_out/sq_${T}_$cfg.log; exit 1; }
  tail -1 gpurun_out/sq_${T}_$cfg.log
done
