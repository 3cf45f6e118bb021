set -o pipefail
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/r2p5
mkdir -p $OUT
MXA_LIB=$R/marl-optimal-execution_amd/lib/libmxa_vexp.so timeout -k 10 300 python tools/prof_phases.py > $OUT/phases_vexp.txt 2>&1 || { echo "phases failed"; tail $OUT/phases_vexp.txt; exit 1; }
cat $OUT/phases_vexp.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_rl -o run -- python3 $R/bench.py --config rmsc03_rl --no-cpu --steps 2 --warmup 1 > $OUT/trace_rl.log 2>&1 || { echo "trace failed"; tail $OUT/trace_rl.log; exit 1; }
