set -o pipefail
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/${PTAG:-r2p1}
mkdir -p $OUT
MXA_LIB=$R/marl-optimal-execution_amd/lib/libmxa_prof.so timeout -k 10 300 python tools/prof_phases.py > $OUT/phases.txt 2>&1 || { echo "phases failed"; tail $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --no-cpu > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
cat $(find $OUT/trace -name '*kernel_stats.csv') | cut -c1-200
