set -o pipefail
O=gpurun_out/wq
mkdir -p $O
L=$PWD/marl-optimal-execution_amd/lib
MXA_LIB=$L/libmxa_noapf03.so timeout -k 10 200 python tools/ab_config.py rmsc03 4096 3 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
for w in 0 3600 3400 3200 3000 2800; do
echo "MXA_RUN_WAVES=$w" >> $O/ab.txt
MXA_RUN_WAVES=$w MXA_LIB=$L/libmxa_wq03.so timeout -k 10 200 python tools/ab_config.py rmsc03 4096 3 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }
done
cat $O/ab.txt
