set -o pipefail
O=gpurun_out/mdc
mkdir -p $O
L=$PWD/marl-optimal-execution_amd/lib
for rep in 1 2; do
for v in old7 new7; do MXA_LIB=$L/libmxa_$v.so timeout -k 10 300 python tools/ab_config.py rmsc02 4096 1 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }; done
for v in old8 new8; do MXA_LIB=$L/libmxa_$v.so timeout -k 10 300 python tools/ab_config.py obi_rmsc02 4096 1 >> $O/ab.txt 2>&1 || { tail $O/ab.txt; exit 1; }; done
done
cat $O/ab.txt
