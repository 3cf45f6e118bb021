set -o pipefail
O=gpurun_out/ph4
mkdir -p $O
MXA_LIB=$PWD/marl-optimal-execution_amd/lib/libmxa_prof2.so timeout -k 10 300 python tools/prof_phases.py sparse_zi_1000 1024 > $O/phases_z1k.txt 2>&1 || { tail $O/phases_z1k.txt; exit 1; }
cat $O/phases_z1k.txt
