set -o pipefail
O=gpurun_out/s12; mkdir -p $O
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof9.so timeout -k 10 400 python tools/prof_phases.py random_fund_value 2048 > $O/phases_rfv.txt 2>&1 || { tail $O/phases_rfv.txt; exit 1; }
cat $O/phases_rfv.txt
