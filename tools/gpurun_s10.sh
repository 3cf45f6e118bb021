set -o pipefail
O=gpurun_out/s10; mkdir -p $O
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
cat $O/prof_replay_ibm.txt
