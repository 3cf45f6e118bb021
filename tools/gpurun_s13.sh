set -o pipefail
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 bash tools/ab_cfg.sh s13 random_fund_value 2048 v9new v9ne && timeout -k 10 400 bash tools/ab_cfg.sh s13 sparse_zi_1000 1024 v2new v2ne || exit 1
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof9.so timeout -k 10 400 python tools/prof_phases.py random_fund_value 2048 > $O/phases_rfv.txt 2>&1 || { tail $O/phases_rfv.txt; exit 1; }
grep -E "total|q_remove|pop\+|q_push|send" $O/phases_rfv.txt
