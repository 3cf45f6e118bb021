# final evidence, part A (on the GPU box): the GPU suite, then the PMC HBM records and kernel stats
# of every bench configuration.  usage: tools/gpurun_final_a.sh TAG
set -o pipefail
T=${1:?tag}
O=gpurun_out/final_$T; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 850 bash tools/final_evidence.sh $T rmsc03:4096 rmsc03_rl:4096 rmsc03_ddqn:4096 sparse_zi_1000:1024 marketreplay:512 marketreplay:512:GOOG_2012-06-21 random_fund_value:2048 sparse_zi_100:4096 value_noise:4096 rmsc03_sbmm:4096 rmsc03_sbmm_poll:4096 rmsc03_sweep:4096 > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 1; }
grep profiled $O/pmc1.log
timeout -k 10 500 bash tools/final_evidence.sh $T rmsc01:4096 rmsc02:4096 obi_rmsc02:4096 random_fund_diverse:2048 hist_fund_value:2048 hist_fund_diverse:2048 > $O/pmc2.log 2>&1 || { tail $O/pmc2.log; exit 1; }
grep profiled $O/pmc2.log
