set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 900 bash tools/sq_counters.sh r04f sparse_zi_1000 1024 > gpurun_out/sq_z1k.log 2>&1 || { tail gpurun_out/sq_z1k.log; exit 1; }
tail -25 gpurun_out/sq_r04f/summary.txt
