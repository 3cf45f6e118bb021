#!/bin/bash
# one iteration on the GPU box: parity suite, smoke, default bench, then the phase profile
# of the MXA_PROF build (libmxa_prof.so, built beforehand by tools/build_variants.sh).
# usage: VTAG=tag bash tools/gpu_iter.sh
set -o pipefail
T=${VTAG:-it}
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo bench failed; tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('bench %.3fG env-steps/s, %.1f ms/step, run kernel %.1f ms' % (d['value']/1e9, d['ms_per_step'], d['roofline']['avg_launch_ms']))"
if [ -f marl-optimal-execution_amd/lib/libmxa_prof.so ]; then
  MXA_LIB=$PWD/marl-optimal-execution_amd/lib/libmxa_prof.so timeout -k 10 300 python tools/prof_phases.py > $O/phases.txt 2>&1 || { echo "phases failed"; tail $O/phases.txt; exit 1; }
  cat $O/phases.txt
fi
timeout -k 10 200 python tools/host_timing.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; tail $O/host_timing.txt; exit 1; }
cat $O/host_timing.txt
if [ -n "$RLT" ]; then
  timeout -k 10 200 python tools/host_timing_rl.py > $O/host_timing_rl.txt 2>&1 || { echo "rl host timing failed"; tail $O/host_timing_rl.txt; exit 1; }
  cat $O/host_timing_rl.txt
fi
