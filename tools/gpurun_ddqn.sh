#!/bin/bash
# r06 ddqn: the fused per-period kernels (libmxa_ddqn.so) — the DDQN GPU tests (the default path is
# the fused one), then rmsc03_ddqn bench lines: x4096 fused and with the PyTorch ops, x512 fused
set -o pipefail
O=gpurun_out/r06ddqn2; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_ddqn.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config rmsc03_ddqn > $O/bench_fused.json 2> $O/bench_fused.err || { tail $O/bench_fused.err; exit 1; }
timeout -k 10 300 python bench.py --config rmsc03_ddqn --ddqn-torch --no-cpu > $O/bench_torch.json 2> $O/bench_torch.err || { tail $O/bench_torch.err; exit 1; }
timeout -k 10 300 python bench.py --config rmsc03_ddqn --envs 512 > $O/bench_rmsc03_ddqn_512.json 2> $O/bench_512.err || { tail $O/bench_512.err; exit 1; }
for f in bench_fused bench_torch bench_rmsc03_ddqn_512; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], '%.4g' % d['value'], 'ms/step %.2f' % d['ms_per_step'], d['config'].get('learner_period'))" $O/$f.json $f; done
