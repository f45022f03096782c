#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_speculate.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_dist.py -v --timeout 300 --timeout-method thread -W ignore > gpurun_out/lean_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/lean_tests.log | head -20; tail -5 gpurun_out/lean_tests.log; exit 1; }
tail -1 gpurun_out/lean_tests.log
timeout -k 10 400 python bench.py --workload logit1b --steps 5 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/lean_logit1b.json 2> gpurun_out/lean_logit1b.err || { tail -20 gpurun_out/lean_logit1b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/lean_logit1b.json')); r=d['roofline']; print('logit1b', round(d['ms_per_step'],2), 'kernel', round(r['kernel_ms'],2), 'frac', round(r['frac'],4), 'ttc', round(d['time_to_converge_s'],4), d['iters_to_converge'], d['deviance'])"
