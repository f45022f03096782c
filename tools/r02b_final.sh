#!/bin/bash
# Final checks: overlap GPU tests, the default bench (stdout = one JSON line), the 2-rank rehearsal.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/fin_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/fin_tests.log | head; tail -5 gpurun_out/fin_tests.log; exit 1; }
tail -1 gpurun_out/fin_tests.log
timeout -k 10 600 python bench.py --gpus 2 --rows 10000000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02b_gpus2.json 2> gpurun_out/r02b_gpus2.err || { echo "gpus2 failed"; tail -20 gpurun_out/r02b_gpus2.err; exit 1; }
wc -l gpurun_out/r02b_gpus2.json
python -c "import json; d=json.load(open('gpurun_out/r02b_gpus2.json')); print(d['n_gpus'], d['config']['parallelism'], d['value'], d['strong_scaling_1b_logit'])"
