#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_wide.py tests/test_gpu_speculate.py -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/ov2_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/ov2_tests.log | head -30; tail -5 gpurun_out/ov2_tests.log; exit 1; }
tail -2 gpurun_out/ov2_tests.log
WL=logit512
for po in 0 8 16; do
  SGLM_PROC_OVERLAP=$po timeout -k 10 400 python bench.py --workload $WL --steps 3 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/ov2_$po.json 2> gpurun_out/ov2_$po.err || { echo "bench $po failed"; tail -20 gpurun_out/ov2_$po.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ov2_$po.json')); b=d['breakdown_ms_per_step']; r=d['roofline']; print('po=$po', round(d['ms_per_step'],2), 'pass', round(b['pass_kernels'],2), 'gram', round(r['kernel_ms'],2), 'rows', round(b['row_kernel'],2), 'frac', round(r['frac'],4), 'ttc', round(d['time_to_converge_s'],3), d['iters_to_converge'], d['deviance'])"
done
