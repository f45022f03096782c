#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_wide.py tests/test_gpu_speculate.py -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/ov_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ov_tests.log; exit 1; }
tail -3 gpurun_out/ov_tests.log
for wl in logit512r gamma2048; do
  for ov in 1 4 8; do
    SGLM_WIDE_OVERLAP=$ov timeout -k 10 300 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/ov_${wl}_$ov.json 2> gpurun_out/ov_${wl}_$ov.err || { echo "bench $wl $ov failed"; tail -20 gpurun_out/ov_${wl}_$ov.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/ov_${wl}_$ov.json')); print('$wl ov=$ov', round(d['ms_per_step'],2), d['breakdown_ms_per_step'], round(d['roofline']['frac'],4), d['time_to_converge_s'], d['iters_to_converge'], d['deviance'])"
  done
done
