#!/bin/bash
# A/B of the banded-schedule pace (SGLM_WIDE_PACE) on the wide workloads + PMC HBM bytes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_wide.py -v --timeout 120 --timeout-method thread -W ignore > gpurun_out/pace_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/pace_tests.log | head -20; tail -5 gpurun_out/pace_tests.log; exit 1; }
tail -1 gpurun_out/pace_tests.log
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/pace_$lab.json 2> gpurun_out/pace_$lab.err || { echo "bench $lab failed"; tail -20 gpurun_out/pace_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/pace_$lab.json')); b=d['breakdown_ms_per_step']; r=d['roofline']; print('$lab', round(d['ms_per_step'],2), 'pass', round(b['pass_kernels'],2), 'gram', round(r['kernel_ms'],2), 'rows', round(b['row_kernel'],2), 'frac', round(r['frac'],4))"
}
for WL in gamma2048 logit512r; do
  run ${WL}_pace1 SGLM_WIDE_PACE=1 || exit 1
  run ${WL}_pace0 SGLM_WIDE_PACE=0 || exit 1
  run ${WL}_pace1b SGLM_WIDE_PACE=1 || exit 1
  run ${WL}_pace0b SGLM_WIDE_PACE=0 || exit 1
done
for v in 1 0; do  # chunk sizes as in the full-size workloads (gamma2048 781K rows, logit512r 3.75M)
  SGLM_WIDE_PACE=$v SGLM_WIDE_OVERLAP=3 WLS="gamma2048" bash tools/pmc_workloads.sh > gpurun_out/pace_pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pace_pmc_$v.log; exit 1; }
  SGLM_WIDE_PACE=$v SGLM_WIDE_OVERLAP=2 WLS="logit512" bash tools/pmc_workloads.sh >> gpurun_out/pace_pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 gpurun_out/pace_pmc_$v.log; exit 1; }
  mv gpurun_out/pmc gpurun_out/pmc_pace$v
  python tools/pmc_traffic.py gpurun_out/pmc_pace$v pace$v gpurun_out/pt$v.json | tail -3
done
