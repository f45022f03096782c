#!/bin/bash
# Every BASELINE config as a bench workload (1 GPU), one JSON line each -> gpurun_out/bench_<wl>.json
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for wl in ${WLS:-poisson64 logit512 gamma2048}; do
  steps=10; warm=2
  [[ $wl == gamma2048 ]] && { steps=3; warm=1; }
  timeout -k 10 400 python bench.py --workload $wl --steps $steps --warmup $warm > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  rc=$?
  echo "$wl rc=$rc"; cat gpurun_out/bench_$wl.json
  [[ $rc -ne 0 ]] && { tail -20 gpurun_out/bench_$wl.err; exit $rc; }
done
exit 0
