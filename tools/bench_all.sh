#!/bin/bash
# Every BASELINE config as a bench workload (1 GPU): one JSON line each -> gpurun_out/bench_<wl>.json,
# and a rocprofv3 --kernel-trace --stats summary of the same command -> gpurun_out/prof_<wl>/
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for wl in ${WLS:-logit256 poisson64 logit512 logit512r gamma2048 logit1b lm20}; do
  steps=10; warm=2
  [[ $wl == lm20 ]] && { steps=50; warm=5; }
  [[ $wl == gamma2048 || $wl == logit512 ]] && { steps=3; warm=1; }
  [[ $wl == logit1b ]] && { steps=5; warm=1; }
  timeout -k 10 400 python bench.py --workload $wl --steps $steps --warmup $warm > gpurun_out/bench_$wl.json 2> gpurun_out/bench_$wl.err
  rc=$?
  echo "$wl rc=$rc"; cat gpurun_out/bench_$wl.json
  [[ $rc -ne 0 ]] && { tail -20 gpurun_out/bench_$wl.err; exit $rc; }
  if [[ -n "$PROF" ]]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$wl" -o run --output-format csv -- python bench.py --workload $wl --steps $steps --warmup $warm --no-cpu-baseline > gpurun_out/prof_bench_$wl.json 2> gpurun_out/prof_bench_$wl.err
    rc=$?
    echo "prof $wl rc=$rc"
    [[ $rc -ne 0 ]] && { tail -20 gpurun_out/prof_bench_$wl.err; exit $rc; }
  fi
done
exit 0
