#!/bin/bash
# Poisson initial-pass table (narrow kernel): bitwise whole-fit A/B against the previous build,
# the GPU suite, then the poisson64 bench line A/B (time to converge).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_CASES="2:30000000:64:poisson:log:multiple,2:30000000:64:poisson:log:single,2:20000000:40:poisson:log:multiple,2:20000000:24:poisson:log:multiple,0:20000000:48:binomial:logit:multiple" \
AB_LIBS=sparkglm_amd/lib_ab/head/libsglm_hip.so,sparkglm_amd/lib/libsglm_hip.so timeout -k 10 600 python tools/ab_fit.py > gpurun_out/ab_fit_pois.log 2>&1; rc=$?
cat gpurun_out/ab_fit_pois.log; [[ $rc -ne 0 ]] && exit $rc
bash tools/r03_gpu.sh test r03e || exit 1
AB_SPECS="sparkglm_amd/lib_ab/head/libsglm_hip.so sparkglm_amd/lib/libsglm_hip.so" REPS=2 BENCH_ARGS="--workload poisson64" bash tools/ab_bench.sh || exit 1
exit 0
