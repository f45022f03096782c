#!/bin/bash
# Initial-pass constants in LDS (K1 / K1r): bitwise whole-fit A/B against the previous build
# (sparkglm_amd/lib_ab/head), the GPU suite + smoke, then the headline bench line A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_LIBS=sparkglm_amd/lib_ab/head/libsglm_hip.so,sparkglm_amd/lib/libsglm_hip.so timeout -k 10 600 python tools/ab_fit.py > gpurun_out/ab_fit.log 2>&1; rc=$?
cat gpurun_out/ab_fit.log; [[ $rc -ne 0 ]] && exit $rc
bash tools/r03_gpu.sh test r03d || exit 1
AB_SPECS="sparkglm_amd/lib_ab/head/libsglm_hip.so sparkglm_amd/lib/libsglm_hip.so" REPS=2 bash tools/ab_bench.sh || exit 1
exit 0
