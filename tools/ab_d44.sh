#!/bin/bash
# Same-box A/B of the K1r diagonal-tile variants (SGLM_K1R_D44 / SGLM_K1R_SCHED builds under
# sparkglm_amd/lib_ab/): bitwise check against the in-tree library + pass time at 20M x 256.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
AB_LIBS=${AB_LIBS:-sparkglm_amd/lib/libsglm_hip.so,sparkglm_amd/lib_ab/d44dpp/libsglm_hip.so,sparkglm_amd/lib_ab/d44dpp4/libsglm_hip.so,sparkglm_amd/lib_ab/d44s0/libsglm_hip.so} \
  AN=${AN:-20000000} AB_REPS=${AB_REPS:-2} timeout -k 10 500 python tools/ab_k1r.py
