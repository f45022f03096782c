#!/bin/bash
# Round-3 A/B of the narrow Poisson pass (125M x 64 + offset + prior): the in-tree library (deviance
# without the per-row log) against sparkglm_amd/lib_ab/withlog (SGLM_POIS_NOLOG=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
AB_LIBS=sparkglm_amd/lib/libsglm_hip.so,sparkglm_amd/lib_ab/withlog/libsglm_hip.so AB_REPS=${AB_REPS:-3} \
  AN=125000000 AP=64 AK=2 AF=poisson AL=log timeout -k 10 600 python tools/ab.py 2>&1 | tee gpurun_out/ab_narrow3.log
