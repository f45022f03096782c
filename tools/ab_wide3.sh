#!/bin/bash
# Round-3 A/B of the wide pass (p = 512 / 2048): the in-tree library (overlapped row kernel at
# 64 VGPRs) against sparkglm_amd/lib_ab/r96 (96 VGPRs, round 2).  (The unified diagonal + off-
# diagonal launch measured 111.0 against 101.2 ms at 20M x 512 and 202.5 against 199.5 ms at
# 3M x 2048 in an earlier version of this script, and was dropped.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for P in 512 2048; do
  if [ $P = 512 ]; then N=${N512:-20000000}; K=0; F=binomial; L=logit; else N=${N2048:-3000000}; K=3; F=gamma; L=inverse; fi
  echo "== p=$P"
  AB_LIBS=sparkglm_amd/lib/libsglm_hip.so,sparkglm_amd/lib_ab/r96/libsglm_hip.so AB_REPS=${AB_REPS:-3} \
    AN=$N AP=$P AK=$K AF=$F AL=$L timeout -k 10 600 python tools/ab.py || exit 1
done 2>&1 | tee gpurun_out/ab_wide3.log
