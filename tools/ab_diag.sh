# A/B of the diagonal super-tile pipeline (WIDE_DIAG2 = 0: one block per stage, lib_ab/d0) against
# the in-tree library on the wide path; then the in-tree library with SGLM_WIDE_BAND=2 at p = 2048.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=sparkglm_amd/lib_ab/d0/libsglm_hip.so,sparkglm_amd/lib/libsglm_hip.so AB_REPS=${AB_REPS:-3}
AN=20000000 AP=512 AK=0 AF=binomial AL=logit timeout -k 10 300 python tools/ab.py 2>&1 | tee gpurun_out/ab_diag1.log &&
AN=3000000 AP=2048 AK=3 AF=gamma AL=inverse timeout -k 10 300 python tools/ab.py 2>&1 | tee gpurun_out/ab_diag2.log &&
AB_LIBS=sparkglm_amd/lib/libsglm_hip.so SGLM_WIDE_BAND=2 AN=3000000 AP=2048 AK=3 AF=gamma AL=inverse timeout -k 10 300 python tools/ab.py 2>&1 | tee gpurun_out/ab_diag3.log
