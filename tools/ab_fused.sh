# A/B of fused-pass (p = 256) build variants under sparkglm_amd/lib_ab/<name>/ against the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=sparkglm_amd/lib/libsglm_hip.so,${AB_VARIANTS:-sparkglm_amd/lib_ab/s18/libsglm_hip.so,sparkglm_amd/lib_ab/k6/libsglm_hip.so,sparkglm_amd/lib_ab/k5/libsglm_hip.so} AB_REPS=${AB_REPS:-3}
AN=30000000 AP=256 AK=0 AF=binomial AL=logit timeout -k 10 600 python tools/ab.py 2>&1 | tee gpurun_out/ab_fused.log
