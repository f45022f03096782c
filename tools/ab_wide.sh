# A/B of the wide path (row + Gram kernels): sparkglm_amd/lib_ab/head (the committed tree, built
# with make variant NAME=head) against the in-tree library, then the wide-path GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=${AB_LIBS:-sparkglm_amd/lib_ab/head/libsglm_hip.so,sparkglm_amd/lib/libsglm_hip.so} AB_REPS=${AB_REPS:-3}
AN=20000000 AP=512 AK=0 AF=binomial AL=logit timeout -k 10 400 python tools/ab.py 2>&1 | tee gpurun_out/ab_wide1.log &&
AN=3000000 AP=2048 AK=3 AF=gamma AL=inverse timeout -k 10 400 python tools/ab.py 2>&1 | tee gpurun_out/ab_wide2.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q -W ignore --timeout 300 --timeout-method thread > gpurun_out/pytest_wide.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_wide.log; exit $rc
