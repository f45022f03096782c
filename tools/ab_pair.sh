# A/B of the narrow pass's row pairs (SGLM_NPAIR=0 build in lib_ab/np0 vs the in-tree library) at
# p = 32 (logit1b's pattern), p = 20 and p = 12, then the narrow-path GPU parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=sparkglm_amd/lib_ab/np0/libsglm_hip.so,sparkglm_amd/lib/libsglm_hip.so AB_REPS=${AB_REPS:-3}
AN=200000000 AP=32 AK=0 AF=binomial AL=logit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab_pair1.log &&
AN=100000000 AP=20 AK=1 AF=gaussian AL=identity timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab_pair2.log &&
AN=100000000 AP=12 AK=0 AF=binomial AL=probit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab_pair3.log &&
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -W ignore --timeout 300 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pair.log; exit $rc
