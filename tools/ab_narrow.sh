# A/B of narrow-pass (p <= 64) builds: sparkglm_amd/lib_ab/base.so vs the in-tree library, then the GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=sparkglm_amd/lib_ab/base.so,sparkglm_amd/lib/libsglm_hip.so AB_REPS=4
AN=200000000 AP=32 AK=0 AF=binomial AL=logit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab1.log &&
AN=60000000 AP=64 AK=2 AF=poisson AL=log timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab2.log &&
AN=100000000 AP=20 AK=0 AF=binomial AL=logit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab3.log &&
timeout -k 10 300 python -m pytest tests -m gpu -x -q -W ignore > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
