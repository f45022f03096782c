#!/bin/bash
# A/B of narrow-pass (p <= 64) builds: sparkglm_amd/lib_ab/base.so vs the in-tree library, on the
# configs[2] shard (125M x 64 poisson + offset + prior), a 200M-row slice of logit1b (p = 32) and
# p = 20, then the narrow-path GPU parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_LIBS=sparkglm_amd/lib_ab/base.so,sparkglm_amd/lib/libsglm_hip.so AB_REPS=${AB_REPS:-3}
AN=200000000 AP=32 AK=0 AF=binomial AL=logit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab1.log &&
AN=125000000 AP=64 AK=2 AF=poisson AL=log timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab2.log &&
AN=100000000 AP=20 AK=0 AF=binomial AL=logit timeout -k 10 240 python tools/ab.py 2>&1 | tee gpurun_out/ab3.log &&
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q -W ignore --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_ab.log; exit $rc
