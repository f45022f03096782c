# A/B of the wide Gram schedule (SGLM_WIDE_BAND 0 = contiguous pieces, 1/2 = banded) on one GPU,
# then the wide-path GPU tests under the default schedule.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export AB_REPS=${AB_REPS:-2}
for b in 0 1 0 1; do
  echo "band=$b"; SGLM_WIDE_BAND=$b AN=20000000 AP=512 AK=0 AF=binomial AL=logit timeout -k 10 300 python tools/ab.py || exit 1
done 2>&1 | tee gpurun_out/ab_band1.log &&
for b in 0 2 0 2; do
  echo "band=$b"; SGLM_WIDE_BAND=$b AN=3000000 AP=2048 AK=3 AF=gamma AL=inverse timeout -k 10 300 python tools/ab.py || exit 1
done 2>&1 | tee gpurun_out/ab_band2.log &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py tests/test_gpu_configs.py -m gpu -x -q -W ignore --timeout 300 --timeout-method thread > gpurun_out/pytest_band.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_band.log; exit $rc
