#!/bin/bash
# The split-role pass K1r generalised to P16 = 6..14 (SGLM_FUSED_SPLIT=6: K1r from P16 = 6 up):
# oracle-parity GPU tests with it, then the mid-width sweep K1 (default) vs K1r.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
SGLM_FUSED_SPLIT=6 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_initpass.py tests/test_gpu_speculate.py tests/test_gpu_fused_split.py -m gpu -v --timeout 300 --timeout-method thread -W ignore > gpurun_out/r03k_pytest.log 2>&1 || { echo "tests failed"; grep -E "FAILED|Error|error" gpurun_out/r03k_pytest.log | head -20; tail -3 gpurun_out/r03k_pytest.log; exit 1; }
tail -1 gpurun_out/r03k_pytest.log
L=sparkglm_amd/lib/libsglm_hip.so
for p in 80 96 128 160 192 224; do
  n=$(( 24000000000 / (p * 8) ))
  AB_LIBS=$L,$L@SGLM_FUSED_SPLIT=6 AN=$n AP=$p AB_REPS=2 timeout -k 10 300 python tools/ab_k1r.py || exit 1
done
exit 0
