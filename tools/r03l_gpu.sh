#!/bin/bash
# Default K1r threshold P16 >= 10: the whole GPU suite + smoke, then the mid-width sweep (default vs K1).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/r03_gpu.sh test r03l || exit 1
L=sparkglm_amd/lib/libsglm_hip.so
for p in 160 192 224 256; do
  n=$(( 24000000000 / (p * 8) ))
  AB_LIBS=$L,$L@SGLM_FUSED_SPLIT=0 AN=$n AP=$p AB_REPS=1 timeout -k 10 300 python tools/ab_k1r.py || exit 1
done
exit 0
