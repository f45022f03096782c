#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
L=sparkglm_amd/lib/libsglm_hip.so
for p in 80 96 128 160 192 224 240 256; do
  n=$(( 24000000000 / (p * 8) ))
  AB_LIBS=$L AN=$n AP=$p AB_REPS=1 timeout -k 10 200 python tools/ab_k1r.py || exit 1
done
exit 0
