#!/bin/bash
# Phase timelines of the narrow pass (diagnostic -DSGLM_STAMPS builds in sparkglm_amd/lib_ab/):
# per wave of workgroup 0, the mean cycles of each phase over 16 steady-state blocks.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in ${STAMP_LIBS:-stamps0 stamps1}; do
  for cfg in "200000000 32 0 binomial logit" "60000000 64 2 poisson log"; do
    set -- $cfg
    echo "== $v n=$1 p=$2 $4/$5"
    SGLM_LIB=sparkglm_amd/lib_ab/$v.so NARROW=1 AN=$1 AP=$2 AK=$3 AF=$4 AL=$5 timeout -k 10 120 python tools/stamps.py || exit 1
  done
done
