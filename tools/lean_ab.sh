#!/bin/bash
# Same-box A/B: narrow logit passes with in-pass statistics on every pass (SGLM_SPECULATE=0) vs
# only where a fit ends (default).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2 3; do
  for sp in 0 1; do
    echo -n "spec=$sp "; SGLM_SPECULATE=$sp AB_REPS=1 AN=200000000 AP=32 AK=0 AF=binomial AL=logit timeout -k 10 300 python tools/ab.py || exit 1
  done
done
