#!/bin/bash
# Round-3 third session: A/B of the K1r diagonal-tile builds, default bench (K1r), rocprof stats
# of the headline, PMC (clock / MFMA busy / HBM bytes) of the p = 256 pass; STAGE=test adds the
# GPU suite + smoke first.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [[ -n "$WITH_TESTS" ]]; then bash tools/r03_gpu.sh test r03c || exit 1; fi
bash tools/ab_d44.sh > gpurun_out/ab_d44.log 2>&1; rc=$?; cat gpurun_out/ab_d44.log; [[ $rc -ne 0 ]] && exit $rc
bash tools/r03_gpu.sh bench r03c || exit 1
WLS=logit256 PROF=1 bash tools/bench_all.sh || exit 1
WLS=logit256 bash tools/pmc_workloads.sh || exit 1
exit 0
