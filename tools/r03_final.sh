#!/bin/bash
# Round-3 final evidence: the GPU suite + smoke, every bench workload with a rocprofv3
# --kernel-trace --stats summary of the same command (tools/bench_all.sh), the PMC passes of every
# workload shape (tools/pmc_workloads.sh), and the 2-rank rehearsal of bench.py --gpus 2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/r03_gpu.sh test r03f || exit 1
PROF=1 bash tools/bench_all.sh || exit 1
WLS="poisson64 logit256 logit512 gamma2048 logit32 logit512p" bash tools/pmc_workloads.sh || exit 1
bash tools/r03_gpu.sh gpus2 r03f || exit 1
exit 0
