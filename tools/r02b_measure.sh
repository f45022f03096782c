#!/bin/bash
# Round-2 (second session) evidence: GPU tests + smoke, then bench + rocprof of the workloads the
# overlapped wide pass changes, then PMC HBM bytes with full-size chunk lengths.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh test || exit 1
PROF=1 WLS="logit512r gamma2048 logit512" bash tools/bench_all.sh > gpurun_out/r02b_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/r02b_bench.log; exit 1; }
grep -E "rc=" gpurun_out/r02b_bench.log
SGLM_WIDE_OVERLAP=3 WLS="gamma2048" bash tools/pmc_workloads.sh > gpurun_out/r02b_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r02b_pmc.log; exit 1; }
SGLM_WIDE_OVERLAP=2 WLS="logit512" bash tools/pmc_workloads.sh >> gpurun_out/r02b_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r02b_pmc.log; exit 1; }
python tools/pmc_traffic.py gpurun_out/pmc r02b_overlap gpurun_out/pmc_traffic_r02b.json | tail -3
