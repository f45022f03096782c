#!/bin/bash
# A/B: Gram kernel issue priority (lib_ab/prio2) under the overlapped row kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/ovab2_$lab.json 2> gpurun_out/ovab2_$lab.err || { echo "bench $lab failed"; tail -20 gpurun_out/ovab2_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ovab2_$lab.json')); b=d['breakdown_ms_per_step']; r=d['roofline']; print('$lab', round(d['ms_per_step'],2), 'pass', round(b['pass_kernels'],2), 'gram', round(r['kernel_ms'],2), 'rows', round(b['row_kernel'],2), 'frac', round(r['frac'],4))"
}
for WL in logit512r gamma2048; do
  run ${WL}_base || exit 1
  for v in prio2 prio2off prio2diag prio1; do
    run ${WL}_$v SGLM_LIB=$GRAFT_REPO_ROOT/sparkglm_amd/lib_ab/$v/libsglm_hip.so || exit 1
  done
  run ${WL}_prio2_serial SGLM_WIDE_OV_SERIAL=1 SGLM_LIB=$GRAFT_REPO_ROOT/sparkglm_amd/lib_ab/prio2/libsglm_hip.so || exit 1
done
