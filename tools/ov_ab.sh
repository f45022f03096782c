#!/bin/bash
# A/B of the overlapped wide pass (SGLM_WIDE_OVERLAP chunks; SGLM_WIDE_OV_SERIAL=1 keeps the
# chunking but serialises the row kernels; lib_ab/nt: non-temporal X loads in the row kernel).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # label env... -- workload
  local lab=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload $WL --steps 5 --warmup 1 --no-cpu-baseline --no-load > gpurun_out/ovab_$lab.json 2> gpurun_out/ovab_$lab.err || { echo "bench $lab failed"; tail -20 gpurun_out/ovab_$lab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ovab_$lab.json')); b=d['breakdown_ms_per_step']; r=d['roofline']; print('$lab', round(d['ms_per_step'],2), 'pass', round(b['pass_kernels'],2), 'gram', round(r['kernel_ms'],2), 'rows', round(b['row_kernel'],2), 'frac', round(r['frac'],4))"
}
for WL in logit512r gamma2048; do
  run ${WL}_ov1 SGLM_WIDE_OVERLAP=1 || exit 1
  run ${WL}_ov8 SGLM_WIDE_OVERLAP=8 || exit 1
  run ${WL}_ov8serial SGLM_WIDE_OVERLAP=8 SGLM_WIDE_OV_SERIAL=1 || exit 1
  run ${WL}_ov8nt SGLM_WIDE_OVERLAP=8 SGLM_LIB=$GRAFT_REPO_ROOT/sparkglm_amd/lib_ab/nt/libsglm_hip.so || exit 1
  run ${WL}_ov16 SGLM_WIDE_OVERLAP=16 || exit 1
done
