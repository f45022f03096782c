#!/bin/bash
# Wave-cycle breakdown per pass kernel (MI355X_MICROARCH.md, rocprofv3 PMC slots): parked on
# s_waitcnt / barrier (SQ_WAIT_ANY), issue-stalled (SQ_WAIT_INST_ANY, of which LDS issue
# SQ_WAIT_INST_LDS), issuing (SQ_ACTIVE_INST_ANY), LDS bank conflicts, vector + matrix co-execution.
# One --pmc pass per workload over tools/pass_bench.py; WLS selects (name:PN:PP:PKIND:PF:PL).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/stalls
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES"
for spec in ${WLS:-logit32:100000000:32:0:binomial:logit poisson64:50000000:64:2:poisson:log mid96:15000000:96:0:binomial:logit mid160:10000000:160:0:binomial:logit logit256:20000000:256:0:binomial:logit}; do
  IFS=: read -r name PN PP PKIND PF PL <<< "$spec"
  export PN PP PKIND PF PL PK=2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$GRAFT_REPO_ROOT/gpurun_out/stalls/$name" -o run --output-format csv -- python tools/pass_bench.py > "gpurun_out/stalls/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc"
  if [[ $rc -ne 0 ]]; then tail -5 "gpurun_out/stalls/$name.log"; exit $rc; fi
done
exit 0
