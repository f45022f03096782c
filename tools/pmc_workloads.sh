#!/bin/bash
# PMC evidence per bench workload: HBM bytes (FETCH_SIZE, WRITE_SIZE: separate passes) and
# clock / MFMA busy, over tools/pass_bench.py at a reduced row count (same per-row pattern).
cd "$GRAFT_REPO_ROOT" || exit 1
run_wl() {  # name PN PP PKIND PF PL [PPROC] [VAR=value: extra environment]
  local name=$1
  export PN=$2 PP=$3 PKIND=$4 PF=$5 PL=$6 PK=2 PPROC=${7:-0}
  # group 4: the fp64 pipe's instruction mix (MFMA + fp64 VALU), for fp64_pipe.pipe_bound_ms
  env ${8:-PMC_WL=$1} bash tools/pmc_counters.sh "$name" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
    "GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU" || exit 1
}
for wl in ${WLS:-poisson64 logit256 logit512 gamma2048 logit32}; do
  case $wl in
    poisson64) run_wl poisson64 50000000 64 2 poisson log ;;
    logit256) run_wl logit256 20000000 256 0 binomial logit ;;
    # wide: chunk lengths as in the bench shards (the banded Gram re-reads X per chunk): 4M-row
    # chunks ~ logit512r's 3.75M, 667K ~ gamma2048's 781K
    logit512) run_wl logit512 8000000 512 0 binomial logit 0 SGLM_WIDE_OVERLAP=2 ;;
    gamma2048) run_wl gamma2048 2000000 2048 3 gamma inverse 0 SGLM_WIDE_OVERLAP=3 ;;
    logit32) run_wl logit32 100000000 32 0 binomial logit ;;   # logit1b's per-row pattern
    mid160) run_wl mid160 10000000 160 0 binomial logit ;;     # mid-width K1r<10>
    mid96) run_wl mid96 15000000 96 0 binomial logit ;;        # mid-width K1<6>, three workgroups per CU
    logit512p) run_wl logit512p 8000000 512 0 binomial logit 1 ;;  # procedural shard (HBM-scratch chunks)
    lm20) run_wl lm20 1000000 20 1 gaussian identity 0 PLM=1 ;;       # configs[0]: the one-pass LM Gram
  esac
done
exit 0
