#!/bin/bash
# PMC passes over tools/pass_bench.py (one counter group per pass, kernel-trace only).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/$name" -o run --output-format csv -- python tools/pass_bench.py > "gpurun_out/pmc/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [[ $rc -ge 124 ]]; then exit $rc; fi
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run clock GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES
run waits SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
exit 0
