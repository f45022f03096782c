#!/bin/bash
# One rocprofv3 --pmc pass per counter group over tools/pass_bench.py (env PN PP PKIND PF PL).
# Usage: pmc_counters.sh OUTNAME "C1 C2 ..." ["C3 C4" ...]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
name=$1; shift
mkdir -p gpurun_out/pmc
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmc/${name}_$i" -o run --output-format csv -- python tools/pass_bench.py > "gpurun_out/pmc/${name}_$i.log" 2>&1
  rc=$?
  echo "$name group $i ($grp) rc=$rc"
  if [[ $rc -ne 0 ]]; then tail -5 "gpurun_out/pmc/${name}_$i.log"; exit $rc; fi
done
exit 0
