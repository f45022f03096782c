#!/bin/bash
# Round-3 GPU-box validation: gpu tests (verbose log), smoke, default bench line.
# usage: tools/r03_gpu.sh [test|bench|all] [TAG]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STAGE=${1:-all}
TAG=${2:-r03}
if [[ $STAGE == all || $STAGE == test ]]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -W ignore \
    > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/${TAG}_pytest_gpu.log | head; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  cat gpurun_out/${TAG}_smoke.log
fi
if [[ $STAGE == all || $STAGE == bench ]]; then
  timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_bench.json
fi
if [[ $STAGE == all || $STAGE == gpus2 ]]; then
  # the --gpus 2 rehearsal on one GPU: two rank processes sharing the device over gloo
  timeout -k 10 600 python bench.py --gpus 2 --rows 10000000 --steps 5 --warmup 1 --no-cpu-baseline \
    > gpurun_out/${TAG}_gpus2.json 2> gpurun_out/${TAG}_gpus2.err || { echo "gpus2 failed"; tail -20 gpurun_out/${TAG}_gpus2.err; exit 1; }
  cat gpurun_out/${TAG}_gpus2.json
fi
