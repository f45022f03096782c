#!/bin/bash
# Round-4 GPU session: configs[3] Gram capture, the GPU suite, smoke, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STAGES=${1:-cap,test,bench}
if [[ ,$STAGES, == *,cap,* ]]; then
  timeout -k 10 300 python -u tools/gram_split_capture.py > gpurun_out/cap.log 2>&1 || { echo "capture failed"; tail -20 gpurun_out/cap.log; exit 1; }
  tail -3 gpurun_out/cap.log
fi
if [[ ,$STAGES, == *,test,* ]]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -W ignore > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [[ ,$STAGES, == *,bench,* ]]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']; s=d.get('strong_scaling_1b_logit') or {}; print(d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['time_to_converge_s'], s.get('ms_per_iter'), s.get('time_to_converge_s'))"
fi
