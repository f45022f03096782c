#!/bin/bash
# Round-end rehearsal: the GPU suite + smoke, the default bench line (headline, 1B x 32 strong point,
# configs_n1), then the same default run under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_stages.sh test,bench || exit 1
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_default" -o run --output-format csv -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-load > gpurun_out/prof_default.json 2> gpurun_out/prof_default.err || { echo "prof failed"; tail -20 gpurun_out/prof_default.err; exit 1; }
echo prof ok
