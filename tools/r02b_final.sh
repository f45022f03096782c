#!/bin/bash
# Final checks of the session: GPU tests + smoke, then the 2-rank launcher rehearsal on one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_round.sh test || exit 1
timeout -k 10 600 python bench.py --gpus 2 --rows 10000000 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02b_gpus2.json 2> gpurun_out/r02b_gpus2.err || { echo "gpus2 failed"; tail -20 gpurun_out/r02b_gpus2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r02b_gpus2.json')); print(d['n_gpus'], d['config']['parallelism'], d['value'], d['strong_scaling_1b_logit'])"
