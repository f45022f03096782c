#!/bin/bash
# Same-box A/B of the headline bench line (configs[1], 100M x 256) across library builds / env
# settings: AB_SPECS="lib@VAR=val ..." (lib relative to the repo root); prints ms/step, pass
# kernel ms and the MFMA fraction per run, alternating REPS times.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in $(seq 1 ${REPS:-2}); do
  for spec in $AB_SPECS; do
    lib=${spec%%@*}; kv=""; [[ $spec == *@* ]] && kv=${spec#*@}
    env SGLM_LIB=$lib ${kv//,/ } timeout -k 10 300 python bench.py --steps ${STEPS:-6} --warmup 2 --no-cpu-baseline --no-load --no-strong --no-configs ${BENCH_ARGS} > gpurun_out/abb.json 2> gpurun_out/abb.err || { tail -5 gpurun_out/abb.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/abb.json'));r=d['roofline'];print('$spec', '%.2f'%d['ms_per_step'], '%.2f'%r['kernel_ms'], '%.4f'%r['frac'], '%.3f'%d['time_to_converge_s'], d['iters_to_converge'], d.get('deviance'))"
  done
done
