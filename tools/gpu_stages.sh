#!/bin/bash
# GPU session stages (one gpurun call runs the listed ones in order; each GPU step under its own timeout):
#   test      pytest -m gpu + smoke()            bench    the default bench line (configs[1] + 1B x 32)
#   benchw    WORKLOADS="..." bench lines         lm       configs[0] LM timeline + rocprof
#   sweep     mid-width sweep (+ rocprof)        cap      full-size configs[3] Gram capture
#   rehearse8 8 ranks over gloo on one GPU        pmcab    PMC of one workload under PMCAB_LIBS
#   abbit     bitwise pass hash + time over ABBIT_LIBS
# usage: bash tools/gpu_stages.sh test,bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STAGES=${1:-cap,test,bench}
if [[ ,$STAGES, == *,cap,* ]]; then
  timeout -k 10 300 python -u tools/gram_split_capture.py > gpurun_out/cap.log 2>&1 || { echo "capture failed"; tail -20 gpurun_out/cap.log; exit 1; }
  tail -3 gpurun_out/cap.log
fi
if [[ ,$STAGES, == *,test,* ]]; then
  timeout -k 10 1000 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -rA --timeout 300 --timeout-method thread -W ignore > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [[ ,$STAGES, == *,sweep,* ]]; then  # mid-width sweep (tools/midp_sweep.py), then the same under rocprofv3
  timeout -k 10 400 python tools/midp_sweep.py ${SWEEP_P:-} > gpurun_out/midp_sweep.log 2>&1 || { echo "sweep failed"; tail gpurun_out/midp_sweep.log; exit 1; }
  cat gpurun_out/midp_sweep.log
  export TMPDIR=/tmp
  SWEEP_PASSES=3 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_midp" -o midp --output-format csv -- python tools/midp_sweep.py ${SWEEP_P:-} > gpurun_out/prof_midp.log 2>&1 || { echo "sweep prof failed"; tail gpurun_out/prof_midp.log; exit 1; }
fi
if [[ ,$STAGES, == *,benchw,* ]]; then  # the other workloads' bench lines (WORKLOADS env: space-separated)
  for w in ${WORKLOADS:-poisson64}; do
    timeout -k 10 600 python bench.py --workload $w --steps 10 --warmup 2 --no-cpu-baseline --no-load > gpurun_out/bench_$w.json 2> gpurun_out/bench_$w.err || { echo "bench $w failed"; tail -20 gpurun_out/bench_$w.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/bench_$w.json')); r=d['roofline']; print('$w', d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['time_to_converge_s'], d['iters_to_converge'])"
  done
fi
if [[ ,$STAGES, == *,lm,* ]]; then  # configs[0] host overhead: wall per fit, then the kernel / copy timeline
  timeout -k 10 300 python tools/lm_timeline.py 300 > gpurun_out/lm_timeline.log 2>&1 || { echo "lm timeline failed"; tail gpurun_out/lm_timeline.log; exit 1; }
  cat gpurun_out/lm_timeline.log
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_lm" -o lm --output-format csv -- python tools/lm_timeline.py 100 > gpurun_out/prof_lm.log 2>&1 || { echo "lm prof failed"; tail gpurun_out/prof_lm.log; exit 1; }
fi
if [[ ,$STAGES, == *,rehearse8,* ]]; then  # 8 ranks sharing this GPU over gloo (the 8-GPU launch path)
  timeout -k 10 900 python bench.py --gpus 8 --rows 10000000 --steps 3 --warmup 1 --no-load > gpurun_out/bench_gpus8.json 2> gpurun_out/bench_gpus8.err || { echo "rehearsal failed"; tail -20 gpurun_out/bench_gpus8.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_gpus8.json')); s=d['strong_scaling_1b_logit']; print('gpus8', d['n_gpus'], d['ms_per_step'], d['iters_to_converge'], s['n_gpus'], s['iters_to_converge'], repr(s['deviance']))"
fi
if [[ ,$STAGES, == *,bench,* ]]; then
  timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench.json')); r=d['roofline']; s=d.get('strong_scaling_1b_logit') or {}; print(d['ms_per_step'], r['kernel'], r['kernel_ms'], r['frac'], d['time_to_converge_s'], s.get('ms_per_iter'), s.get('time_to_converge_s'))"
fi
if [[ ,$STAGES, == *,pmcab,* ]]; then  # PMC of one workload (PMCAB_WL name:PN:PP:PKIND:PF:PL) under each library of PMCAB_LIBS
  export TMPDIR=/tmp
  IFS=: read -r name PN PP PKIND PF PL <<< "${PMCAB_WL:-poisson64:50000000:64:2:poisson:log}"
  export PN PP PKIND PF PL PK=2
  mkdir -p gpurun_out/pmcab
  for spec in ${PMCAB_LIBS:-sparkglm_amd/lib/libsglm_hip.so}; do
    lib=${spec%%@*}; tag=$(basename $(dirname $lib)); extra=""; [[ $spec == *@* ]] && extra=${spec#*@}
    for grp in "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_COEXEC_CYCLES"; do
      g=$(echo $grp | cut -c1-4); d="gpurun_out/pmcab/${name}_${tag}_$(echo $grp | md5sum | cut -c1-6)"
      env SGLM_LIB=$lib $extra timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/$d" -o run --output-format csv -- python tools/pass_bench.py > "$d.log" 2>&1 || { echo "pmcab $tag failed"; tail -5 "$d.log"; exit 1; }
    done
    echo "== $tag"; python tools/pmc_sum.py gpurun_out/pmcab/${name}_${tag}_* --kernel irls_narrow --json > gpurun_out/pmcab/${name}_${tag}.json; python - "$name" "$tag" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/pmcab/{sys.argv[1]}_{sys.argv[2]}.json"))
for k, e in d.items():
    clk = e["GRBM_GUI_ACTIVE"] / 8 / (e["avg_ms"] * 1e-3) / 1e9 if e.get("avg_ms") else 0
    print(k[-60:], f"ms {e['avg_ms']:.3f} clk {clk:.2f}GHz valu/mfma {e['SQ_INSTS_VALU']/max(e['SQ_INSTS_MFMA'],1):.2f} "
          f"mfma_busy {e['SQ_VALU_MFMA_BUSY_CYCLES']/(1024*clk*1e9*e['avg_ms']*1e-3):.3f} "
          f"wait {e['SQ_WAIT_ANY']/e['SQ_WAVE_CYCLES']:.3f} waitinst {e['SQ_WAIT_INST_ANY']/e['SQ_WAVE_CYCLES']:.3f} "
          f"active {e['SQ_ACTIVE_INST_ANY']/e['SQ_WAVE_CYCLES']:.3f} valu_act {e['SQ_ACTIVE_INST_VALU']/e['SQ_WAVE_CYCLES']:.3f} "
          f"lds_inst {e['SQ_INSTS_LDS']:.3g} salu {e['SQ_INSTS_SALU']:.3g} coexec {e['SQ_VALU_MFMA_COEXEC_CYCLES']:.3g}")
PY
  done
fi
if [[ ,$STAGES, == *,abbit,* ]]; then  # bitwise pass hash + pass time (tools/ab_k1r.py) over ABBIT_LIBS for each ABBIT_CASES n:p:kind:fam:link
  export AB_LIBS=${ABBIT_LIBS} AB_REPS=${AB_REPS:-2}
  for spec in ${ABBIT_CASES:-200000000:32:0:binomial:logit}; do
    IFS=: read AN AP AK AF AL <<< "$spec"
    AN=$AN AP=$AP AK=$AK AF=$AF AL=$AL timeout -k 10 300 python tools/ab_k1r.py >> gpurun_out/abbit.log 2>&1 || { echo "abbit failed"; tail gpurun_out/abbit.log; exit 1; }
  done
  cat gpurun_out/abbit.log
fi
