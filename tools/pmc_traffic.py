"""HBM bytes per row, clock and MFMA busy of each PMC workload (tools/pmc_workloads.sh output)
-> the profiles/pmc_traffic.json entries bench.py reads for roofline.traffic.

Method (MI355X_MICROARCH.md, HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE in separate
--pmc passes; FETCH_SIZE doubled (gfx950 reports half of a 16-B/lane streaming read); KB x 1024;
summed over the pass's kernels (narrow / fused: one kernel; wide: row + Gram kernels), per row.
clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES /
(1024 SIMDs x clock cycles).
usage: python tools/pmc_traffic.py gpurun_out/pmc SOURCE_LABEL [profiles/pmc_traffic.json]"""
import json
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
WIDE = ["wide_rows_kernel", "wide_rows_ov_kernel", "wide_gram_kernel", "proc_gen_kernel"]
WL = {  # name: (key, rows, kernel substrings of the pass, substring of the kernel dispatched once per pass)
    "logit32": ("binomial:32", 100_000_000, ["irls_narrow_kernel"], "irls_narrow_kernel"),
    "poisson64": ("poisson:64", 50_000_000, ["irls_narrow_kernel"], "irls_narrow_kernel"),
    "logit256": ("binomial:256", 20_000_000, ["irls_pass_kernel", "irls_pass_r_kernel"], "irls_pass"),
    "logit512": ("binomial:512", 8_000_000, WIDE, "wide_rows_kernel<"),
    "logit512p": ("binomial:512:proc", 8_000_000, WIDE, "wide_rows_kernel<"),
    "lm20": ("gaussian:20:lm", 1_000_000, ["irls_narrow_kernel"], "irls_narrow_kernel"),
    "gamma2048": ("gamma:2048", 2_000_000, WIDE, "wide_rows_kernel<"),
    "mid160": ("binomial:160", 10_000_000, ["irls_pass_kernel", "irls_pass_r_kernel"], "irls_pass"),
    "mid96": ("binomial:96", 15_000_000, ["irls_pass_kernel", "irls_pass_r_kernel"], "irls_pass"),
}


def load(d, wl):
    out = subprocess.run([sys.executable, os.path.join(HERE, "pmc_sum.py")] +
                         [os.path.join(d, f"{wl}_{i}") for i in (1, 2, 3, 4) if os.path.isdir(os.path.join(d, f"{wl}_{i}"))] +
                         ["--kernel", "sglm", "--json"],
                         capture_output=True, text=True, check=True).stdout
    return json.loads(out)


def main():
    d, label = sys.argv[1], sys.argv[2]
    path = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(HERE), "profiles", "pmc_traffic.json")
    tab = json.load(open(path)) if os.path.exists(path) else {}
    for wl, (key, rows, subs, per_pass) in WL.items():
        if not os.path.isdir(os.path.join(d, f"{wl}_1")):
            continue
        ks = {k: v for k, v in load(d, wl).items() if any(s in k for s in subs)}
        # totals over every dispatch (per-dispatch averages x dispatches), per pass: a pass is one
        # dispatch of its pass-defining kernel (the fused / narrow kernel; a wide pass's chunk-0 row
        # kernel) -- chunked wide passes dispatch the Gram kernels once per chunk
        npass = sum(v.get("dispatches", 1) for k, v in ks.items() if per_pass in k) or 1
        tot = lambda c: sum((v.get(c) or 0) * v.get("dispatches", 1) for v in ks.values()) / npass
        fetch = tot("FETCH_SIZE") * 2 * 1024
        write = tot("WRITE_SIZE") * 1024
        ms = tot("avg_ms")
        grbm = tot("GRBM_GUI_ACTIVE")
        mfma = tot("SQ_VALU_MFMA_BUSY_CYCLES")
        cyc = grbm / 8
        entry = {"bytes_per_row": (fetch + write) / rows, "measured_rows": rows, "kernels": sorted(ks),
                 "fetch_bytes_per_row": fetch / rows, "write_bytes_per_row": write / rows,
                 "kernel_ms_profiled": ms, "clock_ghz": cyc / (ms * 1e-3) / 1e9 if ms else None,
                 "mfma_busy_frac": mfma / (1024 * cyc) if cyc else None, "source": label,
                 "method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE / GRBM_GUI_ACTIVE+SQ_VALU_MFMA_BUSY_CYCLES "
                           "in separate passes over tools/pass_bench.py (tools/pmc_workloads.sh); FETCH_SIZE doubled "
                           "(gfx950 reports half of a 16-B/lane streaming read, MI355X_MICROARCH.md); KB x 1024; summed "
                           "over every dispatch of the pass's kernels, per pass; clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time; MFMA busy = "
                           "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x clock cycles)"}
        if any("SQ_INSTS_VALU_MFMA_F64" in v for v in ks.values()):
            # group 4 (the fp64 pipe's instruction mix): wave-level instruction counts per row.  The
            # pipe-bound time bench.py derives from them: MFMA f64 16x16x4 = 64 cycles, fp64 VALU
            # add / mul / fma = 4 cycles (16 lanes per cycle: the 78.6 TF/s vector rate), fp64
            # transcendental = 16 cycles, over 1024 SIMDs at the PMC clock
            entry["fp64_mfma_insts_per_row"] = tot("SQ_INSTS_VALU_MFMA_F64") / rows
            entry["fp64_valu_insts_per_row"] = sum(tot(c) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                                                     "SQ_INSTS_VALU_FMA_F64")) / rows
            entry["fp64_trans_insts_per_row"] = tot("SQ_INSTS_VALU_TRANS_F64") / rows
            entry["valu_insts_per_row"] = tot("SQ_INSTS_VALU") / rows
            entry["method"] += ("; fp64 pipe mix (group 4): SQ_INSTS_VALU_MFMA_F64, SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 "
                                "per row")
        if key in tab:
            prev = tab[key]
            entry["previous"] = {k: prev.get(k) for k in ("bytes_per_row", "clock_ghz", "mfma_busy_frac", "source")}
        tab[key] = entry
        mix = (f"  fp64: mfma {entry['fp64_mfma_insts_per_row']:.3f} valu {entry['fp64_valu_insts_per_row']:.2f} "
               f"trans {entry['fp64_trans_insts_per_row']:.3f} /row") if "fp64_mfma_insts_per_row" in entry else ""
        print(f"{key:20s} {entry['bytes_per_row']:9.1f} B/row (fetch {entry['fetch_bytes_per_row']:.1f}, write "
              f"{entry['write_bytes_per_row']:.1f})  clock {entry['clock_ghz']:.2f} GHz  MFMA busy {entry['mfma_busy_frac']:.3f}{mix}")
    json.dump(tab, open(path, "w"), indent=1)


if __name__ == "__main__":
    main()
