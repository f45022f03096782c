"""Register budgets the overlapped wide pass relies on (engine.cpp enqueue_pass, wide.hip): the
two persistent Gram workgroups of a CU and one overlapped row-kernel workgroup must fit one
SIMD's 512 VGPRs together, or the row kernel's workgroups take Gram slots and the chunk's Gram
runs in two rounds (measured: logit512r Gram 280 -> 320 ms when a change pushed the off-diagonal
kernel from 208 to 224 VGPRs).  Read from the gfx950 code object's metadata notes of the built
device object (build/obj/wide.o), so a CPU run catches a regression."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj", "wide.o")
LLVM = "/opt/rocm/lib/llvm/bin"


def _kernel_meta():
    if not os.path.exists(OBJ) or not os.path.exists(os.path.join(LLVM, "llvm-readelf")):
        pytest.skip("device object or LLVM tools absent (run __graft_entry__.build() first)")
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", OBJ, os.devnull],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True, capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    meta, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = meta.setdefault(m.group(1), {})
            continue
        m = re.match(r"\s+\.(vgpr_count|sgpr_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return meta


def _alloc(v):  # VGPRs are allocated in granules of 8
    return (v + 7) // 8 * 8


def test_overlap_register_budget():
    meta = _kernel_meta()
    off = meta["_ZN4sglm16wide_gram_kernelILb0ELb0EEEvNS_12WideGramArgsE"]
    diag = meta["_ZN4sglm16wide_gram_kernelILb1ELb0EEEvNS_12WideGramArgsE"]
    rows = {k: v for k, v in meta.items() if "wide_rows_ov_kernel" in k}
    assert len(rows) == 6  # one per family/link
    worst_row = max(_alloc(v["vgpr_count"]) for v in rows.values())
    assert all(v["private_segment_fixed_size"] == 0 for v in rows.values())  # no spills
    assert worst_row <= 96
    for gram in (off, diag):
        assert gram["private_segment_fixed_size"] == 0
        assert 2 * _alloc(gram["vgpr_count"]) + worst_row <= 512, (gram, worst_row)


def test_lean_generator_fits_two_waves_beside_the_gram():
    # proc_gen_kernel (SGLM_PROC_LEAN) runs beside the off-diagonal launch: two of its waves and the
    # two Gram waves of a SIMD must fit the 512 VGPRs together; both design kinds (POS = true: the
    # positive gamma design of kind 3) run there
    meta = _kernel_meta()
    off = meta["_ZN4sglm16wide_gram_kernelILb0ELb0EEEvNS_12WideGramArgsE"]
    for pos in (0, 1):
        gen = meta[f"_ZN4sglm15proc_gen_kernelILb{pos}EEEvNS_11ProcGenArgsEPKdPd"]
        assert gen["private_segment_fixed_size"] == 0
        assert 2 * _alloc(off["vgpr_count"]) + 2 * _alloc(gen["vgpr_count"]) <= 512, (pos, off, gen)
