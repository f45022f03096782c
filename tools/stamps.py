"""Phase timeline of the fused pass (diagnostic build with -DSGLM_STAMPS, see kernels.hip):
per wave of workgroup 0, the mean cycles of each phase over 16 steady-state row blocks.
usage: SGLM_LIB=sparkglm_amd/lib_ab/stamps.so AN=20000000 AP=256 python tools/stamps.py"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sparkglm_amd import Engine, _lib  # noqa: E402

n, p = int(os.environ.get("AN", "20000000")), int(os.environ.get("AP", "256"))
narrow = os.environ.get("NARROW") == "1"
kind = int(os.environ.get("AK", "0"))
fam, lnk = os.environ.get("AF", "binomial"), os.environ.get("AL", "logit")
e = Engine(0)
e.synth(kind, 0, n, p, 2)
b = np.full(p, 0.01)
e.irls_pass(b, family=fam, link=lnk)
e.irls_pass(b, family=fam, link=lnk)
lib = _lib.load()
NWV = 8 if narrow else 12
buf = (C.c_ulonglong * (NWV * 16 * 8))()
assert (lib.sglm_debug_nstamps if narrow else lib.sglm_debug_stamps)(buf, NWV * 16 * 8) == 0
t = np.array(buf, dtype=np.float64).reshape(NWV, 16, 8)
if narrow:
    t = t[:, :, :5]
names = (["vmcnt", "row stage", "gram", "dma issue"] if narrow else
         os.environ.get("STAMP_NAMES", "gram 1st,vmcnt,flag,row stage,gram 2nd,barrier,dma issue").split(","))
t0 = t[:, :, 0][t[:, :, 0] > 0].min()
if not narrow:
    hw = (C.c_uint * 16)()
    assert lib.sglm_debug_hwid(hw, 16) == 0
    print("SIMD of each wave of workgroup 0:", [(h >> 4) & 3 for h in list(hw)[:NWV]])
print("wave  " + "  ".join(f"{s:>10s}" for s in names) + "   block total")
for w in range(NWV):
    if not t[w].any():
        continue
    d = np.diff(t[w], axis=1)  # [16][7]
    row = d.mean(axis=0)
    tot = np.diff(t[w, :, 0]).mean()
    print(f"{w:4d}  " + "  ".join(f"{v:10.0f}" for v in row) + f"   {tot:8.0f}")
