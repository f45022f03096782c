"""Per-kernel gfx950 disassembly of the built device objects (build/obj/{kernels,fused_odd,narrow,wide}.o;
ISA_OBJDIR selects a variant build's objects).

    python tools/isa_dump.py OUTDIR            # one OUTDIR/<kernel>.s per kernel symbol
    python tools/isa_dump.py --diff DIR_A DIR_B

Used to show that a source change which should not alter the generated code (e.g. deleting
compile-time knobs at their default values) leaves every kernel's instructions identical.
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def dump(outdir: str) -> int:
    os.makedirs(outdir, exist_ok=True)
    count = 0
    objdir = os.environ.get("ISA_OBJDIR", os.path.join(ROOT, "build", "obj"))  # e.g. build/obj_<variant>
    for name in ("kernels", "fused_odd", "narrow", "wide"):
        obj = os.path.join(objdir, f"{name}.o")
        if not os.path.exists(obj):
            continue
        with tempfile.TemporaryDirectory() as d:
            fat, co = os.path.join(d, "fatbin"), os.path.join(d, "dev.co")
            subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", obj, os.devnull],
                           check=True, capture_output=True)
            subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fat}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                           capture_output=True)
            text = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn",
                                   "--no-leading-addr", co], check=True, capture_output=True, text=True).stdout
        cur, lines = None, []
        for line in text.splitlines():
            m = re.match(r"^(\S+):$", line.strip()) if line and not line.startswith((" ", "\t")) else None
            if m:
                if cur:
                    _write(outdir, cur, lines)
                    count += 1
                cur, lines = m.group(1), []
            elif cur and line.strip():
                # branch targets print as absolute addresses + symbol offsets: keep only the opcode/operands
                lines.append(re.sub(r"\s*//.*$", "", line.strip()))
        if cur:
            _write(outdir, cur, lines)
            count += 1
    return count


def _write(outdir, sym, lines):
    with open(os.path.join(outdir, sym[:200] + ".s"), "w") as fh:
        fh.write("\n".join(lines) + "\n")


def diff(a: str, b: str) -> int:
    fa, fb = set(os.listdir(a)), set(os.listdir(b))
    bad = 0
    for f in sorted(fa | fb):
        if f not in fa or f not in fb:
            print(f"only in {'B' if f not in fa else 'A'}: {f}")
            bad += 1
            continue
        if open(os.path.join(a, f)).read() != open(os.path.join(b, f)).read():
            print(f"differs: {f}")
            bad += 1
    print(f"{len(fa & fb)} common kernels, {bad} differences")
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "--diff":
        sys.exit(1 if diff(sys.argv[2], sys.argv[3]) else 0)
    print(f"{dump(sys.argv[1])} symbols")
