"""Build-time check of the MFMA -> accumulator-read distance in the gfx950 code objects.

Several kernels issue their MFMAs through inline asm (the accumulators pinned in the
accumulator file: gemm.hip mfma_acc, flash.hip mfma_acc_a).  An asm MFMA is invisible to the
compiler's hazard recognizer, so nothing guarantees the wait states between it and an
instruction that reads its result -- a compiler-inserted v_accvgpr_read / v_accvgpr_mov copy on
a loop edge read one MFMA early in round 5 (silent wrong result).  This script disassembles every
object's gfx950 code and flags, per kernel, any instruction that reads an accumulator register
written by a v_mfma fewer than MIN_WAIT wait states earlier (an s_nop N counts N + 1, every other
instruction 1), except the MFMA accumulate chains on the same register range (srcC == vdst),
which need none.  Kernels with asm MFMAs (ASM_KERNELS) must keep MIN_WAIT = 18 wait states (the
16-pass XDL write -> read requirement plus margin); every other kernel is held to FLOOR = 8, the
smallest distance the compiler itself leaves after a builtin v_mfma_f32_16x16x32_bf16 in these
objects (a read closer than that would be a compiler or asm error too).

Usage: python check_hazards.py OBJ... (exit 1 on a finding).  Test infrastructure for the
build (called by __graft_entry__.build); no GPU needed.
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MIN_WAIT = 18
FLOOR = 8
ASM_KERNELS = ("gemm_w4b_kernel",)

_REG = re.compile(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def _aregs(text):
    out = set()
    for m in _REG.finditer(text):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def disassemble(obj):
    """gfx950 disassembly of a hipcc -c object (its .hip_fatbin bundle)."""
    with tempfile.TemporaryDirectory() as td:
        fb, co = os.path.join(td, "fb"), os.path.join(td, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb],
                       check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}",
                        f"--input={fb}", f"--output={co}", "--unbundle"], check=True)
        return subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                              check=True, capture_output=True, text=True).stdout


def check(text, min_wait=MIN_WAIT):
    """[(kernel, distance, mfma, reader)] for every accumulator read closer than min_wait."""
    findings = []
    func = None
    recent = []   # (wait states since, dst regs, dst text) of MFMAs in the window
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            func, recent = m.group(1), []
            continue
        ins = line.split("//")[0].strip()
        if not ins or func is None or ins.endswith(":"):
            continue
        op, _, rest = ins.partition(" ")
        if op.startswith("s_nop"):
            n = int(rest.strip(), 0) + 1 if rest.strip() else 1
            recent = [(w + n, d, t) for w, d, t in recent if w + n < min_wait]
            continue
        if op.startswith("s_branch") or op.startswith("s_cbranch") or op.startswith("s_setpc"):
            pass   # straight-line analysis; loop back edges are covered by the drains' own nops
        ops = [o.strip() for o in rest.split(",")]
        if op.startswith("v_mfma"):
            dst, srcs = ops[0], ops[1:]
            dregs = _aregs(dst)
            for w, d, t in recent:
                for k, s in enumerate(srcs):
                    r = _aregs(s)
                    if r & d and not (k == len(srcs) - 1 and s == t and dst == t):
                        findings.append((func, w, t, ins))
            # a later write of the same registers supersedes the earlier one (a chain's last MFMA
            # is the one its readers wait for)
            recent = [(w + 1, d, t) for w, d, t in recent if w + 1 < min_wait and not d <= dregs]
            if dregs:
                recent.append((0, dregs, dst))
            continue
        # any other instruction: its sources (all operands but a VALU / load destination)
        srcs = ops[1:] if (op.startswith("v_") or "load" in op or "read" in op) else ops
        for w, d, t in recent:
            if any(_aregs(s) & d for s in srcs):
                findings.append((func, w, t, ins))
        recent = [(w + 1, d, t) for w, d, t in recent if w + 1 < min_wait]
    return findings


def main(objs):
    bad = 0
    for obj in objs:
        f = [x for x in check(disassemble(obj), MIN_WAIT)
             if x[1] < FLOOR or any(k in x[0] for k in ASM_KERNELS)]
        for func, w, t, ins in f[:20]:
            print(f"{os.path.basename(obj)}: {func}: {ins!r} reads {t} {w} wait states after its MFMA")
        bad += len(f)
    print(f"check_hazards: {len(objs)} objects, {bad} accumulator reads inside an MFMA's window")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
