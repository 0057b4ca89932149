"""The weight-stationary GEMM issues its MFMAs by inline asm (so that weights
are read straight from AGPRs, csrc/gemm_x6.hip).  hipcc pads no wait states
around inline asm: if the compiler ever placed one of its own instructions
that reads or writes an MFMA accumulator (a register copy, a store, an add)
too soon after the asm MFMA that writes it, the instruction would see a stale
value (the XDL write -> VALU / VMEM access hazard).  This CPU test compiles
the kernel to gfx950 assembly and checks every such access: between the asm
MFMA that last wrote a register and any non-MFMA-asm access to it there must
be at least WAIT independent wait states (one per instruction, s_nop N counts
N + 1).  The other direction is checked too (advisor r04): a compiler VALU
write (v_mov, v_accvgpr_write, ...) of a register that a later asm MFMA reads
as its A, B or C operand needs VALU_WAIT wait states before that MFMA, which
the compiler cannot pad either, since it does not see the MFMA inside the
asm statement."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "drone_rl_amd", "csrc", "gemm_x6.hip")
# the weight-stationary GEMM and (round 5) its first-layer-backward form
# the weight-stationary forward and its first-layer-backward form (round 6:
# both on v_mfma_f32_16x16x32_bf16)
KERNELS = ("gemm_x6_ws16_kernel", "gemm_x6_fl16_kernel")
# XDL write VGPR -> VALU, VMEM or LDS access of it: 11 wait states for an
# 8-pass XDL op on gfx940-class parts (v_mfma_f32_16x16x32_bf16 has fewer
# passes); checked with margin
WAIT = 18
# VALU (or v_accvgpr_write) write of a VGPR / AGPR -> an MFMA reading it as
# SrcA / SrcB / SrcC: 2 wait states on gfx940-class parts (the CDNA3/4 ISA
# manual's required-NOPs table); checked with margin
VALU_WAIT = 4

_VREG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")
_AREG = re.compile(r"\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def _regs(text, pat=_VREG, tag=""):
    out = set()
    for m in pat.finditer(text):
        if m.group(1) is not None:
            out.update(tag + str(r) if tag else r for r in range(int(m.group(1)),
                                                                 int(m.group(2)) + 1))
        else:
            out.add(tag + m.group(3) if tag else int(m.group(3)))
    return out


def _any_regs(text):
    """VGPRs as 'v<n>' and AGPRs as 'a<n>'."""
    return _regs(text, _VREG, "v") | _regs(text, _AREG, "a")


_ASM = {}


def _kernel_asm(kernel):
    if "s" not in _ASM:
        _ASM["s"] = _compile()
    s = _ASM["s"]
    name = next(l.split(":")[0] for l in s.splitlines()
                if kernel in l.split(":")[0] and re.match(r"^[_A-Za-z0-9]+:", l))
    a = s.index(name + ":")
    b = s.index(".Lfunc_end", a)
    return s[a:b].splitlines()


def _compile():
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    with tempfile.TemporaryDirectory() as d:
        asm = os.path.join(d, "gemm_x6.s")
        out = subprocess.run(
            [hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
             "-fno-fast-math", "-fno-slp-vectorize", "-I", os.path.join(ROOT, "include"),
             "--cuda-device-only", "-S", SRC, "-o", asm],
            capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        return open(asm).read()


def _scan(lines):
    """(number of asm MFMAs, list of violations) for an assembly listing."""
    pending = {}           # register -> wait states elapsed since its MFMA write
    written = {}           # register -> wait states since a compiler VALU wrote it
    in_asm = False
    n_mfma = 0
    bad = []
    for i, raw in enumerate(lines):
        l = raw.strip() if raw.strip().startswith(";;#") else raw.split(";")[0].strip()
        if l.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if l.startswith(";;#ASMEND"):
            in_asm = False
            continue
        if not l or l.startswith(".") or l.endswith(":"):
            continue
        op = l.split()[0]
        if in_asm and op.startswith("v_mfma"):
            n_mfma += 1
            ops = l[len(op):].split(",")
            for r in sorted(_any_regs(",".join(ops[1:])) & set(written)):
                if written[r] < VALU_WAIT:
                    bad.append(f"line {i}: asm '{l}' reads {r} {written[r]} wait states after "
                               f"a compiler VALU wrote it")
            dst = _regs(ops[0])
            for r in list(pending):
                pending[r] += 1
            for r in dst:
                pending[r] = 0
            for r in list(written):
                written[r] += 1
                if written[r] >= VALU_WAIT:
                    del written[r]
            continue
        step = int(l.split()[1]) + 1 if op == "s_nop" else 1
        if not in_asm:
            for r in _regs(l[len(op):]) & set(pending):
                if pending[r] < WAIT:
                    bad.append(f"line {i}: '{l}' touches v{r} {pending[r]} wait states after "
                               f"its asm MFMA write")
        for r in list(pending):
            pending[r] += step
            if pending[r] >= WAIT:
                del pending[r]
        for r in list(written):
            written[r] += step
            if written[r] >= VALU_WAIT:
                del written[r]
        if not in_asm and op.startswith("v_") and not op.startswith(("v_cmp", "v_readlane",
                                                                      "v_readfirstlane")):
            for r in _any_regs(l[len(op):].split(",")[0]):
                written[r] = 0
    return n_mfma, bad


def test_scanner_flags_a_copy_right_after_an_asm_mfma():
    """The pattern that once corrupted a variant of this kernel: the compiler
    copying an accumulator (v_mov) right after the asm MFMA group wrote it."""
    lines = """\
\t;;#ASMSTART
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[178:181], a[76:79], v[0:15]
\t;;#ASMEND
\tv_mov_b64_e32 v[30:31], v[14:15]
\ts_nop 7
\t;;#ASMSTART
\tv_mfma_f32_32x32x16_bf16 v[32:47], v[178:181], a[76:79], v[32:47]
\t;;#ASMEND
\ts_nop 7
\ts_nop 7
\ts_nop 7
\tv_add_f32_e32 v40, v40, v41
""".splitlines()
    n, bad = _scan(lines)
    assert n == 2 and len(bad) == 2 and "v14" in bad[0] and "v15" in bad[1]


def test_scanner_flags_an_operand_written_right_before_an_asm_mfma():
    """A compiler write of an MFMA source (here the A fragment v178 and the
    AGPR weight a77) with no wait states before the asm MFMA that reads it."""
    lines = """\
\tv_mov_b32_e32 v178, v3
\tv_accvgpr_write_b32 a77, v4
\t;;#ASMSTART
\tv_mfma_f32_32x32x16_bf16 v[0:15], v[178:181], a[76:79], v[0:15]
\t;;#ASMEND
\tv_mov_b32_e32 v200, v250
\ts_nop 4
\t;;#ASMSTART
\tv_mfma_f32_32x32x16_bf16 v[32:47], v[198:201], a[76:79], v[32:47]
\t;;#ASMEND
""".splitlines()
    n, bad = _scan(lines)
    assert n == 2 and len(bad) == 2, bad
    assert any("reads v178" in b for b in bad) and any("reads a77" in b for b in bad)


@pytest.mark.parametrize("kernel", KERNELS)
def test_no_compiler_access_to_asm_mfma_results_without_wait_states(kernel):
    n_mfma, bad = _scan(_kernel_asm(kernel))
    assert n_mfma >= 192, f"expected the kernel's asm MFMAs, found {n_mfma}"
    assert not bad, "\n".join(bad[:20])
