"""Wait-state hazards between inline asm and compiler code in the bf16
kernels (CPU only: static check of the gfx950 ISA from tests/isa_util.py).

hipcc pads the hazards between instructions it generates; it pads nothing
inside an `asm volatile` string and sees no instruction in it, so every pair
whose producer or consumer sits in inline asm is the kernel author's to pad
(cdna_hip_programming.md, "Insert its wait states").  The kernels issue their
MFMAs, query-fragment loads and LDS-DMA from asm, so this walks each kernel's
instruction stream in layout order, counting wait states (1 per instruction,
N + 1 per `s_nop N`), and checks the pairs the kernels can form:

  A. a VALU write of a VGPR/AGPR -> an asm MFMA reading it (A, B or C):
     >= 2 states;
  B. an MFMA's result -> any other access of those registers, except the
     next MFMA of the same accumulation chain (D taken whole as C), where
     either side is asm: >= passes + 4 states (32x32x16: 8 passes, 12
     states; 16x16x32: 4 passes, 8 states);
  C. a VALU write of an SGPR (v_readfirstlane, v_readlane, v_cmp ... e64)
     -> an asm memory instruction reading it as descriptor / offset / base:
     >= 5 states;
  D. an SALU write of M0 -> an asm LDS-DMA: >= 1 state.

Layout order follows fall-through paths only: a pair joined by a taken
branch is not seen.  The kernels keep every asm MFMA stream and its padding
in straight-line code, so the pairs that matter are in reach.
"""
import re

import pytest

from isa_util import all_isa, have_hipcc

_REG = re.compile(r"\b([vas])(?:(\d+)|\[(\d+):(\d+)\])")
_PASSES = {"v_mfma_f32_32x32x16_bf16": 8, "v_mfma_f32_16x16x32_bf16": 4,
           "v_mfma_f32_32x32x2_f32": 16, "v_mfma_f32_16x16x4_f32": 8}
_MEM = ("buffer_", "global_", "scratch_", "flat_")


def regs(op):
    """The register set an operand names: {('v', 3), ('s', 4), ...}; m0 as ('m', 0)."""
    op = op.strip()
    if op == "m0":
        return {("m", 0)}
    if op in ("vcc", "vcc_lo"):
        return {("s", "vcc")}
    m = _REG.fullmatch(op)
    if not m:
        return set()
    kind = m.group(1)
    if m.group(2) is not None:
        return {(kind, int(m.group(2)))}
    return {(kind, i) for i in range(int(m.group(3)), int(m.group(4)) + 1)}


class Ins:
    __slots__ = ("op", "args", "asm", "line", "states")

    def __init__(self, op, args, asm, line):
        self.op, self.args, self.asm, self.line = op, args, asm, line
        self.states = int(args[0]) + 1 if op == "s_nop" else 1

    def dst(self):
        """Registers written by the instruction's own pipeline (memory loads,
        which complete under a counter, are not wait-state producers)."""
        if not self.args:
            return set()
        if self.op.startswith("v_cmpx"):
            return set()
        if self.op.startswith("v_cmp"):
            return regs(self.args[0]) if self.op.endswith("_e64") else {("s", "vcc")}
        if self.op.startswith("v_") or self.op.startswith("s_"):
            if self.op.startswith(("s_cmp", "s_cbranch", "s_branch", "s_waitcnt", "s_barrier", "s_nop",
                                   "s_endpgm", "s_set", "s_sleep", "s_bitcmp")):
                return set()
            return regs(self.args[0])
        return set()

    def uses(self):
        out = set()
        for a in self.args:
            out |= regs(a)
        return out

    def srcs(self):
        if self.op.startswith(("buffer_store", "global_store", "ds_write", "scratch_store", "flat_store")) or \
                self.op.startswith(("s_cmp", "s_bitcmp")):
            first = 0
        else:
            first = 1
        out = set()
        for a in self.args[first:]:
            out |= regs(a)
        return out

    def is_mfma(self):
        return self.op.startswith("v_mfma")

    def is_valu(self):
        return self.op.startswith("v_") and not self.is_mfma()


def kernels(asm_text):
    """{kernel name: [Ins]} in layout order."""
    out, cur, name, inasm = {}, None, None, False
    for raw in asm_text.splitlines():
        if re.match(r"^_Z\S+:", raw):
            name = raw.split(":")[0]
            cur = out.setdefault(name, [])
            inasm = False
            continue
        if cur is None:
            continue
        if ";;#ASMSTART" in raw:
            inasm = True
            continue
        if ";;#ASMEND" in raw:
            inasm = False
            continue
        line = raw.split(";")[0].strip()
        if not line or line.endswith(":") or line.startswith("."):
            if line.startswith(".Lfunc_end"):
                cur, name = None, None
            continue
        parts = line.split(None, 1)
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        cur.append(Ins(op, args, inasm, raw.strip()))
    return out


def check(instrs, window=80):
    """Violations [(rule, producer, consumer, states, required)]."""
    bad = []
    n = len(instrs)
    for p, c in enumerate(instrs):
        # A: VALU write -> asm MFMA operand
        if c.is_mfma() and c.asm:
            need = c.srcs()
            st = 0
            for q in range(p - 1, max(-1, p - window), -1):
                w = instrs[q]
                if st >= 2:
                    break
                if w.is_valu() and w.dst() & need:
                    bad.append(("A", w.line, c.line, st, 2))
                    break
                st += w.states
        # B: MFMA result -> other access
        if c.is_mfma():
            d = regs(c.args[0])
            req = _PASSES.get(c.op, 16) + 4
            st = 0
            for q in range(p + 1, min(n, p + window)):
                r = instrs[q]
                if st >= req:
                    break
                if r.uses() & d:
                    chain = r.is_mfma() and regs(r.args[0]) == d and len(r.args) > 3 and regs(r.args[3]) == d
                    if not chain and (c.asm or r.asm):
                        bad.append(("B", c.line, r.line, st, req))
                    break
                st += r.states
        # C / D: SGPR from VALU -> asm memory instruction; M0 -> LDS-DMA
        if c.asm and c.op.startswith(_MEM):
            sg = {x for x in c.srcs() if x[0] == "s"}
            st = 0
            for q in range(p - 1, max(-1, p - window), -1):
                w = instrs[q]
                if st >= 5:
                    break
                if w.is_valu() and w.dst() & sg:
                    bad.append(("C", w.line, c.line, st, 5))
                    break
                st += w.states
            if c.args and c.args[-1].split()[-1] == "lds":
                st = 0
                for q in range(p - 1, max(-1, p - window), -1):
                    w = instrs[q]
                    if ("m", 0) in w.dst():
                        if st < 1:
                            bad.append(("D", w.line, c.line, st, 1))
                        break
                    st += w.states
                    if st >= 1:
                        break
    return bad


@pytest.mark.skipif(not have_hipcc(), reason="hipcc not available")
def test_no_unpadded_hazards_around_inline_asm():
    failures = []
    for (src, defs), asm in all_isa().items():
        for name, ins in kernels(asm).items():
            for rule, a, b, st, req in check(ins)[:3]:
                failures.append(f"{src} {' '.join(defs)} {name[:60]}: rule {rule}: '{a}' -> '{b}' "
                                f"after {st} of {req} wait states")
    assert not failures, "\n".join(failures)


def _asm(*lines):
    out = ["_Zk:"]
    for ln in lines:
        if ln.startswith("ASM "):
            out += [";;#ASMSTART", "\t" + ln[4:], ";;#ASMEND"]
        else:
            out.append("\t" + ln)
    return "\n".join(out + ["\ts_endpgm", ".Lfunc_end0:"])


def _rules(text):
    return [b[0] for b in check(kernels(text)["_Zk"])]


def test_detector_rules():
    mf = "v_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]"
    # A: a VALU write of an operand right before the asm MFMA, then padded
    assert _rules(_asm("v_mov_b32 v17, 0", "ASM " + mf, "ASM s_nop 7", "ASM s_nop 4")) == ["A"]
    assert _rules(_asm("v_mov_b32 v17, 0", "s_nop 1", "ASM " + mf, "ASM s_nop 7", "ASM s_nop 4")) == []
    # B: the accumulator read too early; the chain's next MFMA is fine
    assert _rules(_asm("ASM " + mf, "v_add_f32_e32 v30, v3, v3")) == ["B"]
    assert _rules(_asm("ASM " + mf, "ASM " + mf, "ASM s_nop 7", "ASM s_nop 4", "v_add_f32_e32 v30, v3, v3")) == []
    # C: a descriptor fresh from readfirstlane
    ld = "buffer_load_dwordx4 v[40:43], v1, s[8:11], 0 offen"
    assert _rules(_asm("v_readfirstlane_b32 s9, v2", "ASM " + ld)) == ["C"]
    assert _rules(_asm("v_readfirstlane_b32 s9, v2", "ASM s_nop 4", "ASM " + ld)) == []
    # D: M0 set right before an LDS-DMA
    dma = "buffer_load_dword v1, s[8:11], 0 offen lds"
    assert _rules(_asm("ASM s_mov_b32 m0, s3", "ASM " + dma)) == ["D"]
    assert _rules(_asm("ASM s_mov_b32 m0, s3", "ASM s_nop 0", "ASM " + dma)) == []
