"""Build-level guard for the inline-asm MFMA kernels (CPU only: hipcc
cross-compiles gfx950 here; skipped where hipcc is absent).

The bf16 kernels issue their MFMAs from inline asm, so LLVM cannot see them
and pads none of their register hazards.  Any spill or reload the register
allocator puts next to them is unpadded: at PMM_WS_NST = KS = 6 the
wave-specialised kernel spilled 592 B per lane into its MFMA loop and
returned wrong scores (csrc/pmm_bf16_ws_kernel.h, Carve::SLOT_REPEATS).  This
test compiles every instantiation to ISA and asserts that no basic block
holding an MFMA holds scratch (spill) code.

Scope: this guards spill/reload code next to the asm MFMAs; the wait-state
rules between asm statements and compiler code are checked on the same ISA
by tests/test_asm_hazards.py.
"""
import re

import pytest

from isa_util import all_isa, have_hipcc

_LABEL = re.compile(r"^(\.LBB\S*:|; %bb\.\d+:)")


def compiler_m0_uses(asm: str):
    """Lines outside inline asm that name M0: the 256-row kernel (ff) sets M0
    in asm for its LDS-DMA (M0 cannot be declared clobbered), which is safe only
    while the compiler itself never relies on M0 in that kernel."""
    out, inasm, func = [], False, None
    for line in asm.splitlines():
        if re.match(r"^_Z\S+:", line):
            func = line.split(":")[0]
        if ";;#ASMSTART" in line:
            inasm = True
            continue
        if ";;#ASMEND" in line:
            inasm = False
            continue
        s = line.strip()
        if not inasm and func and "_ff_" in func and not s.startswith(";") and re.search(r"\bm0\b", s):
            out.append((func, s))
    return out


def mfma_blocks_with_spills(asm: str):
    """(function, block label) of every basic block with both an MFMA and a
    scratch access."""
    bad, func, label, has_mfma, has_scr = [], None, None, False, False

    def close():
        if has_mfma and has_scr:
            bad.append((func, label))

    for line in asm.splitlines():
        if re.match(r"^_Z\S+:", line):
            close()
            func, label, has_mfma, has_scr = line.split(":")[0], "entry", False, False
            continue
        if _LABEL.match(line) or line.strip().startswith("s_endpgm"):
            close()
            label, has_mfma, has_scr = line.split(":")[0], False, False
            continue
        s = line.strip()
        if s.startswith("v_mfma"):
            has_mfma = True
        elif s.startswith("scratch_"):
            has_scr = True
    close()
    return bad


@pytest.mark.skipif(not have_hipcc(), reason="hipcc not available")
def test_no_spill_code_beside_inline_asm_mfmas():
    failures = []
    for (src, defs), asm in all_isa().items():
        assert "v_mfma" in asm, f"{src} {defs}: no MFMA in the ISA"
        bad = mfma_blocks_with_spills(asm)
        if bad:
            failures.append(f"{src} {' '.join(defs)}: {bad[:4]}")
        m0 = compiler_m0_uses(asm)
        if m0:
            failures.append(f"{src} {' '.join(defs)}: compiler M0 use {m0[:2]}")
    assert not failures, "spill code in MFMA blocks / compiler M0 use:\n" + "\n".join(failures)


def test_detector_flags_a_spill_in_an_mfma_block():
    asm = "\n".join([
        "_Zkern:",
        ".LBB0_1:",
        "\tv_mfma_f32_32x32x16_bf16 v[0:15], v[16:19], v[20:23], v[0:15]",
        "\tscratch_load_dwordx4 v[16:19], off, off",
        ".LBB0_2:",
        "\tscratch_store_dword off, v3, off",
        "\ts_endpgm",
    ])
    assert mfma_blocks_with_spills(asm) == [("_Zkern", ".LBB0_1")]


def _makefile_var(name):
    import os
    mk = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "polars-matmul_amd", "Makefile")
    for line in open(mk):
        m = re.match(rf"^{name}\s*:?=\s*(.*)$", line.strip())
        if m:
            return m.group(1).split()
    raise KeyError(name)


@pytest.mark.skipif(not have_hipcc(), reason="hipcc not available")
def test_f64_mfmas_keep_their_accumulators_in_vgprs():
    # pmm_f64.hip is built with the MFMAs in their VGPR form (Makefile
    # F64_FLAGS): with the compiler's AGPR choice every 16-wide K chunk copied
    # the accumulators VGPR -> AGPR and back (64 v_accvgpr moves per 16 MFMAs,
    # 42.1 vs 39.8 ms at 4096 x 1M x 256).  Every f64 MFMA kernel of the
    # product build must be free of accumulator moves.
    import os
    import subprocess
    import tempfile

    from isa_util import CSRC, FLAGS, HIPCC

    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "f64.s")
        subprocess.run([HIPCC, *FLAGS, *_makefile_var("F64_FLAGS"), "-I", CSRC, "-o", out,
                        os.path.join(CSRC, "pmm_f64.hip")], check=True, capture_output=True, timeout=600)
        asm = open(out).read()
    funcs, func = {}, None
    for line in asm.splitlines():
        if re.match(r"^_Z\S+:", line):
            func = line.split(":")[0]
            funcs[func] = [0, 0]
        elif func:
            s = line.strip()
            funcs[func][0] += s.startswith("v_mfma_f64")
            funcs[func][1] += s.startswith("v_accvgpr")
    mfma = {f: c for f, c in funcs.items() if c[0]}
    assert len(mfma) >= 6, sorted(mfma)  # store (3 metrics) + top-k (3 metrics x 2 tiles)
    bad = {f: c[1] for f, c in mfma.items() if c[1]}
    assert not bad, f"accumulator moves in f64 MFMA kernels: {bad}"


def scratch_by_kernel(asm: str):
    """{kernel: (private segment bytes, scratch instructions)} from the ISA's
    kernel descriptors and bodies."""
    sizes, counts, func, desc = {}, {}, None, None
    for line in asm.splitlines():
        m = re.match(r"^(_Z\S+):", line)
        if m:
            func = m.group(1)
            counts.setdefault(func, 0)
            continue
        s = line.strip()
        m = re.match(r"^\.amdhsa_kernel\s+(\S+)", s)
        if m:
            desc = m.group(1)
            continue
        m = re.match(r"^\.amdhsa_private_segment_fixed_size\s+(\d+)", s)
        if m and desc:
            sizes[desc] = int(m.group(1))
            continue
        if func and s.startswith("scratch_"):
            counts[func] += 1
    return {k: (sizes.get(k, -1), counts.get(k, 0)) for k in set(sizes) | set(counts)}


@pytest.mark.skipif(not have_hipcc(), reason="hipcc not available")
def test_f32_gemm_and_merge_kernels_use_no_scratch():
    # the two-pass pre-filter reads acc[c][e] by a wave-uniform
    # runtime index; that must stay a register-indexed move, never demote the
    # accumulators to scratch (a compiler change could, silently).  And the
    # merge kernels: a scratch-resident value read per candidate batch waits
    # for every load in flight (scratch counts in vmcnt) -- round 5's
    # threshold did, serialising the batch pipeline.
    asm = all_isa()[("pmm_kernels.hip", ())]
    sc = scratch_by_kernel(asm)
    gemm = {k: v for k, v in sc.items() if "gemm_f32_kernel" in k}
    merge = {k: v for k, v in sc.items() if "merge_kernel" in k}
    assert len(gemm) >= 10 and len(merge) >= 5, (sorted(gemm)[:3], sorted(merge))
    bad = {k: v for k, v in {**gemm, **merge}.items() if v != (0, 0)}
    assert not bad, f"scratch (bytes, instructions) in: {bad}"
