"""gfx950 ISA of the inline-asm kernels, compiled once per test session
(hipcc cross-compiles here; no GPU).  Shared by tests/test_kernel_resources.py
and tests/test_asm_hazards.py."""
import functools
import os
import shutil
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "polars-matmul_amd", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
         "--cuda-device-only", "-S"]

# (source, defines): every padded-D instantiation of the wave-specialised
# kernel (and of its 32x32x16 form at a few), the ring sizes whose slot
# sequence repeats per tile, the one-wave-per-SIMD bf16 kernel at the largest
# D, every instantiation of the fire-and-forget 256-row kernel
BUILDS = [("pmm_bf16_ws_ks.hip", (f"-DPMM_BF16_KS={k}",)) for k in range(1, 7)] + [
    ("pmm_bf16_ws_ks.hip", ("-DPMM_BF16_KS=6", "-DPMM_WS_NST=6")),
    ("pmm_bf16_ws_ks.hip", ("-DPMM_BF16_KS=6", "-DPMM_WS_NST=3")),
    ("pmm_bf16_ks.hip", ("-DPMM_BF16_KS=6",)),
] + [
    # the 32x32x16 form of the wave-specialised kernel (PMM_WS_MFMA16=0)
    ("pmm_bf16_ws_ks.hip", (f"-DPMM_BF16_KS={k}", "-DPMM_WS_MFMA16=0")) for k in (1, 2, 3, 6)] + [
    ("pmm_bf16_ff_ks.hip", (f"-DPMM_BF16_KS={k}",)) for k in range(1, 7)] + [
    ("pmm_kernels.hip", ())]  # (the f32 seed prologue's asm LDS-DMA)


def have_hipcc():
    return os.path.exists(HIPCC)


@functools.lru_cache(maxsize=None)
def all_isa():
    """{(source, defines): assembly text} for every entry of BUILDS, compiled
    in parallel."""
    tmp = tempfile.mkdtemp(prefix="pmm_isa_")
    try:
        procs = []
        for i, (src, defs) in enumerate(BUILDS):
            out = os.path.join(tmp, f"b{i}.s")
            cmd = [HIPCC, *FLAGS, *defs, "-I", CSRC, "-o", out, os.path.join(CSRC, src)]
            procs.append((src, defs, out, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                           stderr=subprocess.STDOUT)))
        res = {}
        for src, defs, out, p in procs:
            log = p.communicate(timeout=600)[0].decode(errors="replace")
            if p.returncode != 0:
                raise RuntimeError(f"{src} {defs}: {log[-2000:]}")
            with open(out) as f:
                res[(src, defs)] = f.read()
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
