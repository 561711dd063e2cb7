"""Scratch (spill) budget of the LDS-DMA GEMM kernels, checked from the gfx950
assembly on the CPU host.

Round 3 found twice that an LDS-DMA implicit-GEMM variant computes wrong rows
once it spills more around its `buffer_load ... lds` stages: the stride-2
data gradient with the MASKX epilogue on 256x256 tiles (moved to 256x128), and
a runtime epilogue branch that doubled the 256x256 3x3-dgrad MASKX tile's
spill 44 -> 88 bytes (the full-network trajectory went NaN at step 2,
tests/test_trajectory_gpu.py; fixed by making the branch compile-time).  A
code change that grows these spills must be measured on the GPU first: this
test pins the budgets measured to be correct.

Round 6: the main loop issues every LDS-DMA piece from inline asm that sets M0
in the same statement (no compiler-placed M0 write a spill could separate
from its load) and spreads the pieces over the MFMAs with double-buffered
fragments; the dense MASKX / RESBITS 256x256 epilogues now spill 28 / 128 B,
none of it inside the MFMA loop, measured correct on MI355X
(tests/test_igemm_gpu.py with every tile config forced, the full-network
fp32-truth and trajectory tests).
"""
import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"

# kernel-name fragment -> max private_segment_fixed_size (bytes) measured correct on MI355X
BUDGET = {
    "igemm_kernelILi256ELi256ELi2ELi4ELi2ELi2ELi1ELi2E": 44,  # 3x3 dgrad, MASKX, 256x256 (stages 3)
    "igemm_kernelILi256ELi256ELi2ELi4ELi2ELi1ELi1ELi2E": 12,  # 3x3 forward, STATS, 256x256
    "igemm_kernelILi256ELi256ELi2ELi4ELi0ELi3ELi1ELi2E": 128,  # dense RESBITS, 256x256 (epilogue only)
    "igemm_kernelILi256ELi256ELi2ELi4ELi0ELi2ELi1ELi2E": 28,   # dense MASKX, 256x256 (epilogue only)
    "igemm_kernelILi256ELi128ELi4ELi2ELi3ELi2ELi1ELi2E": 0,   # stride-2 dgrad, MASKX, 256x128 (in use)
    "igemm_kernelILi128ELi128ELi2ELi2ELi2ELi2ELi2ELi2E": 0,   # 3x3 dgrad, MASKX, 128x128
}


def _meta(asm: str):
    out = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", asm, re.S):
        sz = re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(2))
        out[m.group(1)] = int(sz.group(1)) if sz else 0
    return out


@pytest.mark.skipif(not Path(HIPCC).exists() or shutil.which("python3") is None, reason="no hipcc")
def test_igemm_spill_budgets(tmp_path):
    src = ROOT / "csrc" / "igemm.hip"
    out = tmp_path / "igemm.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S",
                        f"-I{ROOT / 'csrc'}", str(src), "-o", str(out)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    meta = _meta(out.read_text())
    for frag, budget in BUDGET.items():
        hits = {k: v for k, v in meta.items() if frag in k}
        assert hits, f"kernel {frag} not found"
        for k, v in hits.items():
            assert v <= budget, f"{k}: {v} B of scratch > the {budget} B measured correct"


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="no hipcc")
def test_igemm_main_loop_has_no_spill(tmp_path):
    """No scratch access between the first and the last MFMA of any LDS-DMA
    GEMM kernel: a spill there would cost every K-step (round-6 main loop)."""
    src = ROOT / "csrc" / "igemm.hip"
    out = tmp_path / "igemm.s"
    r = subprocess.run([HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "--offload-device-only", "-S",
                        f"-I{ROOT / 'csrc'}", str(src), "-o", str(out)], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    asm = out.read_text()
    n = 0
    for m in re.finditer(r"\n(_ZN3kdl\S*igemm_kernel\S*):(.*?)s_endpgm", asm, re.S):
        body = m.group(2).splitlines()
        mf = [k for k, ln in enumerate(body) if "v_mfma" in ln]
        if not mf:
            continue
        n += 1
        inside = [ln for ln in body[mf[0]:mf[-1]] if "scratch_" in ln]
        assert not inside, (m.group(1)[:90], inside[:4])
    assert n > 20
