"""Host-side (no GPU) checks of the HIP extension's launch planning: the
extension imports on a CPU host, and the workspace sizing functions the engine
allocates by agree with the kernels' dispatch rules."""
import os

import pytest


def _ext():
    try:
        from kubedl_amd.ops import _ext
        return _ext.load()
    except Exception as e:  # not built in this checkout
        pytest.skip(f"extension not built: {e}")


def test_conv3x3_wgrad_slabs_cover_the_halo_path():
    ext = _ext()
    # 56x56 / 64 -> 64 / stride 1: one slab per halo block (one image's 14 tiles per block at batch 256)
    assert ext.conv3x3_wgrad_slabs(256, 56, 56, 64, 64, 1) == 256
    assert ext.conv3x3_wgrad_slabs(20, 56, 56, 64, 64, 1) == 140  # 280 tiles, 2 per block
    assert ext.conv3x3_wgrad_slabs(1, 56, 56, 64, 64, 1) >= 14
    # every other geometry: the implicit GEMM's split-M slab count -- at 128 x 128 tiles the
    # 1x1 rule's, at 256 x 256 tiles (Cin, Cout % 256 == 0) one round of one block per CU
    for nb, h, cin, cout, s in [(256, 28, 128, 128, 1), (256, 56, 128, 128, 2), (4, 56, 64, 128, 1),
                                (4, 55, 64, 64, 1)]:
        ho = (h - 1) // s + 1
        assert ext.conv3x3_wgrad_slabs(nb, h, h, cin, cout, s) == \
            ext.conv1x1_wgrad_splits(nb * ho * ho, cout, 9 * cin)
    target = int(384) // 2  # KDL_TUNE wgrad_blocks default; 256x256 tiles: one block per CU
    for nb, h, c, s, tiles in [(256, 14, 256, 1, 9), (256, 7, 512, 1, 36), (256, 14, 512, 2, 36)]:
        ho = (h - 1) // s + 1
        assert ext.conv3x3_wgrad_slabs(nb, h, h, c, c, s) == max(1, target // tiles)
        assert ext.conv3x3_wgrad_slabs(nb, h, h, c, c, s) >= ext.conv1x1_wgrad_splits(nb * ho * ho, c, 9 * c)


def test_bn_workspace_layout_size():
    ext = _ext()
    # [32][2C] fwd replicas | [32][2C] bwd | [5C] coefficients | [32] finalize descriptor | [64] tile counters
    for c in (64, 256, 2048):
        assert ext.bn_workspace_floats(c) == 32 * 4 * c + 5 * c + 32 + 64


def test_native_tune_knobs_parse(tmp_path):
    """csrc/tune.h: every native A/B knob comes from the one KDL_TUNE variable."""
    import shutil
    import subprocess
    from pathlib import Path
    gxx = shutil.which("g++")
    if gxx is None:
        import pytest
        pytest.skip("no g++")
    root = Path(__file__).resolve().parents[1]
    src = tmp_path / "t.cpp"
    src.write_text('#include "tune.h"\n#include <cstdio>\n'
                   'int main() { printf("%d %d %d %d %d\\n", kdl::tune_int("gemm_cfg", -1), kdl::tune_int("igemm_cfg", -1),'
                   ' kdl::tune_int("halo", 1), (int)kdl::tune_has("wgrad_big"), kdl::tune_int("gemm", 7)); }\n')
    exe = tmp_path / "t"
    subprocess.run([gxx, "-std=c++17", f"-I{root / 'csrc'}", str(src), "-o", str(exe)], check=True)
    env = dict(os.environ, KDL_TUNE="gemm_cfg=5, igemm_cfg=2,wgrad_big=0")
    out = subprocess.run([str(exe)], env=env, capture_output=True, text=True, check=True).stdout.split()
    assert out == ["5", "2", "1", "1", "7"], out
    env.pop("KDL_TUNE")
    out = subprocess.run([str(exe)], env=env, capture_output=True, text=True, check=True).stdout.split()
    assert out == ["-1", "-1", "1", "0", "7"], out


def test_extension_loads_on_the_host():
    """ops/_ext.load() imports the in-tree kubedl_amd/_C.so (no GPU needed to
    import it), and KDL_C_PATH loads an A/B build of the same module."""
    from pathlib import Path
    from kubedl_amd.ops import _ext
    so = Path(__file__).resolve().parents[1] / "kubedl_amd" / "_C.so"
    if not so.exists():
        pytest.skip("extension not built")
    m = _ext.load()
    assert hasattr(m, "conv1x1_gemm") and hasattr(m, "set_gemm_core")
