"""Weight layouts of the ResNet conv kernels that are not plain GEMMs.

Stride-2 3x3 data gradient as four sub-pixel class GEMMs.

For a 3x3 / pad 1 / stride 2 conv y = conv(x, w), dx pixel (2i + py, 2j + px)
receives dy(oh, ow) * w[:, :, r, s] only where 2 oh - 1 + r = 2i + py, i.e.

    py = 0: r = 1 (oh = i)          py = 1: r = 0 (oh = i + 1), r = 2 (oh = i)

and the same for columns.  Each class (py, px) is therefore a plain GEMM over
the dy-sized pixel grid with 1, 2, 2 or 4 taps -- 9 taps in total, none of
them zero, and no zero-filled dx.  ``csrc/igemm.hip`` (G_DGRAD2) runs the four
classes as M-tile ranges of one launch; ``CLASS_TAPS`` is its tap order and
``s2_dgrad_weights`` the class-major weight matrix it reads.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

# (r, s) taps of class c = 2 py + px, in the kernel's order (ri major, si minor;
# r = py ? (0, 2)[ri] : 1, s = px ? (0, 2)[si] : 1)
CLASS_TAPS = (
    ((1, 1),),
    ((1, 0), (1, 2)),
    ((0, 1), (2, 1)),
    ((0, 0), (0, 2), (2, 0), (2, 2)),
)
S2_TAPS = [t for taps in CLASS_TAPS for t in taps]  # flattened: column block t of the weights
_IDX_CACHE: dict = {}


def _tap_index(device) -> torch.Tensor:
    idx = _IDX_CACHE.get(device)
    if idx is None:
        idx = torch.tensor([3 * r + s for r, s in S2_TAPS], device=device)
        _IDX_CACHE[device] = idx
    return idx


def s2_dgrad_weights(w: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] conv weight -> [Cin, 9 * Cout] bf16 with column block
    t (the t-th tap of ``CLASS_TAPS`` flattened) = w[:, :, r_t, s_t]^T."""
    cout, cin = w.shape[:2]
    wt = w.permute(1, 2, 3, 0).reshape(cin, 9, cout)  # [Cin][r*3+s][Cout]
    return wt.index_select(1, _tap_index(w.device)).reshape(cin, 9 * cout).to(torch.bfloat16).contiguous()


def s2_dgrad_reference(dy: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The class decomposition in plain PyTorch (NCHW, any dtype): dx of
    conv2d(x, w, stride=2, padding=1) for even input sizes 2 Hd x 2 Wd."""
    nb, cout, hd, wd = dy.shape
    cin = w.shape[1]
    dyp = F.pad(dy, (0, 1, 0, 1))  # dy(i + 1, j + 1) past the edge reads zero
    dx = dy.new_zeros(nb, cin, 2 * hd, 2 * wd)
    for c, taps in enumerate(CLASS_TAPS):
        py, px = c >> 1, c & 1
        acc = dy.new_zeros(nb, cin, hd, wd)
        for r, s in taps:
            di, dj = int(r == 0), int(s == 0)
            src = dyp[:, :, di:di + hd, dj:dj + wd]
            acc = acc + torch.einsum("nohw,oi->nihw", src, w[:, :, r, s])
        dx[:, :, py::2, px::2] = acc
    return dx


# ---------------------------------------------------------------------------- stem
STEM_K = 224  # 7 r x 8 s x 4 c (s = 7 and c = 3 are zero padding)


def stem_weights(w: torch.Tensor) -> torch.Tensor:
    """[64, 3, 7, 7] stem weight -> [64, 224] bf16 in csrc/stem.hip's K order
    k = r * 32 + s * 4 + c (so an 8-deep MFMA fragment is two horizontally
    adjacent input pixels of 4 channels)."""
    cout = w.shape[0]
    wt = F.pad(w.permute(0, 2, 3, 1), (0, 1, 0, 1))  # [Cout, 7 r, 8 s, 4 c]
    return wt.reshape(cout, STEM_K).to(torch.bfloat16).contiguous()


def stem_reference(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """The stem kernel's GEMM in plain PyTorch: patches of the NHWC input in
    the same K order times ``stem_weights`` (fp32) -> NCHW output."""
    nb, _, h, wd = x.shape
    oh, ow = (h + 6 - 7) // 2 + 1, (wd + 6 - 7) // 2 + 1
    xp = F.pad(x.float().permute(0, 2, 3, 1), (0, 1, 3, 4, 3, 3))  # [Nb, H+6, W+7, 4]
    cols = []
    for r in range(7):
        for s in range(8):
            cols.append(xp[:, r:r + 2 * oh:2, s:s + 2 * ow:2, :])  # [Nb, oh, ow, 4]
    patches = torch.stack(cols, dim=3).reshape(nb, oh, ow, STEM_K)
    wt = F.pad(w.float().permute(0, 2, 3, 1), (0, 1, 0, 1)).reshape(w.shape[0], STEM_K)
    return (patches @ wt.t()).permute(0, 3, 1, 2)


def stem_grad_from_k(dwk: torch.Tensor) -> torch.Tensor:
    """[64, 224] (stem K order) -> [64, 3, 7, 7] (the s = 7 / c = 3 padding columns dropped)."""
    return dwk.view(dwk.shape[0], 7, 8, 4)[:, :, :7, :3].permute(0, 3, 1, 2)
