import sys, os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
from kubedl_amd.ops import _ext
from kubedl_amd.ops.conv import stem_weights
ext = _ext.load()
torch.manual_seed(35)
nb = 2
x = torch.randn(nb, 224, 224, 3, device="cuda").bfloat16().permute(0, 3, 1, 2)
w = (torch.randn(64, 3, 7, 7, device="cuda") / 12).bfloat16().contiguous(memory_format=torch.channels_last)
ya = torch.empty(nb, 64, 112, 112, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
yb = torch.empty_like(ya)
ext.stem7x7_fwd(x, stem_weights(w), ya, None, None)
ext.stem7x7_fwd(x, w, yb, None, None)
ext.stem7x7_fwd(x, stem_weights(w), ya2 := torch.empty_like(ya), None, None)
ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
torch.cuda.synchronize()
d = (ya.float() - yb.float()).abs()
print("ya vs ya2 equal:", torch.equal(ya, ya2))
print("ya vs yb: n diff", int((d > 0).sum()), "max", float(d.max()))
print("ya-ref max", float((ya.float() - ref).abs().max()), "yb-ref max", float((yb.float() - ref).abs().max()))
idx = (d > 0).nonzero()
print("diff channels:", sorted(set(idx[:, 1].tolist()))[:20], "rows", sorted(set(idx[:, 2].tolist()))[:10])
wk = stem_weights(w)
# rebuild the kernel's raw reorder on the host and compare with stem_weights
flat = w.permute(0, 2, 3, 1).reshape(64, 147)  # memory order [n][r][s][c]
k = torch.arange(224, device="cuda")
r, s, c = k >> 5, (k >> 2) & 7, k & 3
valid = (s < 7) & (c < 3)
src = (r * 7 + s.clamp(max=6)) * 3 + c.clamp(max=2)
raw = torch.where(valid[None, :], flat[:, src], torch.zeros((), dtype=flat.dtype, device="cuda"))
print("host raw reorder == stem_weights:", torch.equal(raw, wk))
print("w strides", w.stride())
