"""Run one fused 1x1-conv GEMM shape repeatedly (for rocprofv3 --pmc passes)."""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from kubedl_amd.ops import _ext  # noqa: E402

ext = _ext.load()
cin, cout, h, epi = (int(a) for a in sys.argv[1:5])
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 20
B = 256
M = B * h * h
x = torch.randn(M, cin, device="cuda").bfloat16()
w = (torch.randn(cout, cin, device="cuda") / cin ** 0.5).bfloat16()
y = torch.empty(M, cout, device="cuda", dtype=torch.bfloat16)
ws = torch.zeros(ext.bn_workspace_floats(cout), device="cuda")
sh = torch.zeros(cout, device="cuda")
ex = torch.randn(M, cout, device="cuda").bfloat16()
bits = torch.randint(0, 256, (M * cout // 8,), device="cuda", dtype=torch.uint8)
mean = torch.zeros(cout, device="cuda")
coef = torch.cat([torch.ones(cout, device="cuda"), torch.zeros(cout, device="cuda")])
for _ in range(reps):
    if epi == 1:
        ext.conv1x1_gemm(x, w, y, M, cout, cin, 0, 0, 0, 0, 1, None, 1, sh, ws, None, None, None, None, 1, 0, 0,
                         None, None, None, None)
    elif epi == 3:
        ext.conv1x1_gemm(x, w, y, M, cout, cin, 0, 0, 0, 0, 1, None, 3, None, ws, ex, mean, None, ex, 1, h, h, bits,
                         None, None, None)
    else:
        ext.conv1x1_gemm(x, w, y, M, cout, cin, 0, 0, 0, 0, 1, None, 0, None, None, None, None, None, None, 1, 0, 0,
                         None, None, None, None)
torch.cuda.synchronize()
print("done")
