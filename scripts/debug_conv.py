import torch, torch.nn.functional as F
from unet_distributed_amd import native
C = native.require()
dev = torch.device("cuda")
ptr = lambda t: int(t.data_ptr())
st = lambda: int(torch.cuda.current_stream().cuda_stream)
torch.set_printoptions(precision=3, linewidth=200)
# 1x1 conv = plain GEMM: out[m][n] = sum_c x[m][c] w[n][c]
M, K, N = 256, 32, 32
x = torch.zeros(1, 1, M, K, device=dev)
for m in range(M): x[0, 0, m, m % K] = 1.0 + m // K     # one-hot rows
x = x.bfloat16()
w = torch.arange(N * K, device=dev, dtype=torch.float32).reshape(N, K).div(64).bfloat16()
out = torch.zeros(1, 1, M, N, device=dev, dtype=torch.bfloat16)
C.conv_fwd(dict(N=1, OH=1, OW=M, IH=1, IW=M, C1=K, src1=ptr(x), wgt=ptr(w), Cout=N, dst1=ptr(out)), st())
ref = x.float().reshape(M, K) @ w.float().t()
o = out.float().reshape(M, N)
print("1x1 max err", (o - ref).abs().max().item())
bad = (o - ref).abs().amax(1) > 1e-2
print("bad rows", bad.nonzero().flatten()[:40].tolist())
print("out rows 0..3\n", o[:4, :8]); print("ref rows 0..3\n", ref[:4, :8])
print("out rows 16..19\n", o[16:20, :8]); print("ref\n", ref[16:20, :8])
