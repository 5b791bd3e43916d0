import torch, torch.nn.functional as F
from unet_distributed_amd import native
C = native.require()
dev = torch.device("cuda")
ptr = lambda t: int(t.data_ptr())
st = lambda: int(torch.cuda.current_stream().cuda_stream)
torch.set_printoptions(precision=1, linewidth=220)
def run(X, G, KH, pad, splits=1):
    N, H, W, Mc = X.shape; Nc = G.shape[-1]
    KT = KH * KH
    slab = torch.zeros(splits * KT * Mc * Nc, device=dev)
    C.wgrad(dict(N=N, QH=H, QW=W, AH=H, AW=W, KH=KH, KW=KH, pad=pad, M1=Mc, a1=ptr(X), b=ptr(G), Nc=Nc,
                 splits=splits, slab=ptr(slab)), st())
    torch.cuda.synchronize()
    return slab.view(splits, KT, Mc, Nc).sum(0)
Q = 32
X = torch.zeros(1, 1, Q, 32, device=dev); G = torch.zeros(1, 1, Q, 32, device=dev)
for q in range(Q):
    X[0, 0, q, q] = 1.0
    G[0, 0, q, :] = torch.arange(32, device=dev) + 100 * (q % 4)
X, G = X.bfloat16(), G.bfloat16()
out = run(X, G, 3, 1)[4]     # center tap == 1x1 product
ref = X.float().reshape(Q, 32).t() @ G.float().reshape(Q, 32)
print("center err", (out - ref).abs().max().item())
print("out[:6,:8]\n", out[:6, :8]); print("ref[:6,:8]\n", ref[:6, :8])
print("out[:, 0]", out[:, 0].tolist())
bad = ((out - ref).abs() > 1e-3).nonzero()
print("num bad", bad.shape[0], bad[:20].tolist())
