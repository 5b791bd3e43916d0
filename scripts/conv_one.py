"""Run one conv_fwd shape repeatedly (for rocprofv3 counter collection).
usage: conv_one.py B H C1 C2 Cout tile reps"""
import os
import sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from unet_distributed_amd import native
C = native.require()
B, H, C1, C2, Co, tile, reps = [int(v) for v in sys.argv[1:8]]
dev = torch.device("cuda")
ptr = lambda t: int(t.data_ptr())
x = torch.randn(B, H, H, C1, device=dev).bfloat16()
x2 = torch.randn(B, H, H, max(C2, 1), device=dev).bfloat16()
Kp = (9 * (C1 + C2) + 63) // 64 * 64
w = (torch.randn(Co, Kp, device=dev) * 0.05).bfloat16()
out = torch.empty(B, H, H, Co, device=dev, dtype=torch.bfloat16)
d = dict(N=B, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, C2=C2, src1=ptr(x),
         src2=ptr(x2) if C2 else None, wgt=ptr(w), Cout=Co, relu=1, dst1=ptr(out), tile=tile)
st = int(torch.cuda.current_stream().cuda_stream)
for _ in range(reps):
    C.conv_fwd(d, st)
torch.cuda.synchronize()
print("done")
