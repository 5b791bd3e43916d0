"""Implicit-GEMM tile sweep on the b1024 shapes that take the GEMM path (level-5 3x3
convs and their data gradients, the 16- / 8-wide transposed-conv data gradients):
   python scripts/gemm_tiles.py [batch]"""
import sys
import torch
from unet_distributed_amd import native
C = native.require()
dev = torch.device("cuda")
ptr = lambda t: int(t.data_ptr())
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
# (name, coarse/out H, Cin (K channels), Cout, kind) kind: conv3 | tdg (2x2 s2 dgrad: input fine 2H)
shapes = [("L5 conv 256->512", 8, 256, 512, "conv3"), ("L5 conv 512->512", 8, 512, 512, "conv3"),
          ("L5 dgrad 512->256", 8, 512, 256, "conv3"), ("tconv7 dgrad 128(fine 32)->256", 16, 128, 256, "tdg"),
          ("tconv6 dgrad 256(fine 16)->512", 8, 256, 512, "tdg")]
st = int(torch.cuda.current_stream().cuda_stream)
for name, H, Ci, Co, kind in shapes:
    IH = 2 * H if kind == "tdg" else H
    x = torch.randn(B, IH, IH, Ci, device=dev).bfloat16()
    taps = 4 if kind == "tdg" else 9
    Kp = (taps * Ci + 63) // 64 * 64
    w = (torch.randn(Co, Kp, device=dev) * 0.05).bfloat16()
    out = torch.empty(B, H, H, Co, device=dev, dtype=torch.bfloat16)
    if kind == "tdg":
        d = dict(N=B, OH=H, OW=H, IH=IH, IW=IH, KH=2, KW=2, stride=2, pad=0, C1=Ci, src1=ptr(x), wgt=ptr(w),
                 Cout=Co, relu=0, dst1=ptr(out))
    else:
        d = dict(N=B, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Ci, src1=ptr(x), wgt=ptr(w), Cout=Co,
                 relu=0, dst1=ptr(out))
    fl = 2.0 * B * H * H * taps * Ci * Co
    res = {}
    for t in (0, 1, 2, 3, 4, 5):
        try:
            C.conv_fwd(dict(d, tile=t), st)
        except Exception as ex:
            continue
        ts = []
        for rnd in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                C.conv_fwd(dict(d, tile=t), st)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        res[t] = min(ts)
    print("%-34s " % name + "  ".join("t%d %.3f ms %4.0f TF" % (t, v, fl / v / 1e9) for t, v in res.items()), flush=True)
