"""Time conv_fwd tile variants on UNet layer shapes (interleaved rounds, one process)."""
import sys, time, json
import torch
from unet_distributed_amd import native
C = native.require()
dev = torch.device("cuda")
ptr = lambda t: int(t.data_ptr())
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
shapes = [  # (name, H, Cin, Cout, C2)
    ("L1 32->32", 128, 32, 32, 0), ("L1 concat 32+32->32", 128, 32, 32, 32), ("L2 64->64", 64, 64, 64, 0),
    ("L2 32->64", 64, 32, 64, 0), ("L3 128->128", 32, 128, 128, 0), ("L4 256->256", 16, 256, 256, 0),
    ("L5 512->512", 8, 512, 512, 0), ("L1 dgrad 64->32", 128, 32, 64, 0), ("L2 concat 64+64->64", 64, 64, 64, 64),
    ("L3 64->128", 32, 64, 128, 0)]
res = {}
for name, H, Cin, Co, C2 in shapes:
    x = torch.randn(B, H, H, Cin, device=dev).bfloat16()
    x2 = torch.randn(B, H, H, C2, device=dev).bfloat16() if C2 else None
    Kp = (9 * (Cin + C2) + 63) // 64 * 64
    w = (torch.randn(Co, Kp, device=dev) * 0.05).bfloat16()
    out = torch.empty(B, H, H, Co, device=dev, dtype=torch.bfloat16)
    d = dict(N=B, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=Cin, C2=C2, src1=ptr(x),
             src2=ptr(x2) if C2 else None, wgt=ptr(w), Cout=Co, relu=1, dst1=ptr(out))
    tiles = [t for t in (1, 2, 3, 4, 5, 6) if Co % (128 if t == 1 else 64 if t in (2, 5) else 32) == 0]
    if H < 16 or Cin % 32:
        tiles = [t for t in tiles if t < 6]
    times = {t: [] for t in tiles}
    st = int(torch.cuda.current_stream().cuda_stream)
    for rnd in range(5):
        for t in tiles:
            dd = dict(d, tile=t)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                C.conv_fwd(dd, st)
            e1.record(); torch.cuda.synchronize()
            times[t].append(e0.elapsed_time(e1) / 5)
    fl = 2.0 * B * H * H * 9 * (Cin + C2) * Co
    r = {t: (min(v), fl / min(v) / 1e9) for t, v in times.items()}
    res[name] = r
    print("%-24s " % name + "  ".join("t%d %.3fms %4.0fTF" % (t, ms, tf) for t, (ms, tf) in r.items()), flush=True)
