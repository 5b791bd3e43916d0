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

# ---- wgrad: row-window (win=0) vs tiled (win=-1) on the fine-level shapes
wshapes = [("L1 32x32", 128, 32, 0, 32), ("L1 concat 32+32 -> 32", 128, 32, 32, 32), ("L2 32->64", 64, 32, 0, 64),
           ("L2 64x64", 64, 64, 0, 64), ("L2 concat 64+64 -> 64", 64, 64, 64, 64), ("L3 64->128", 32, 64, 0, 128),
           ("L3 128x128", 32, 128, 0, 128), ("L3 concat 128+128 -> 128", 32, 128, 128, 128),
           ("L4 256x256", 16, 256, 0, 256), ("L4 concat 256+256 -> 256", 16, 256, 256, 256),
           ("L5 256->512", 8, 256, 0, 512), ("L5 512x512", 8, 512, 0, 512)]
for name, H, C1, C2, Co in wshapes:
    a = torch.randn(B, H, H, C1, device=dev).bfloat16()
    a2 = torch.randn(B, H, H, max(C2, 1), device=dev).bfloat16()
    dy = torch.randn(B, H, H, Co, device=dev).bfloat16()
    Mt = C1 + C2
    st = int(torch.cuda.current_stream().cuda_stream)
    res = {}
    for win in (0, -1):
        BM, BN, NTAP, sm = C.wgrad_pick(C1, C2, Co, 9, QW=H, win=win)
        tiles = (Mt // BM) * (Co // BN) * (9 // NTAP)
        splits = max(1, min(-(-512 // tiles), max(1, B * H * H // 1024)))
        slab = torch.empty(splits * 9 * Mt * Co, device=dev)
        bsl = torch.empty(splits * 8 * max(Mt, Co), device=dev)
        d = dict(N=B, QH=H, QW=H, AH=H, AW=H, KH=3, KW=3, pad=1, M1=C1, M2=C2, a1=ptr(a), a2=ptr(a2) if C2 else None,
                 b=ptr(dy), Nc=Co, bias_mode=1 if BM < 128 else 0, splits=splits, slab=ptr(slab), bias_slab=ptr(bsl),
                 win=win)
        ts = []
        for rnd in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                C.wgrad(d, st)
            e1.record(); torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 5)
        fl = 2.0 * B * H * H * 9 * Mt * Co
        res[win] = (min(ts), fl / min(ts) / 1e9, splits)
    print("wgrad %-26s " % name + "  ".join("%s %.3fms %4.0fTF (splits %d)" % ("win" if w == 0 else "tiled", *v)
                                           for w, v in res.items()), flush=True)
