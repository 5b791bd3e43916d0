"""Diagnostic of the register-prefetched window chunk loop (conv_win.h PF): per-chunk
contributions against the single-buffered kernel (prints max |diff|)."""
import torch
import torch.nn.functional as F
from unet_distributed_amd import native


def main():
    C = native.require()
    dev = torch.device("cuda:0")
    st = int(torch.cuda.current_stream().cuda_stream)
    torch.manual_seed(0)
    for (N, H, C1, Co) in [(2, 64, 64, 64), (2, 32, 64, 64), (2, 16, 128, 64), (2, 64, 64, 32)]:
        x = F.relu(torch.randn(N, H, H, C1, device=dev)).bfloat16()
        w = (torch.randn(Co, 9 * C1, device=dev) * 0.1).bfloat16()
        kp = (9 * C1 + 63) // 64 * 64
        wp = torch.zeros(Co, kp, device=dev, dtype=torch.bfloat16)
        wp[:, :9 * C1] = w
        b = torch.randn(Co, device=dev)
        for extra in (dict(relu=1), dict(bias=int(b.data_ptr())), dict(bias=int(b.data_ptr()), relu=1),
                      dict(relu=1, relu_bits=1)):
            outs = []
            for pf in (0, 1):
                y = torch.full((N, H, H, Co), 7.0, device=dev, dtype=torch.bfloat16)
                bits = torch.zeros(N * H * H * Co // 8, device=dev, dtype=torch.uint8)
                ex = dict(extra)
                if "relu_bits" in ex:
                    ex["relu_bits"] = int(bits.data_ptr())
                C.conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, src1=int(x.data_ptr()),
                                wgt=int(wp.data_ptr()), Cout=Co, dst1=int(y.data_ptr()), win_pf=pf, **ex), st)
                torch.cuda.synchronize()
                outs.append(y.float())
            print("  %s: max|pf0-pf1|=%.4g" % (sorted(extra), (outs[0] - outs[1]).abs().max().item()), flush=True)
        for zero in (None,):
            xx = x.clone()
            if zero == "lo":
                xx[..., :32] = 0
            elif zero == "hi":
                xx[..., 32:] = 0
            outs = []
            for pf in (0, 1):
                y = torch.full((N, H, H, Co), 7.0, device=dev, dtype=torch.bfloat16)
                C.conv_fwd(dict(N=N, OH=H, OW=H, IH=H, IW=H, KH=3, KW=3, pad=1, C1=C1, src1=int(xx.data_ptr()),
                                wgt=int(wp.data_ptr()), Cout=Co, dst1=int(y.data_ptr()), win_pf=pf), st)
                torch.cuda.synchronize()
                outs.append(y.float())
            d = (outs[0] - outs[1]).abs().max().item()
            print("N=%d H=%d C1=%d Co=%d zero=%s  max|pf0-pf1|=%.4g  |pf0|max=%.3g |pf1|max=%.3g" % (
                N, H, C1, Co, zero, d, outs[0].abs().max().item(), outs[1].abs().max().item()), flush=True)


if __name__ == "__main__":
    main()
