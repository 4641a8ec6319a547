"""Debug: fused vs unfused stride-2 depthwise + BN0/GELU backward on small odd shapes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "ssl-vit-video-analytics_amd")]
import torch
import torch.nn.functional as F
from ssl_mae_amd import kernels as K
torch.manual_seed(0)
dev = "cuda"
for (Fr, H, C, s) in [(4, 19, 64, 2), (4, 20, 64, 2), (4, 19, 64, 1), (3, 30, 32, 2)]:
    W = H
    Ho = (H - 1) // s + 1
    a1 = (torch.randn(Fr * H * W, C, device=dev) * 1.5 + 0.2).to(torch.bfloat16)
    g0 = torch.randn(C, device=dev) * 0.2 + 1.0
    b0 = torch.randn(C, device=dev) * 0.2
    wdw = torch.randn(C, 9, device=dev) * 0.3
    m0, r0 = K.bn_stats(a1)
    act0 = (m0, r0, g0, b0, True)
    da2 = (torch.randn(Fr * Ho * Ho, C, device=dev) * 1e-2).to(torch.bfloat16)
    dw_u = torch.zeros(C, 9, device=dev)
    dh1 = K.dwconv_fused_bwd(da2, a1, act0, wdw, dw_u, Fr, H, W, C, s)
    dg_u, db_u = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    da1_u = K.bn_bwd(dh1, a1, m0, r0, g0, b0, True, dg_u, db_u)
    dw_f = torch.zeros(C, 9, device=dev)
    dg_f, db_f = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    da1_f = K.dwconv_bn_bwd(da2, a1, act0, wdw, dw_f, dg_f, db_f, Fr, H, W, C, stride=s)
    # fp32 reference
    x = a1.float().view(Fr, H, W, C).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    tg, tb = g0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
    tw = wdw.clone().requires_grad_(True)
    u = F.batch_norm(x, None, None, tg, tb, True, 0.0, 1e-5)
    y = F.conv2d(F.gelu(u), tw.view(C, 1, 3, 3), None, s, 1, 1, C)
    y.backward(da2.float().view(Fr, Ho, Ho, C).permute(0, 3, 1, 2))
    rel = lambda a, b: ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
    gx = x.grad.permute(0, 2, 3, 1).reshape(-1, C)
    print(f"F{Fr} H{H} C{C} s{s}: da1 fused {rel(da1_f, gx):.4f} unfused {rel(da1_u, gx):.4f} | dw fused "
          f"{rel(dw_f, tw.grad):.4f} unf {rel(dw_u, tw.grad):.4f} | dg fused {rel(dg_f, tg.grad):.4f} unf "
          f"{rel(dg_u, tg.grad):.4f} | db fused {rel(db_f, tb.grad):.4f} unf {rel(db_u, tb.grad):.4f} | "
          f"fused-vs-unf dg {rel(dg_f, dg_u):.4f}", flush=True)
    # per-pixel error map of da1 (fused vs ref), by row/col parity
    e = (da1_f.float() - gx).abs().view(Fr, H, W, C).amax((0, 3))
    print("   worst rows", e.amax(1).topk(3).indices.tolist(), "worst cols", e.amax(0).topk(3).indices.tolist())
