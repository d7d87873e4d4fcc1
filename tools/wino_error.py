"""fp32 rounding error of the 1-D Winograd F(2,3) 3x3 convolution vs the direct sum (CPU, torch):
the transform the fp32 Winograd kernel uses (conv3x3.hip), evaluated in fp32 against an fp64 conv2d.

    python tools/wino_error.py
"""
import torch
torch.manual_seed(0)
def direct(x, w):  # x [C,H,W+2 padded], w [Co,C,3,3] ; conv with pad in H done by caller
    return torch.nn.functional.conv2d(x[None], w, padding=1)[0]
def wino(x, w):
    # F(2,3) along W: for each dy, outputs pairs. x: [C,H,W], w [Co,C,3,3]; pad 1
    C,H,W = x.shape
    dt = x.dtype
    xp = torch.nn.functional.pad(x, (1,1,1,1))
    g0,g1,g2 = w[...,0], w[...,1], w[...,2]   # [Co,C,3(dy)]
    U = torch.stack([g0, (g0+g1+g2)*0.5, (g0-g1+g2)*0.5, g2])  # [4,Co,C,3]
    out = torch.zeros(w.shape[0], H, W, dtype=dt)
    M = torch.zeros(4, w.shape[0], H, W//2, dtype=dt)
    for dy in range(3):
        rows = xp[:, dy:dy+H, :]           # [C,H,W+2]
        d = [rows[:, :, j:j+W:2][..., :W//2] for j in range(4)]  # d_j at x=2p+j (padded coords)
        V = [d[0]-d[2], d[1]+d[2], d[2]-d[1], d[1]-d[3]]
        for xi in range(4):
            # M[xi][co,h,p] += sum_c U[xi][co,c,dy] * V[xi][c,h,p]
            M[xi] += torch.einsum('oc,chp->ohp', U[xi][:,:,dy], V[xi])
    out[:, :, 0::2] = M[0]+M[1]+M[2]
    out[:, :, 1::2] = M[1]-M[2]-M[3]
    return out
for C in (64, 256, 512):
    x = torch.relu(torch.randn(C, 32, 32))
    w = torch.randn(C, C, 3, 3) * (2.0/(9*C))**0.5
    ref = direct(x.double(), w.double())
    d32 = direct(x, w).double()
    w32 = wino(x, w).double()
    sc = ref.abs().max()
    rms = lambda e: (e.pow(2).mean().sqrt()/ref.pow(2).mean().sqrt()).item()
    print(C, "direct max %.2e rms %.2e" % (((d32-ref).abs().max()/sc).item(), rms(d32-ref)),
          "wino max %.2e rms %.2e" % (((w32-ref).abs().max()/sc).item(), rms(w32-ref)))
