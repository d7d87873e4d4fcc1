"""Per-parameter gradient errors of the smoke() configuration (2 x 3 x S x S, selective) against the
CPU oracle, for debugging: python tools/smoke_debug.py [S]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if os.environ.get("SMOKE_PKG_ROOT"):  # an older build of the package (bisecting)
    sys.path.insert(0, os.environ["SMOKE_PKG_ROOT"])
import selectivenet_for_semantic_segmentation_binary_amd as S  # noqa: E402
import selectivenet_for_semantic_segmentation_binary_amd.layout as L  # noqa: E402
from oracle import unet_b_cpu as O  # noqa: E402
from selectivenet_for_semantic_segmentation_binary_amd.synthetic import make_batch  # noqa: E402

size = int(sys.argv[1]) if len(sys.argv) > 1 else 32
print("package", S.__file__)
x, lab = make_batch(2, size, seed=5)
p = L.seeded_params(0, "RGB", True)
net = S.UNet_B("RGB", selective=True)
with torch.no_grad():
    for k, t in net.named_parameters():
        t.copy_(torch.tensor(p[k]))
net = net.to("cuda:0").train()
xt, lt = torch.tensor(x, device="cuda:0"), torch.tensor(lab, device="cuda:0")
out, sel, aux = net(xt)
sl, cov = S.calc_selective_risk_image_b(out, sel, lt, lamb=2)
loss = S.BCEWithLogitsLoss()(aux, lt) + sl
loss.backward()
torch.cuda.synchronize()
params, buffers = O.make_state(0, "RGB", True)
o2, s2, a2 = O.forward(params, buffers, torch.tensor(x), True, training=True)
for nm, a, b in (("out", out, o2), ("sel", sel, s2), ("aux", aux, a2)):
    print(f"{nm}: max rel {float((a.detach().cpu() - b.detach()).abs().max() / b.detach().abs().max()):.2e}")
sl2, cov2 = O.selective_risk_b_stable(o2, s2, torch.tensor(lab), lamb=2)
loss2 = O.bce_with_logits_mean(a2, torch.tensor(lab)) + sl2
loss2.backward()
print(f"size {size} X2={os.environ.get('SELUNET_X2')} SHIFT={os.environ.get('SELUNET_BN_SHIFT')}: "
      f"loss {loss.item():.7f} oracle {loss2.item():.7f}")
for k, q in net.named_parameters():
    g = params[k].grad
    e = float((q.grad.cpu() - g).abs().max() / (g.abs().max() + 1e-12))
    if e > 1e-5:
        print(f"  {k:40s} {e:.2e}")
