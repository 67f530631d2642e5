"""Diagnostic (GPU): plain discriminator gradients vs the fp64 oracle, next to the same oracle run under
torch autocast (bf16 / fp16) on the CPU -- the envelope reduced precision alone produces."""
import sys

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

from oracle import climsr_ref as ref  # noqa: E402
from tests.helpers import plain_d_params  # noqa: E402


def grads(p, x, wgt, cast=None):
    keys = ref.trainable_keys(p)
    for k in keys:
        p[k].requires_grad_(True)
    xx = x.clone().requires_grad_(True)
    if cast is None:
        s = ref.plain_discriminator_forward(p, xx, training=True)
    else:
        with torch.autocast("cpu", dtype=cast):
            s = ref.plain_discriminator_forward(p, xx, training=True)
    g = torch.autograd.grad((s.double() * wgt).sum(), [xx] + [p[k] for k in keys])
    return dict(zip(["x"] + keys, [t.double() for t in g]))


def cmp(a, b):
    c = float((a * b).sum() / (a.norm() * b.norm() + 1e-30))
    r = float((a - b).norm() / (b.norm() + 1e-30))
    return c, r


x = ref.synthetic_batch(2, 128, seed=11)["hr"]
wgt = torch.tensor([[0.7], [-1.3]], dtype=torch.float64)
g64 = grads(plain_d_params(torch.float64), x.double(), wgt)
gbf = grads(plain_d_params(torch.float32), x.float(), wgt, torch.bfloat16)
from climsr_amd.models.discriminator import Discriminator  # noqa: E402

d = Discriminator(1)
d.load_state_dict(plain_d_params(torch.float32))
d = d.cuda().train()
xg = x.cuda().requires_grad_(True)
s = d(xg)
(s * wgt.float().cuda()).sum().backward()
torch.cuda.synchronize()
nat = {"x": xg.grad.double().cpu()}
nat.update({k: v.grad.double().cpu() for k, v in d.named_parameters()})
print(f"{'tensor':40s} {'native cos':>10s} {'rel':>8s} | {'bf16-ac cos':>11s} {'rel':>8s}")
for k in g64:
    c1, r1 = cmp(nat[k], g64[k])
    c2, r2 = cmp(gbf[k], g64[k])
    print(f"{k:40s} {c1:10.5f} {r1:8.4f} | {c2:11.5f} {r2:8.4f}")
