"""Diagnostic (not collected by pytest): per-tensor gradient error of the native G vs the fp64 oracle."""
import sys
sys.path.insert(0, "/root/repo")
import torch
from oracle import climsr_ref as ref
from tests.helpers import gen_params
from climsr_amd.models.esrgan import ESRGANGenerator
from climsr_amd.losses.l1 import l1_loss

DEV = "cuda"
nb = 1
g = ESRGANGenerator(3, 1, nf=64, nb=nb, gc=16)
g.load_state_dict(gen_params(nb, torch.float32))
g = g.to(DEV)
p64 = gen_params(nb, torch.float64)
bt = ref.synthetic_batch(2, 64, seed=3)
mode = sys.argv[1] if len(sys.argv) > 1 else "l1"
sr = g(bt["lr"].to(DEV), bt["elevation"].to(DEV), bt["mask"].to(DEV))
if mode == "l1":
    loss = l1_loss(sr, bt["hr"].to(DEV))
else:
    loss = (sr * bt["hr"].to(DEV)).mean()
loss.backward()
keys = list(p64.keys())
for k in keys:
    p64[k].requires_grad_(True)
b64 = {k: v.double() for k, v in bt.items()}
sr_ref = ref.generator_forward(p64, b64["lr"], b64["elevation"], b64["mask"], nb)
lref = ref.l1_loss(sr_ref, b64["hr"]) if mode == "l1" else (sr_ref * b64["hr"]).mean()
grads = torch.autograd.grad(lref, [p64[k] for k in keys])
named = dict(g.named_parameters())
for k, gr in zip(keys, grads):
    got = named[k].grad.double().cpu()
    rel = float((got - gr).norm() / (gr.norm() + 1e-30))
    cos = float((got * gr).sum() / (got.norm() * gr.norm() + 1e-30))
    print(f"{k:40s} rel {rel:.3e} cos {cos:.6f} |g| {float(gr.norm()):.3e}")
