"""Diagnostic (GPU, not collected by pytest): config 1 (nb 11, B 2, 32->128) first-step gradients of the native
generator vs the fp64 oracle and the oracle's autocast fp16 / bf16 runs, per tensor, worst ratios first; then the same
for the update vectors of three AdamW steps.  python tools/diag_config1.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import climsr_ref as ref  # noqa: E402
from tests.helpers import gemm_conv, gen_params, rel_l2  # noqa: E402


def main():
    from climsr_amd.losses.l1 import l1_loss
    from climsr_amd.models.esrgan import ESRGANGenerator

    want = json.load(open(os.path.join(ROOT, "tests", "golden", "config1_steps.json")))
    nb, b, hr = want["nb"], want["batch"], want["hr_size"]
    p64 = gen_params(nb, torch.float64)
    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
    g.load_state_dict({k: v.float() for k, v in p64.items()})
    g = g.cuda()
    bt = {k: v.cuda() for k, v in ref.synthetic_batch(b, hr, seed=want["seeds"][0]).items()}
    l1_loss(g(bt["lr"], bt["elevation"], bt["mask"]), bt["hr"]).backward()
    native = {k: p.grad.double().cpu() for k, p in g.named_parameters()}
    keys = list(p64.keys())

    def grads(dev, dtype, autocast=None):
        p = {k: v.to(dev, dtype).requires_grad_(True) for k, v in p64.items()}
        b_ = {k: v.to(dev, dtype) for k, v in ref.synthetic_batch(b, hr, seed=want["seeds"][0], dtype=torch.float64).items()}
        if autocast is None:
            loss = ref.l1_loss(ref.generator_forward(p, b_["lr"], b_["elevation"], b_["mask"], nb), b_["hr"])
        else:
            with torch.autocast("cuda", dtype=autocast):
                loss = ref.l1_loss(ref.generator_forward(p, b_["lr"], b_["elevation"], b_["mask"], nb).float(), b_["hr"])
        gs = torch.autograd.grad(loss, [p[k] for k in keys])
        return {k: v.double().cpu() for k, v in zip(keys, gs)}

    g64 = grads("cpu", torch.float64)
    ref._conv = gemm_conv
    amps = [grads("cuda", torch.float32, dt) for dt in (torch.float16, torch.bfloat16)]
    rows = []
    for k in keys:
        r = rel_l2(native[k], g64[k])
        ra = max(rel_l2(a[k], g64[k]) for a in amps)
        rows.append((r / max(ra, 1e-12), k, r, ra, int(native[k].numel())))
    rows.sort(reverse=True)
    print("first-step gradients: native rel L2 vs fp64 / worst autocast rel L2 (ratio, tensor, native, autocast, numel)")
    for row in rows[:15]:
        print("  %.2f %-40s %.3e %.3e %d" % row)
    k = "srcnn.conv1.bias"
    print(k, "native", native[k][:8].tolist())
    print(k, "fp64  ", g64[k][:8].tolist())
    print(k, "amp16 ", amps[0][k][:8].tolist())


if __name__ == "__main__":
    main()
