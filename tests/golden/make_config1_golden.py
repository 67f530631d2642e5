"""Config-1 golden fixture (BASELINE.json configs[0]): the RRDB generator (conf/generator/esrgan.yaml: nf 64, nb 11,
gc 16, 3 -> 1 channels, x4) trained pixel-loss-only on 32x32 -> 128x128 tiles, batch 2, three optimizer steps with
conf/optimizers/adamw.yaml (lr = training.lr = 1e-4, weight_decay 1e-4) and conf/schedulers/one_cycle_schedule.yaml
(num_training_steps -1 -> inferred from the trainer: limit_train_batches 10, max_epochs 1 -> total_steps 10).

Run in the build container (needs /root/reference; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_config1_golden.py

The generator is the REFERENCE's own ``climsr/models/esrgan.py`` (imported read-only) in float64; the step is
``climsr/task/pl_generator_pre_training.py:18-33`` (hr, sr = common_step; L1; backward; AdamW; OneCycleLR per step,
``core/task.py:173-226`` + ``core/instantiator.py:48-64``: OneCycleLR total_steps = num_training_steps).  Lightning
is not importable here, so its automatic-optimisation order (zero_grad, step, backward, optimizer.step,
scheduler.step) is restated.  Output: tests/golden/config1_steps.json.
"""
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from make_golden import ESRGANGenerator, batch, checks, det_state, load, to64  # noqa: E402

SEEDS = (200, 201, 202)
TOTAL_STEPS = 10


def main():
    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=11, gc=16, scale_factor=4)
    g = load(g, det_state(g)).double().train()
    opt = torch.optim.AdamW(g.parameters(), lr=1e-4, weight_decay=1e-4)
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-4, total_steps=TOTAL_STEPS, epochs=1, pct_start=0.05,
                                              div_factor=2, final_div_factor=100)
    crit = nn.L1Loss()
    rec = {"nb": 11, "batch": 2, "lr_size": 32, "hr_size": 128, "seeds": list(SEEDS), "total_steps": TOTAL_STEPS}
    for s, seed in enumerate(SEEDS):
        bt = to64(batch(2, 128, seed=seed))
        opt.zero_grad()
        sr = g(bt["lr"], bt["elevation"], bt["mask"])
        loss = crit(sr, bt["hr"])
        loss.backward()
        if s == 0:
            rec["grads0"] = checks((k, p.grad) for k, p in g.named_parameters())
        rec.setdefault("loss", []).append(float(loss))
        rec.setdefault("lr", []).append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
        print("step", s, float(loss), flush=True)
    rec["params_after"] = checks(g.named_parameters())
    with open(os.path.join(HERE, "config1_steps.json"), "w") as f:
        json.dump(rec, f)


if __name__ == "__main__":
    main()
