"""Eager launches of the fused RDB chain (forward + pull) for rocprofv3 counter passes."""
import sys

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import BatchedPacker, ConvPlan, RdbChain  # noqa: E402

dev, n, dc = "cuda", 32, 128
dense = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
dz = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
plans = []
for k in range(1, 6):
    cin, cout = 64 + 16 * (k - 1), (16 if k < 5 else 64)
    p = ConvPlan(cin, cout, 3, 1, None, f"conv{k}")
    p.bind((torch.randn(cout, cin, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(cout, device=dev), need_t=False)
    plans.append(p)
chain = RdbChain(plans, "prof")
BatchedPacker(plans, torch.device(dev), chain.pack_descs()).run()
pd = chain.pull_descs()
arr = (_lib.PullPackDesc * len(pd))(*pd)
tab = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
_lib.check(_lib.load().climsr_pack_pull_weights_batched(tab.data_ptr(), len(pd), 16 * 9 * 128, _lib.stream_ptr()), "pack")
for _ in range(3):
    chain.forward(dense, dc, n, 64, 64)
    chain.pull(dz, dense, dc, n, 64, 64)
torch.cuda.synchronize()
print("ok")
