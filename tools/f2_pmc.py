"""The batched reward (f2, agent/pg/pg.py:40-82) forward + backward of the product library,
`--calls` times per shape, for rocprofv3 kernel-trace / PMC passes (tools/run_r04_f2pmc.sh):
what bounds batch_reward_rows_quad_kernel (VALU issue or memory) at 65,536 and 16,384 rows.

    python tools/f2_pmc.py --shapes 65536x30,16384x30 --calls 20
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="65536x30,16384x30")
ap.add_argument("--calls", type=int, default=20)
ap.add_argument("--kind", default="log_returns")
a = ap.parse_args()
dev = torch.device("cuda:0")
lib = _abi.load()
kind = _abi.REWARD_KINDS[a.kind]
st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
for shp in a.shapes.split(","):
    B, N = (int(x) for x in shp.split("x"))
    g = torch.Generator(device=dev).manual_seed(B + N)
    act = torch.randn(B, N, device=dev, generator=g)
    v = 25000 * torch.exp(0.1 * torch.randn(B, device=dev, generator=g))
    p = 1 + 0.01 * torch.randn(B, N, device=dev, generator=g)
    go = torch.ones((), device=dev)
    work = torch.empty(lib.pmenv_batch_reward_workspace(B) // 8, dtype=torch.float64, device=dev)
    rew = torch.empty((), device=dev)
    grad = torch.empty(B, N, device=dev)
    for _ in range(a.calls):
        assert lib.pmenv_batch_reward_forward(act.data_ptr(), v.data_ptr(), p.data_ptr(), B, N, kind, 0, 1.0,
                                              work.data_ptr(), rew.data_ptr(), None, st) == 0
        assert lib.pmenv_batch_reward_backward(act.data_ptr(), v.data_ptr(), p.data_ptr(), B, N, kind, 1.0,
                                               work.data_ptr(), go.data_ptr(), grad.data_ptr(), st) == 0
    torch.cuda.synchronize()
    print(f"# {shp} reward {float(rew):.6f}", flush=True)
