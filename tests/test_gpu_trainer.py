"""HIP batched trainer reward (pmenv.trainer, through the C ABI) vs the reference's
PG._reward / A2C._loss autograd vectors and vs the CPU oracle. Needs an MI355X."""
import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import batch_reward as or_batch_reward

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(DEV)


def test_gpu_batch_reward_matches_reference_autograd():
    from pmenv.trainer import pg_reward, a2c_loss
    d = np.load(gu.GOLDEN_DIR + "/trainer_reward.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_a")})
    for key in keys:
        dt, shape, akind, kind = key.split("_", 3)
        B, N = (int(x) for x in shape.split("x"))
        for tag, fn in (("pg", pg_reward), ("a2c", a2c_loss)):
            a = torch.tensor(d[key + "_a"], device=DEV).reshape(B, N, 1).requires_grad_(True)
            v = torch.tensor(d[key + "_v"], device=DEV).reshape(B, 1, 1)
            p = torch.tensor(d[key + "_p"], device=DEV).reshape(B, N, 1)
            r = fn(a, v, None, p, reward=kind)
            r.backward()
            r_ref, g_ref = float(d[f"{key}_{tag}_r"]), d[f"{key}_{tag}_grad"]
            if np.isnan(r_ref):
                assert torch.isnan(r), key
                continue
            loose = dt == "f32" and kind == "sharpe_ratio"
            rtol = 1e-6 if dt == "f64" else (1e-3 if loose else 2e-5)   # the op returns fp32
            assert np.isclose(float(r.detach()), r_ref, rtol=rtol, atol=1e-12 if dt == "f64" else 1e-7), \
                (key, tag, float(r.detach()), r_ref)
            g = a.grad.reshape(B, N).cpu().numpy()
            scale = np.abs(g_ref).max() + 1e-30
            np.testing.assert_allclose(g, g_ref, rtol=1e-5 if dt == "f64" else (3e-2 if loose else 1e-3),
                                       atol=(1e-6 if dt == "f64" else 3e-2 if loose else 2e-4) * scale,
                                       err_msg=f"{key} {tag}")


@pytest.mark.parametrize("B,N", [(65536, 30), (4096, 500), (7, 64), (5, 65), (33, 129), (17, 256), (3, 700), (1, 3),
                                 (64, 30), (64, 8), (65, 30)])   # B <= 64, N <= 64: the one-workgroup forward
@pytest.mark.parametrize("kind", ["log_returns", "returns", "sharpe_ratio"])
@pytest.mark.parametrize("norm", ["global_or", "row_or", "none"])
def test_gpu_batch_reward_vs_oracle(B, N, kind, norm):
    from pmenv.trainer import batch_reward
    rng = np.random.default_rng(B + N)
    a_np = rng.standard_normal((B, N)).astype(np.float32)
    if norm != "global_or":
        a_np[::2] = np.abs(a_np[::2]) / np.abs(a_np[::2]).sum(1, keepdims=True)   # some rows on the simplex
    v_np = (25000.0 * np.exp(0.1 * rng.standard_normal(B))).astype(np.float32)
    p_np = (1.0 + 0.01 * rng.standard_normal((B, N))).astype(np.float32)
    a = torch.tensor(a_np, device=DEV).reshape(B, N, 1).requires_grad_(True)
    r, ret = batch_reward(a, torch.tensor(v_np, device=DEV), torch.tensor(p_np, device=DEV).reshape(B, N, 1),
                          reward=kind, norm=norm, return_ret=True)
    (2.0 * r).backward()
    R, oret, og = or_batch_reward(a_np, v_np, p_np, reward=kind, norm=norm)
    assert np.isclose(float(r.detach()), np.float32(R), rtol=1e-6, atol=1e-12, equal_nan=True), (float(r.detach()), R)
    np.testing.assert_allclose(ret.cpu().numpy(), oret, rtol=1e-7, atol=0)
    g = a.grad.reshape(B, N).cpu().numpy()
    np.testing.assert_allclose(g, 2.0 * og, rtol=1e-5, atol=1e-6 * (np.abs(og).max() + 1e-30))


def test_gpu_batch_reward_trains_like_reference_update():
    """One PG.update-style step (pg.py:96-103): loss = -reward, backward, Adam step —
    the policy gradient reaches the parameters through the fused op."""
    from pmenv.trainer import pg_reward
    torch.manual_seed(0)
    B, N = 64, 30
    lin = torch.nn.Linear(8, 1).to(DEV)
    opt = torch.optim.Adam(lin.parameters(), lr=1e-3)
    x = torch.randn(B, N, 8, device=DEV)
    v = torch.full((B, 1, 1), 25000.0, device=DEV)
    p = 1.0 + 0.01 * torch.randn(B, N, 1, device=DEV)
    w0 = lin.weight.detach().clone()
    opt.zero_grad()
    loss = -pg_reward(lin(x), v, None, p)
    loss.backward()
    assert lin.weight.grad is not None and torch.isfinite(lin.weight.grad).all()
    ref_loss = -torch.log((torch.softmax(lin(x), dim=1) * p).sum(1)).mean()
    ref_loss.backward()
    opt.step()
    assert abs(float(loss) - float(ref_loss)) < 1e-6 and not torch.equal(w0, lin.weight)


@pytest.mark.parametrize("B,N", [(65536, 30), (8192, 500), (3, 20)])
def test_gpu_batch_reward_forward_is_deterministic(B, N):
    """The forward folds per-block partials in a fixed order: repeated calls on one
    workspace pre-filled with garbage give the same bits, and match the oracle."""
    import ctypes
    from pmenv import _abi
    lib = _abi.load()
    g = torch.Generator(device=DEV).manual_seed(B + N)
    a = torch.randn(B, N, device=DEV, generator=g)
    v = torch.rand(B, device=DEV, generator=g) + 1.0
    p = 1.0 + 0.01 * torch.randn(B, N, device=DEV, generator=g)
    work = torch.full((lib.pmenv_batch_reward_workspace(B) // 8,), float("nan"), dtype=torch.float64, device=DEV)
    work.view(torch.int32)[::3] = 0x7ffffff3                  # garbage
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = []
    for kind in (0, 2):
        for _ in range(5):
            r = torch.empty((), device=DEV)
            assert lib.pmenv_batch_reward_forward(P(a), P(v), P(p), B, N, kind, 0, 1.0, P(work), P(r), None, s) == 0
            outs.append((kind, r.clone(), work[6 * B:6 * B + 5].clone()))
    torch.cuda.synchronize()
    for kind in (0, 2):
        ref = [o for o in outs if o[0] == kind]
        for o in ref[1:]:
            assert torch.equal(o[1], ref[0][1]) and torch.equal(o[2], ref[0][2]), kind
        R, _, _ = or_batch_reward(a.cpu().numpy(), v.cpu().numpy(), p.cpu().numpy(),
                                  reward="log_returns" if kind == 0 else "sharpe_ratio", norm="global_or")
        assert np.isclose(float(ref[0][1]), np.float32(R), rtol=1e-6, atol=1e-12), (kind, float(ref[0][1]), R)


@pytest.mark.parametrize("B,N,norm", [(300, 129, "global_or"), (64, 500, "row_or"), (33, 65, "none")])
def test_gpu_batch_reward_backward_without_per_row_returns(B, N, norm):
    """The backward takes each row's normalisation choice from the forward's workspace
    itself: with or without the per-row returns requested, the gradients are the same."""
    from pmenv.trainer import batch_reward
    rng = np.random.default_rng(B * N)
    a_np = rng.standard_normal((B, N)).astype(np.float32)
    a_np[::3] = np.abs(a_np[::3]) / np.abs(a_np[::3]).sum(1, keepdims=True)
    v = torch.tensor((25000.0 * np.exp(0.1 * rng.standard_normal(B))).astype(np.float32), device=DEV)
    p = torch.tensor((1.0 + 0.01 * rng.standard_normal((B, N))).astype(np.float32), device=DEV).reshape(B, N, 1)
    grads = []
    for want in (False, True):
        a = torch.tensor(a_np, device=DEV).reshape(B, N, 1).requires_grad_(True)
        out = batch_reward(a, v, p, reward="sharpe_ratio", norm=norm, return_ret=want)
        (out[0] if want else out).backward()
        grads.append(a.grad.clone())
    assert torch.equal(grads[0], grads[1])
    _, _, og = or_batch_reward(a_np, v.cpu().numpy(), p.reshape(B, N).cpu().numpy(), reward="sharpe_ratio", norm=norm)
    np.testing.assert_allclose(grads[0].reshape(B, N).cpu().numpy(), og, rtol=1e-5, atol=1e-6 * (np.abs(og).max() + 1e-30))


def test_gpu_batch_reward_bits_match_the_library_of_record():
    """Kernel rewrites of the batched reward must not move a bit: the reward, per-row
    returns and gradient at every row form (quad EPL 8 / 16, wave form), reward kind and
    norm mode, over simplex, raw and NaN-holding batches, against the fingerprints the
    round-4 library of record wrote (tools/f2_bits.py -> tests/golden/f2_bits.json)."""
    import json
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import f2_bits
    want = json.load(open(os.path.join(gu.GOLDEN_DIR, "f2_bits.json")))
    got = f2_bits.fingerprints(str(DEV))
    assert set(got) == set(want)
    bad = sorted(k for k in want if got[k] != want[k])
    assert not bad, f"{len(bad)} of {len(want)} fingerprints moved, e.g. {bad[:5]}"
