"""The one-launch step for wide envs (64 < N <= 512): step_flat_vec_kernel (step_flat.h),
fixed 16 KiB tiles of the flat window, the scalar step — the packed scalar step of the
two-launch path (scalar_vec.h: the same loads and reductions, so the same bits) — run by
every tile an env straddles, the state snapshot / halo by parity.

It is checked against the CPU oracle in every mode and over shapes that put the env's end
at every tile position, and bit for bit against the two-launch path through resets, masked
resets, checkpoint restores, window-buffer changes, resident-series days (one past the
series) and caller prices, and at BASELINE config 5's shape (8,192 envs x 500 assets).
Needs an MI355X."""
import zlib

import numpy as np
import pytest
import torch

from test_gpu_parity import DEV, MODES, _gpu, _run_both  # noqa: F401  (_gpu: autouse fixture)

pytestmark = pytest.mark.gpu

# (N, W, B), N * W * F 16-B granular: A = 2 / 4 / 8 strided assets per lane, env windows from
# 16 KiB tiles + a few chunks to 32 tiles, the 512-asset maximum, the smallest window the
# tiles take (W = 14: 60 rows of a tile per env)
SHAPES = [(65, 52, 7), (100, 50, 9), (129, 20, 11), (256, 16, 5), (257, 44, 3), (500, 50, 4),
          (512, 50, 3), (128, 44, 6), (100, 14, 9)]
IMPLS = ["flat"]
KERNEL = {"flat": "step_flat_vec_kernel"}


def _mode_id(k):
    return "-".join(f"{a}={b}" for a, b in k.items()) or "reference"


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("kind", ["simplex", "mixed", "rawpos"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
@pytest.mark.parametrize("kw", MODES, ids=_mode_id)
def test_gpu_wide_vs_oracle_modes(kind, db, kw, impl):
    """Every reward / ring / norm / commission mode, in place and double-buffered, past
    the ring wrap, against the oracle (B = 13 envs of 100 assets: 6,250 chunks each, so
    tiles hold one env or the end of one and the start of the next)."""
    _run_both(kw, B=13, N=100, W=50, T=56, kind=kind, seed=zlib.crc32(f"wide{kw}{kind}{db}".encode()),
              double_buffer=db, impl=impl)


@pytest.mark.parametrize("impl,N,W,B", [(i,) + s for i in IMPLS for s in SHAPES])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_wide_shapes_vs_oracle(impl, N, W, B, db):
    _run_both({}, B=B, N=N, W=W, T=W + 7, kind="mixed", seed=N * 13 + W, double_buffer=db, impl=impl)
    _run_both({"ring": "chrono", "commission": 0.0025}, B=B, N=N, W=W, T=W + 3, kind="simplex", seed=N + 7 * W,
              double_buffer=db, impl=impl)


def test_gpu_wide_paths_refuse_what_they_do_not_cover():
    from pmenv import TradingEnv
    from pmenv._abi import PmenvError
    for impl, n, w in [("flat", 513, 50), ("flat", 100, 12)]:
        with pytest.raises((PmenvError, ValueError)):
            TradingEnv(num_envs=4, num_assets=n, window=w, device=DEV, step_impl=impl)


def _state(e):
    return (e._value.clone(), e._counter.clone(), e._ring.clone(), e._w_new.clone(), e._last_close.clone(),
            e._stat_a.clone(), e._stat_b.clone())


def _same(ga, gb, what):
    for i, (x, y) in enumerate(zip(ga, gb)):
        assert torch.equal(x.nan_to_num(7.0), y.nan_to_num(7.0)), f"{what}: state field {i}"


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("N,W,B", [(100, 50, 9), (300, 20, 5), (500, 50, 3)])
@pytest.mark.parametrize("kw", [dict(), dict(commission=0.0025, reward="sharpe_ratio"),
                                dict(ring="chrono", reward="diff_sharpe")], ids=_mode_id)
def test_gpu_wide_bitwise_vs_two_launch_through_state_changes(N, W, B, kw, impl):
    """The one-launch wide step and the two-launch path, driven with the same inputs through full and
    masked resets, a checkpoint restore, a switch to another path and back, a fresh window
    buffer, in place and double-buffered steps, caller prices and resident-series days,
    agree on every window, reward, returned weight and state field, bit for bit."""
    from pmenv import TradingEnv, synth
    T = W + 24
    ser = synth.series(W + T, B, N, seed=zlib.crc32(f"walk{N}{W}{kw}".encode()), device=DEV)
    act = synth.actions(T, B, N, seed=5, device=DEV)
    kind_mixed = torch.randn(T, B, N, device=DEV, generator=torch.Generator(DEV).manual_seed(3))
    res = synth.series(T + W + 8, 1, N, seed=9, device=DEV)[:, 0].contiguous()
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i, track_info=True, **kw)
            for i in (impl, "two_launch")]
    assert KERNEL[impl] in envs[0].step_path and KERNEL[impl] not in envs[1].step_path
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    cks, obs_cks = [None, None], [None, None]
    rng = np.random.default_rng(N + W)
    for t in range(T):
        a = kind_mixed[t] if t % 5 == 3 else act[t]
        mask9 = torch.as_tensor(rng.random(B) < 0.4, device=DEV) if t == 9 else None
        outs = []
        for i, e in enumerate(envs):
            if mask9 is not None:
                e.reset(obs[i], mask=mask9)
            if t == 14:
                cks[i], obs_cks[i] = e.state_dict(), obs[i].clone()
            if t == 20 and i == 0:
                e.set_step_impl("two_launch")
            if t == 22 and i == 0:
                e.set_step_impl(impl)
            if t == 26:
                e.load_state_dict(cks[i])
                obs[i].copy_(obs_cks[i])
            wo = torch.empty(B, N, device=DEV)
            if t % 4 == 1:
                r, obs[i] = e.step(a, obs[i], bar=ser[W + t], out=torch.empty_like(obs[i]), weights_out=wo)
            elif t % 7 == 5:
                obs[i] = obs[i].clone()
                r, _ = e.step(a, obs[i], bar=ser[W + t], weights_out=wo)
            elif t % 6 == 2:
                day = torch.full((B,), t + W, dtype=torch.int32, device=DEV)
                day[::3] += 2
                day[-1] = 10 ** 6 if t == 8 else day[-1]          # a day past the series: NaN bar
                r, _ = e.step(a, obs[i], series=res, day=day, weights_out=wo)
            elif t % 9 == 4:
                r, _ = e.step(a, obs[i], bar=ser[W + t], prices=ser[W + t, ..., 3] / ser[W + t - 1, ..., 3],
                              weights_out=wo)
            else:
                r, _ = e.step(a, obs[i], bar=ser[W + t], weights_out=wo)
            outs.append((r.clone(), wo, e.info["returns"][-1]))
        assert torch.equal(obs[0].nan_to_num(7.0), obs[1].nan_to_num(7.0)), f"step {t}: windows"
        assert torch.equal(outs[0][0].nan_to_num(7.0), outs[1][0].nan_to_num(7.0)), f"step {t}: rewards"
        assert torch.equal(outs[0][1].nan_to_num(7.0), outs[1][1].nan_to_num(7.0)), f"step {t}: weights"
        assert torch.equal(outs[0][2].nan_to_num(7.0), outs[1][2].nan_to_num(7.0)), f"step {t}: returns"
        _same(_state(envs[0]), _state(envs[1]), f"step {t}")


@pytest.mark.parametrize("impl", IMPLS)
@pytest.mark.parametrize("commission", [0.0, 0.0025])
def test_gpu_wide_config5_shape_bitwise_vs_two_launch(commission, impl):
    """BASELINE config 5's shape (8,192 envs x 500 assets x 50 x 5, differential Sharpe):
    the one-launch step equals the two-launch path bit for bit over the ring wrap, in place."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 8192, 500, 50, 53
    ser = synth.series(W + T, B, N, seed=11, device=DEV)
    act = synth.actions(T, B, N, seed=12, device=DEV)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i, reward="diff_sharpe",
                       commission=commission) for i in (impl, "two_launch")]
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    for t in range(T):
        rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
    assert torch.equal(obs[0], obs[1])
    _same(_state(envs[0]), _state(envs[1]), "end")
