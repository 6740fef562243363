"""The reference's own training driver swaps pmenv's TradingEnv in unchanged.

train/on_policy.py:35 builds `TradingEnv()` with no arguments, hands the same object to
Metrics and Visualizer (:39-40), and drives it with the data loader's CPU tensors:
_evaluate (:76-90), _rollout (:56-67, RolloutBuffer.add(s, a, np.array(env.value), r)),
_evaluate again. Metrics reads env.info["returns" / "values" / "actions"]
(util/eval.py:14-37) and Visualizer unpacks env.info.values() in order (util/plot.py:61,
74-75). tests/golden/onpolicy_driver.npz records that sequence run on the reference
itself with F = 8 feature channels (len(pool.features), data/data_loader.py:48) at
config/base.py's NUM_ASSETS = WINDOW_SIZE = 32. Needs an MI355X.
"""
import numpy as np
import pandas as pd
import pytest
import torch

import golden_util as gu

pytestmark = pytest.mark.gpu

PHASES = (("eval0", "test_series", "T_eval"), ("rollout", "train_series", "T_roll"), ("eval1", "test_series", "T_eval"))
# the reference stores the value and the return in the fp32 of its tensors; pmenv computes
# them in f64 and keeps that precision (same container types and shapes)
FLOAT_OK = {"float32", "float64"}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(0)


def _tname(x):
    kind = type(x).__name__
    dt = str(x.dtype).replace("torch.", "") if hasattr(x, "dtype") else None
    shape = "x".join(map(str, tuple(x.shape))) if hasattr(x, "shape") else None
    return kind, dt, shape


def _same_types(got, want):
    """Entry types of one info list against the reference's ('int', 'Tensor:float32:32', ...)."""
    assert len(got) >= len(want)
    for x, w in zip(got, want):
        parts = w.split(":")
        kind, dt, shape = _tname(x)
        assert kind == parts[0], (kind, w)
        if len(parts) > 1:
            assert dt == parts[1] or {dt, parts[1]} <= FLOAT_OK, (dt, w)
            assert shape == parts[2], (shape, w)


def test_gpu_onpolicy_driver_sequence_unchanged():
    from pmenv import TradingEnv
    g = gu.load_driver()
    m = g["meta"]
    N, W, F = m["N"], m["W"], m["F"]
    env = TradingEnv()                                   # on_policy.py:35, no arguments
    held = env                                           # Metrics(self.env, ...) / Visualizer(..., self.env, ...)
    assert float(env.value) == g["init_value"]
    _same_types([v[0] for v in env.info.values()], [t[0] for t in g["init_info_types"].values()])
    for phase, skey, tkey in PHASES:
        series, T = g[skey], m[tkey]
        acts, prices = g[f"{phase}_actions_in"], g[f"{phase}_prices"]
        rewards, values, buf_v = np.full(T + 1, np.nan), np.zeros(T + 1), np.full(T + 1, np.nan)
        rew_tot = 0
        s = None
        for step in range(T + 1):                        # for step, (datetime, prices, data) in enumerate(dl)
            data = torch.tensor(series[:, step:step + W, :])
            if step == 0:
                s = env.reset(data)
                assert s is data
            else:
                a = torch.tensor(acts[step]).reshape(N, 1)          # agent.act(s): [N, 1]
                r, s_ = env.step(a, data, torch.tensor(prices[step]))
                assert s_ is data and r.dim() == 0 and r.device.type == "cpu"
                rew_tot += r
                rewards[step] = float(r)
                if phase == "rollout":
                    buf_v[step] = float(np.array(env.value))        # RolloutBuffer.add (rollout_buffer.py:55)
                s = s_
            values[step] = float(env.value)
        assert env.cfg.features == F and env.cfg.num_assets == N and env.cfg.window == W
        info = held.info
        # util/plot.py:61 unpacks the dict in the reference's order; :74-75 np.array the lists
        assert list(info.keys()) == ["values", "actions", "rewards", "returns"]
        vals, wts, rews, rets = info.values()
        for k, got in info.items():
            _same_types(got[:2], g[f"{phase}_info_types"][k])
        assert len(vals) == len(wts) == len(rews) == len(rets) == T + 1
        # util/eval.py:14-30: DataFrames indexed by the last len(...) dates
        dates = pd.date_range("2020-01-01", periods=T + 1, freq="D")
        df_ret = pd.DataFrame(info["returns"], index=dates[-len(info["returns"]):])
        df_val = pd.DataFrame(info["values"], index=dates[-len(info["values"]):])
        weights = np.array(info["actions"])                          # eval.py:33
        assert weights.shape == (T + 1, N)
        # fp32 reference vs f64 pmenv (golden_util.tolerances for f32 cases)
        np.testing.assert_allclose(df_val.to_numpy()[:, 0].astype(np.float64), g[f"{phase}_info_values"], rtol=2e-5)
        np.testing.assert_allclose(df_ret.to_numpy()[:, 0].astype(np.float64), g[f"{phase}_info_returns"], rtol=2e-5)
        np.testing.assert_allclose(np.array(rews, dtype=np.float64), g[f"{phase}_info_rewards"], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(weights, g[f"{phase}_info_actions"], rtol=1e-5, atol=2e-7)
        np.testing.assert_allclose(rewards[1:], g[f"{phase}_rewards"][1:], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(values, g[f"{phase}_values"], rtol=2e-5)
        if phase == "rollout":
            np.testing.assert_allclose(buf_v[1:], g["rollout_buffer_value"][1:], rtol=2e-5)
        # eval.py:32-37 average turnover and :50 the final value's format
        turn = sum(np.sum(np.abs(weights[i] - weights[i - 1])) for i in range(1, len(weights))) / (len(weights) - 1)
        wref = g[f"{phase}_info_actions"]
        tref = sum(np.sum(np.abs(wref[i] - wref[i - 1])) for i in range(1, len(wref))) / (len(wref) - 1)
        assert np.isclose(turn, tref, rtol=1e-5)
        final = f"{info['values'][-1]:.2f}"                            # eval.py:50 formats a 0-dim tensor
        assert abs(float(final) - g[f"{phase}_info_values"][-1]) <= 0.01 + 2e-5 * g[f"{phase}_info_values"][-1]
        np.testing.assert_allclose(s[:, :, -1].numpy(), g[f"{phase}_chan"], rtol=1e-5, atol=2e-7)
        assert np.array_equal(s[:, :, :-1].numpy(), series[:, T:T + W, :-1])
        assert np.isclose(float(rew_tot), np.nansum(g[f"{phase}_rewards"]), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("name", [n for n in gu.cases() if n.startswith("feat")])
def test_gpu_feature_count_bound_by_first_reset(name):
    """F != 5 windows through TradingEnv() with no arguments: the first reset binds N, W
    and F (and the close channel), surface contract with host tensors, reference goldens."""
    from pmenv import TradingEnv
    from test_oracle_golden import compare
    g = gu.load(name)
    mt = g["meta"]
    N, W, F, T = mt["N"], mt["W"], mt["F"], mt["T"]
    env = TradingEnv()
    out = {"rewards": np.full(T + 1, np.nan), "values": np.zeros(T + 1), "rets": np.full(T + 1, np.nan),
           "wpost": np.full((T + 1, N), np.nan), "chans": {}, "market_ok": True}
    for i in range(T + 1):
        obs = torch.tensor(gu.window(g, i)[0])
        if g["ops"][i]:
            env.reset(obs)
        else:
            r, obs2 = env.step(torch.tensor(g["actions"][i]).reshape(N, 1), obs, torch.tensor(g["prices"][i]))
            assert obs2 is obs
            out["rewards"][i] = float(r)
            out["rets"][i] = float(env.info["returns"][-1])
            out["wpost"][i] = env.info["actions"][-1]
        out["values"][i] = float(env.value)
        out["chans"][i] = obs[:, :, -1].numpy()
    assert (env.cfg.num_assets, env.cfg.window, env.cfg.features) == (N, W, F)
    compare(g, out)


@pytest.mark.parametrize("B,N,W,F", [(1, 32, 32, 5), (1, 5, 50, 5), (3, 7, 10, 3), (2, 30, 50, 8)])
def test_gpu_host_io_direct_equals_staged_bitwise(B, N, W, F):
    """pmenv_step_host (action, prices and the last closes in through mapped staging, the
    [N, W] channel out) gives bitwise what round 4's whole-window staging gave: rewards,
    values, returns, post-drift weights and every float of the caller's window, through
    a reset mid-run and past the ring's wrap."""
    from pmenv import TradingEnv
    rng = np.random.default_rng(B * 1000 + N)
    T = 2 * W + 5
    shape = (N, W, F) if B == 1 else (B, N, W, F)
    wins = rng.uniform(0.5, 1.5, (T + 1,) + shape).astype(np.float32)
    acts = rng.standard_normal((T + 1, B, N)).astype(np.float32)
    acts[::3] = np.abs(acts[::3])                              # raw positive: the AND rule keeps them
    prices = rng.uniform(0.95, 1.05, (T + 1, B, N)).astype(np.float32)
    res = []
    for direct in (True, False):
        env = TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device="cuda:0", track_info=True)
        env._HOST_DIRECT = direct
        rec = {"r": [], "v": [], "win": []}
        for t in range(T + 1):
            x = torch.tensor(wins[t])
            if t in (0, W + 2):
                env.reset(x)
            else:
                r, y = env.step(torch.tensor(acts[t]).reshape(shape[:-2] + (1,)) if B == 1 else torch.tensor(acts[t]),
                                x, torch.tensor(prices[t]))
                assert y is x and r.device.type == "cpu"
                rec["r"].append(r.numpy().copy())
            rec["v"].append(np.array(env.value, dtype=np.float64).copy())
            rec["win"].append(x.numpy().copy())
        inf = env.info
        rec["info"] = [np.array([np.asarray(e, dtype=np.float64) for e in inf[k][1:]]) for k in inf]
        res.append(rec)
    d, s = res
    for key in ("r", "v", "win"):
        for a, b in zip(d[key], s[key]):
            assert np.array_equal(np.atleast_1d(a).view(np.uint8), np.atleast_1d(b).view(np.uint8)), key
    for a, b in zip(d["info"], s["info"]):
        assert np.array_equal(a, b)


def test_gpu_host_io_resident_across_idle_exits_and_device_steps():
    """pmenv_step_host runs in one resident workgroup (no launch per call) that exits after
    20 ms without a call and is relaunched on the next; device-tensor steps of the same handle
    run between host steps. Bitwise what the staged path gives for the same sequence."""
    import time
    from pmenv import TradingEnv
    N, W, F, T = 7, 12, 5, 40
    rng = np.random.default_rng(77)
    wins = rng.uniform(0.5, 1.5, (T + 1, N, W, F)).astype(np.float32)
    acts = rng.standard_normal((T + 1, N)).astype(np.float32)
    prices = rng.uniform(0.95, 1.05, (T + 1, N)).astype(np.float32)
    res = []
    for direct in (True, False):
        env = TradingEnv(num_envs=1, num_assets=N, window=W, features=F, device="cuda:0")
        env._HOST_DIRECT = direct
        rec = []
        for t in range(T + 1):
            x = torch.tensor(wins[t])
            if t == 0:
                env.reset(x)
                continue
            if t % 9 == 4:                                   # the resident workgroup exits idle
                time.sleep(0.03)
            if t % 7 == 3:                                   # a device-tensor step on the same handle
                xd = x.to("cuda:0")
                r, _ = env.step(torch.tensor(acts[t]).reshape(N, 1).to("cuda:0"), xd, torch.tensor(prices[t]).to("cuda:0"))
                x = xd.cpu()
            else:
                r, _ = env.step(torch.tensor(acts[t]).reshape(N, 1), x, torch.tensor(prices[t]))
            v = torch.as_tensor(env.value).detach().to("cpu", torch.float64).numpy().copy()
            rec.append((r.detach().cpu().numpy().copy(), v, x.numpy().copy()))
        res.append(rec)
    for (ra, va, xa), (rb, vb, xb) in zip(*res):
        assert np.array_equal(np.atleast_1d(ra).view(np.uint8), np.atleast_1d(rb).view(np.uint8))
        assert np.array_equal(np.atleast_1d(va).view(np.uint8), np.atleast_1d(vb).view(np.uint8))
        assert np.array_equal(xa.view(np.uint8), xb.view(np.uint8))


def test_gpu_given_dims_are_checked_against_the_first_tensor():
    """A dimension the constructor fixes is not rebound: a window of another shape raises
    ValueError (as the reference's fixed-size ring fails on it)."""
    from pmenv import TradingEnv
    env = TradingEnv(num_assets=7)
    with pytest.raises(ValueError):
        env.reset(torch.zeros(5, 10, 3))
    env = TradingEnv(num_assets=7)
    env.reset(torch.zeros(7, 10, 3))
    assert (env.cfg.num_assets, env.cfg.window, env.cfg.features, env.cfg.close_channel) == (7, 10, 3, 1)
    with pytest.raises(ValueError):                      # bound now: a later window must match
        env.step(torch.full((7, 1), 1 / 7), torch.zeros(7, 12, 3), torch.ones(7))


def test_gpu_batched_shape_bound_by_first_device_window():
    """TradingEnv(device=...) with a [B, N, W, F] device window binds B too; info is then
    opt-in (not kept for B > 1 unless asked)."""
    from pmenv import TradingEnv
    env = TradingEnv(device="cuda:0")
    obs = torch.rand(64, 32, 50, 5, device="cuda:0")
    env.reset(obs)
    assert env.num_envs == 64 and env.info is None
    r, o = env.step(torch.full((64, 32), 1 / 32, device="cuda:0"), obs, torch.ones(64, 32, device="cuda:0"))
    assert o is obs and r.shape == (64,)
    torch.testing.assert_close(env.value, torch.full((64,), 25000.0, dtype=torch.float64, device="cuda:0"))
