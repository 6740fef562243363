"""The CPU oracle (oracle/pmenv_oracle.c) against golden vectors produced by the
reference env itself (tests/golden/gen_golden.py) — pins the oracle before it is
trusted as the checker of the HIP path."""
import numpy as np
import pytest

import golden_util as gu
from oracle import OracleEnv, gae, moments, philox4x32, synth_series, synth_actions
from pmenv.config import EnvConfig


def replay_oracle(g, mode):
    m = g["meta"]
    N, W, F, T = m["N"], m["W"], m["F"], m["T"]
    env = OracleEnv(EnvConfig(num_envs=1, num_assets=N, window=W, features=F, close_channel=gu.close_channel(g)))
    out = {"rewards": np.full(T + 1, np.nan), "values": np.zeros(T + 1), "rets": np.full(T + 1, np.nan),
           "wpost": np.full((T + 1, N), np.nan), "chans": {}, "market_ok": True}
    obs = None
    for i in range(T + 1):
        if g["ops"][i]:
            obs = gu.window(g, i)
            env.reset(obs)
        else:
            if mode == "surface":
                obs = gu.window(g, i)
                r, ret, w = env.step(g["actions"][i], obs, prices=g["prices"][i].astype(np.float32))
            else:
                r, ret, w = env.step(g["actions"][i], obs, bar=gu.bar(g, i))
                out["market_ok"] &= np.array_equal(obs[..., :-1], gu.window(g, i)[..., :-1])
            out["rewards"][i], out["rets"][i], out["wpost"][i] = r[0], ret[0], w[0]
        out["values"][i] = env.value[0]
        out["chans"][i] = obs[0, :, :, -1].copy()
    return out


def compare(g, out, allow_prefix=True):
    rtol, afloor = gu.tolerances(g)
    L = gu.finite_prefix(g) if allow_prefix else len(g["values"])
    steps = np.nonzero(g["ops"][:L] == 0)[0]
    np.testing.assert_allclose(out["values"][:L], g["values"][:L], rtol=rtol, atol=0)
    np.testing.assert_allclose(out["rets"][steps], g["rets"][steps], rtol=rtol, atol=0)
    err = np.abs(out["rewards"][steps] - g["rewards"][steps])
    tol = rtol * np.abs(g["rewards"][steps]) + afloor
    assert np.all(err <= tol), f"reward err {err.max():.3e} > tol at step {steps[np.argmax(err - tol)]}"
    np.testing.assert_allclose(out["wpost"][steps], g["wpost"][steps], rtol=1e-5, atol=2e-7)
    for k, s in enumerate(g["chan_steps"]):
        if s < L:
            np.testing.assert_allclose(out["chans"][int(s)], g["chans"][k], rtol=1e-5, atol=2e-7,
                                       err_msg=f"weight channel at step {s}")


@pytest.mark.parametrize("name", gu.cases())
@pytest.mark.parametrize("mode", ["surface", "advance"])
def test_oracle_matches_reference(name, mode):
    g = gu.load(name)
    out = replay_oracle(g, mode)
    assert out["market_ok"]
    compare(g, out)


def test_golden_cases_cover_feature_counts():
    """The reference's windows carry len(pool.features) channels (data/data_loader.py:48):
    goldens exist for F != 5, below and above OHLC + weight."""
    fs = {gu.load(n)["meta"]["F"] for n in gu.cases()}
    assert {3, 5, 8, 12} <= fs


PHASES = (("eval0", "test_series", "T_eval"), ("rollout", "train_series", "T_roll"), ("eval1", "test_series", "T_eval"))


def test_oracle_matches_reference_driver_sequence():
    """train/on_policy.py's call sequence (TradingEnv(), evaluate, rollout, evaluate: one env
    object, resets between phases, F = 8 windows) replayed on the oracle."""
    g = gu.load_driver()
    m = g["meta"]
    N, W, F = m["N"], m["W"], m["F"]
    env = OracleEnv(EnvConfig(num_envs=1, num_assets=N, window=W, features=F, close_channel=m["close_channel"]))
    for phase, skey, tkey in PHASES:
        ser, T = g[skey], m[tkey]
        rets, rews, vals = [0.0], [0.0], [env.value[0]]
        for step in range(T + 1):
            obs = np.ascontiguousarray(ser[None, :, step:step + W, :])
            if step == 0:
                env.reset(obs)
                vals = [env.value[0]]
            else:
                r, ret, _ = env.step(g[f"{phase}_actions_in"][step], obs, prices=g[f"{phase}_prices"][step])
                rews.append(r[0])
                rets.append(ret[0])
                vals.append(env.value[0])
        np.testing.assert_allclose(vals, g[f"{phase}_info_values"], rtol=2e-5)
        np.testing.assert_allclose(rets, g[f"{phase}_info_returns"], rtol=2e-5)
        np.testing.assert_allclose(rews, g[f"{phase}_info_rewards"], rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(obs[0, :, :, -1], g[f"{phase}_chan"], rtol=1e-5, atol=2e-7)


def test_reference_reward_module():
    """env/reward.py:20-31 values vs the restated formulas."""
    d = np.load(gu.GOLDEN_DIR + "/reward_module.npz")
    rf = float(d["risk_free_rate"])
    for L in (2, 3, 10, 64):
        v = d[f"values_{L}"]
        ratios = v[1:] / v[:-1]
        assert np.isclose(d[f"returns_{L}"], ratios[-1], rtol=1e-15)
        assert np.isclose(d[f"log_returns_{L}"], np.log(ratios[-1]), rtol=1e-15)
        # Welford restatement used by the kernel / oracle (SHARPE reward)
        mean = m2 = 0.0
        for i, x in enumerate(ratios, 1):
            dx = x - mean
            mean += dx / i
            m2 += dx * (x - mean)
        n = len(ratios)
        sharpe = np.nan if n < 2 else (mean - rf) / np.sqrt(m2 / (n - 1))
        if np.isnan(d[f"sharpe_{L}"]):
            assert np.isnan(sharpe)
        else:
            assert np.isclose(sharpe, d[f"sharpe_{L}"], rtol=1e-9)


def test_oracle_sharpe_reward_matches_reference_formula():
    """SHARPE reward over an env trajectory == reward.py:26-31 on info['values']."""
    g = gu.load("simplex_n5_w50_t64_f64")
    m = g["meta"]
    env = OracleEnv(EnvConfig(num_envs=1, num_assets=m["N"], window=m["W"], reward="sharpe_ratio"))
    obs = gu.window(g, 0)
    env.reset(obs)
    vals = [env.value[0]]
    for i in range(1, 20):
        r, _, _ = env.step(g["actions"][i], obs, bar=gu.bar(g, i))
        vals.append(env.value[0])
        x = np.array(vals)
        x = x[1:] / x[:-1]
        ref = np.nan if len(x) < 2 else (x.mean() - 0.04) / x.std(ddof=1)
        if np.isnan(ref):
            assert np.isnan(r[0])
        else:
            assert np.isclose(r[0], ref, rtol=1e-5)


def test_philox_known_answers():
    """Random123 known-answer vectors for Philox4x32-10."""
    assert list(philox4x32([0, 0, 0, 0], [0, 0])) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert list(philox4x32([0xffffffff] * 4, [0xffffffff] * 2)) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert list(philox4x32([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0])) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


def test_synth_sharding_and_shape():
    full = synth_series(12, 6, 3, env_offset=0)
    part = synth_series(12, 2, 3, env_offset=4)
    assert np.array_equal(full[:, 4:6], part)
    o, h, lo, c = (full[..., i] for i in range(4))
    assert np.all(h >= np.maximum(o, c)) and np.all(lo <= np.minimum(o, c)) and np.all(lo > 0)
    a = synth_actions(5, 6, 7)
    assert np.allclose(a.sum(-1), 1.0, atol=1e-6) and np.all(a > 0)
    assert np.array_equal(a[:, 2:4], synth_actions(5, 2, 7, env_offset=2))


def test_gae_oracle_vs_numpy():
    rng = np.random.default_rng(0)
    T, B = 33, 7
    r = rng.standard_normal((T, B)).astype(np.float32)
    v = rng.standard_normal((T + 1, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.1
    adv, ret = gae(r, v, d, 0.97, 0.9)
    ref = np.zeros((T, B))
    a = np.zeros(B)
    for t in range(T - 1, -1, -1):
        nd = 1.0 - d[t]
        delta = r[t] + 0.97 * nd * v[t + 1] - v[t]
        a = delta + 0.97 * 0.9 * nd * a
        ref[t] = a
    np.testing.assert_allclose(adv, ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret, ref + v[:-1], rtol=1e-5, atol=1e-5)
    x = rng.standard_normal(1001).astype(np.float32)
    mo = moments(x)
    assert mo[0] == 1001 and np.isclose(mo[1], x.astype(np.float64).sum()) and \
        np.isclose(mo[2], (x.astype(np.float64) ** 2).sum())


def _trainer_cases():
    d = np.load(gu.GOLDEN_DIR + "/trainer_reward.npz")
    keys = sorted({k.rsplit("_", 1)[0] for k in d.files if k.endswith("_a")})
    return d, keys


@pytest.mark.parametrize("norm", ["global_or"])
def test_oracle_batch_reward_matches_reference_autograd(norm):
    """PG._reward / A2C._loss (forward + torch autograd grad) run from the reference."""
    from oracle import batch_reward
    d, keys = _trainer_cases()
    assert len(keys) == 60
    for key in keys:
        dt, shape, akind, kind = key.split("_", 3)
        a, v, p = d[key + "_a"], d[key + "_v"], d[key + "_p"]
        R, _, g = batch_reward(a, v, p, reward=kind, norm=norm)
        for tag, sign in (("pg", 1.0), ("a2c", -1.0)):
            r_ref, g_ref = float(d[f"{key}_{tag}_r"]), d[f"{key}_{tag}_grad"]
            # fp32 references: the batch Sharpe divides by a tiny std (ill-conditioned)
            rtol = 1e-9 if dt == "f64" else (1e-3 if kind == "sharpe_ratio" else 2e-5)
            if np.isnan(r_ref):
                assert np.isnan(R), key
                continue
            assert np.isclose(sign * R, r_ref, rtol=rtol, atol=1e-12 if dt == "f64" else 1e-7), (key, tag, R, r_ref)
            scale = np.abs(g_ref).max() + 1e-30
            loose = dt == "f32" and kind == "sharpe_ratio"
            np.testing.assert_allclose(sign * g, g_ref, rtol=1e-6 if dt == "f64" else (3e-2 if loose else 1e-3),
                                       atol=1e-7 * scale if dt == "f64" else (3e-2 if loose else 2e-4) * scale,
                                       err_msg=f"{key} {tag}")
