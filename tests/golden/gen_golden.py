"""Generate golden vectors by running the REFERENCE env (zachramsey/pm-rl) itself.

Run in the build container only (it reads /root/reference at run time; nothing it
reads is copied into this repository — the outputs are data):

    python tests/golden/gen_golden.py            # writes tests/golden/*.npz

Loader notes:
  * config constants bind at import (weight_buffer.py:1, trading_env.py:1), so
    config.base.WINDOW_SIZE / NUM_ASSETS are patched before each (re)import;
  * env/sim/trading_env.py:115 is a PEP 701 f-string inside the dead
    `log_info` method that Python 3.10 cannot compile; the source text is read,
    that one line is replaced by `pass`, and the module is compiled under its
    original filename. reset()/step() are untouched;
  * fp64 goldens use torch.set_default_dtype(torch.float64) before the env is
    built, so the ring and every step op run in f64.

Data alignment follows the reference's intended loop (train/on_policy.py:59-67 with
data/instrument.py:79 and :339-356): at loop index i the env gets
window_i = series[:, i:i+W] and prices_i = fl32(close[i+W-1] / close[i+W-2]).
"""
import json
import os
import sys
import types

import numpy as np

sys.dont_write_bytecode = True  # never write __pycache__ into the read-only reference
REF = os.environ.get("PMRL_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def load_reference(W, N, commission=0.0):
    import torch  # noqa: F401
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import config.base as cb
    cb.WINDOW_SIZE, cb.NUM_ASSETS, cb.COMISSION = W, N, commission
    for m in ["env.sim.weight_buffer", "env.reward", "env.sim.trading_env"]:
        sys.modules.pop(m, None)
    import env.sim.weight_buffer  # noqa: F401  (binds W, N)
    import env.reward  # noqa: F401
    path = os.path.join(REF, "env/sim/trading_env.py")
    lines = open(path).read().split("\n")
    assert "self.info[" in lines[114] and lines[114].lstrip().startswith("f.write(f"), lines[114]
    indent = lines[114][: len(lines[114]) - len(lines[114].lstrip())]
    lines[114] = indent + "pass"
    mod = types.ModuleType("env.sim.trading_env")
    mod.__file__ = path
    exec(compile("\n".join(lines), path, "exec"), mod.__dict__)
    sys.modules["env.sim.trading_env"] = mod
    return mod.TradingEnv


def close_channel(F):
    """The close's channel: OHLC's 3 from F = 5 up, else the last market channel."""
    return min(3, F - 2)


def make_series(rng, N, D, F=5, sigma=0.01):
    """OHLC random walk [N, D, F] fp32; channel F-1 is a zero placeholder that
    trading_env.py:103 overwrites with the weight history. F = 5 is [open, high, low,
    close, weight]; F > 5 adds indicator-like channels (the reference's pool carries
    len(pool.features) channels, data/data_loader.py:48); F < 5 keeps [open, close][-F+1:]
    with the close in close_channel(F)."""
    z = rng.standard_normal((N, D + 1, 4))
    close = np.empty((N, D + 1))
    close[:, 0] = 100.0 * np.exp(0.2 * rng.standard_normal(N))
    for d in range(1, D + 1):
        close[:, d] = close[:, d - 1] * np.exp(sigma * z[:, d, 0])
    prev = close[:, :-1]
    c = close[:, 1:]
    o = prev * np.exp(0.3 * sigma * z[:, 1:, 1])
    h = np.maximum(o, c) * np.exp(np.abs(0.5 * sigma * z[:, 1:, 2]))
    lo = np.minimum(o, c) * np.exp(-np.abs(0.5 * sigma * z[:, 1:, 3]))
    s = np.zeros((N, D, F), np.float32)
    if F >= 5:
        s[:, :, 0], s[:, :, 1], s[:, :, 2], s[:, :, 3] = o, h, lo, c
        for f in range(4, F - 1):                   # scaled indicator-like channels in [0, 1]
            s[:, :, f] = rng.uniform(0.0, 1.0, (N, D))
    elif F == 4:
        s[:, :, 0], s[:, :, 1], s[:, :, 2] = o, h, c
    elif F == 3:
        s[:, :, 0], s[:, :, 1] = o, c
    else:
        s[:, :, 0] = c
    return s


def make_actions(rng, kind, T, N):
    a = np.zeros((T + 1, N), np.float32)
    for i in range(1, T + 1):
        if kind == "simplex":
            z = rng.standard_normal(N).astype(np.float32)
            e = np.exp(z - z.max())
            a[i] = (e / e.sum()).astype(np.float32)
        elif kind == "mixed":
            a[i] = rng.standard_normal(N).astype(np.float32)
        elif kind == "rawpos":
            a[i] = rng.uniform(0.0, 1.0, N).astype(np.float32)
        elif kind == "negsum1":
            m = rng.integers(-4, 9, N)
            m[1] = -abs(m[1]) - 1                     # at least one negative
            m[0] = 8 - m[1:].sum()                    # sum exactly 8
            a[i] = (m / 8.0).astype(np.float32)       # sum exactly 1, exactly representable
        else:
            raise ValueError(kind)
    return a


def run_case(name, N, W, T, dtype, kind, resets=(), chan_steps=None, seed=0, F=5):
    import torch
    torch.set_default_dtype(torch.float64 if dtype == "f64" else torch.float32)
    tdt = torch.get_default_dtype()
    TradingEnv = load_reference(W, N)
    rng = np.random.default_rng(seed)
    cc = close_channel(F)
    series = make_series(rng, N, T + W, F)
    actions = make_actions(rng, kind, T, N)
    # instrument.py:79 divides float32 close tensors, so the relatives the env sees
    # are fp32-rounded even when the env itself runs in f64
    close = series[:, :, cc]
    prices = np.zeros((T + 1, N), np.float64 if dtype == "f64" else np.float32)
    for i in range(1, T + 1):
        prices[i] = (close[:, i + W - 1] / close[:, i + W - 2]).astype(np.float32)
    ops = np.zeros(T + 1, np.int8)
    ops[0] = 1
    for r in resets:
        ops[r] = 1
    if chan_steps is None:
        chan_steps = list(range(T + 1))
    chan_steps = sorted(set(chan_steps))

    env = TradingEnv()
    rewards = np.full(T + 1, np.nan)
    values = np.zeros(T + 1)
    rets = np.full(T + 1, np.nan)
    wpost = np.full((T + 1, N), np.nan)
    chans = []
    for i in range(T + 1):
        window = torch.tensor(series[:, i:i + W, :], dtype=tdt)
        if ops[i]:
            obs = env.reset(window)
        else:
            a = torch.tensor(actions[i], dtype=tdt).reshape(N, 1)      # agent emits [N, 1]
            p = torch.tensor(prices[i], dtype=tdt)
            r, obs = env.step(a, window, p)
            rewards[i] = float(r)
            rets[i] = float(env.info["returns"][-1])
            wpost[i] = np.asarray(env.info["actions"][-1], np.float64)
        values[i] = float(env.value)
        if i in chan_steps:
            chans.append(obs[:, :, -1].numpy().astype(np.float64))
        # market channels are returned untouched (in-place write of channel F-1 only)
        assert np.array_equal(obs[:, :, :-1].numpy().astype(np.float32), series[:, i:i + W, :-1])
    meta = dict(name=name, N=N, W=W, F=F, close_channel=cc, T=T, dtype=dtype, kind=kind, resets=list(resets),
                seed=seed, reference="zachramsey/pm-rl @ 2025-03-04 env/sim/trading_env.py",
                torch=torch.__version__)
    np.savez_compressed(
        os.path.join(OUT, name + ".npz"), meta=np.array(json.dumps(meta)), series=series,
        actions=actions, prices=prices, ops=ops, rewards=rewards, values=values, rets=rets,
        wpost=wpost, chan_steps=np.array(chan_steps, np.int32), chans=np.array(chans))
    return meta


def reward_module_vectors():
    """env/reward.py:15-31 on fixed value histories (the class is dead code in
    step(), but it defines the returns / log_returns / sharpe_ratio semantics)."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import config.base as cb
    sys.modules.pop("env.reward", None)
    import env.reward as rw
    rng = np.random.default_rng(7)
    out = {}
    for L in (2, 3, 10, 64):
        vals = [25000.0]
        for _ in range(L - 1):
            vals.append(vals[-1] * float(1.0 + 0.01 * rng.standard_normal()))
        fake = types.SimpleNamespace(info={"values": vals})
        R = rw.Reward(fake)
        out[f"values_{L}"] = np.array(vals)
        out[f"returns_{L}"] = np.array(R.returns())
        out[f"log_returns_{L}"] = np.array(R.log_returns())
        with np.errstate(all="ignore"):
            out[f"sharpe_{L}"] = np.array(R.sharpe_ratio())
    out["risk_free_rate"] = np.array(cb.RISK_FREE_RATE)
    np.savez_compressed(os.path.join(OUT, "reward_module.npz"), **out)


def trainer_vectors():
    """agent/pg/pg.py:40-82 PG._reward and agent/a2c.py/a2c.py:40-82 A2C._loss, forward
    and torch-autograd gradient wrt the policy output `a`, run from the reference."""
    import importlib.util
    import torch
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import agent.pg.pg as pg
    spec = importlib.util.spec_from_file_location("a2c_ref", os.path.join(REF, "agent/a2c.py/a2c.py"))
    a2c = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(a2c)
    out = {}
    rng = np.random.default_rng(11)
    for dt in ("f64", "f32"):
        torch.set_default_dtype(torch.float64 if dt == "f64" else torch.float32)
        tdt = torch.get_default_dtype()
        for (B, N) in ((32, 30), (16, 5), (3, 7), (1, 5), (2, 1)):
            for akind in ("normal", "simplex"):
                z = rng.standard_normal((B, N)).astype(np.float32)
                a_np = z if akind == "normal" else (np.exp(z) / np.exp(z).sum(1, keepdims=True)).astype(np.float32)
                v_np = (25000.0 * np.exp(0.1 * rng.standard_normal(B))).astype(np.float32)
                p_np = (1.0 + 0.01 * rng.standard_normal((B, N))).astype(np.float32)
                for kind in ("log_returns", "returns", "sharpe_ratio"):
                    key = f"{dt}_{B}x{N}_{akind}_{kind}"
                    for mod, fn, tag in ((pg, pg.PG._reward, "pg"), (a2c, a2c.A2C._loss, "a2c")):
                        mod.REWARD, mod.REWARD_SCALE = kind, 1
                        a = torch.tensor(a_np, dtype=tdt).reshape(B, N, 1).requires_grad_(True)
                        v = torch.tensor(v_np, dtype=tdt).reshape(B, 1, 1)
                        pp = torch.tensor(p_np, dtype=tdt).reshape(B, N, 1)
                        r = fn(None, a, v, None, pp)
                        r.backward()
                        out[f"{key}_{tag}_r"] = np.array(float(r))
                        out[f"{key}_{tag}_grad"] = a.grad.reshape(B, N).detach().numpy().astype(np.float64)
                    out[f"{key}_a"], out[f"{key}_v"], out[f"{key}_p"] = a_np, v_np, p_np
    pg.REWARD, a2c.REWARD = "log_returns", "log_returns"
    np.savez_compressed(os.path.join(OUT, "trainer_reward.npz"), **out)


def driver_vectors(T_eval=40, T_roll=48, F=8, seed=77):
    """train/on_policy.py's env call sequence, run on the reference env: `TradingEnv()` with
    no arguments (:35, config/base.py's NUM_ASSETS / WINDOW_SIZE), then _evaluate(0)
    (:76-90), _rollout (:56-67, recording what buffer.add receives: np.array(env.value)),
    and _evaluate(1) — one env object throughout, as Metrics / Visualizer hold it
    (:39-40). The windows carry F feature channels (len(pool.features), not 5), the agent's
    actions are [N, 1] (simplex, with every 7th step mixed-sign to reach the normalisation
    branch). After each phase the info lists are recorded as util/eval.py:14-37 and
    util/plot.py:61,74-75 read them, plus each entry's type (trading_env.py:13-18, :80-100)."""
    import torch
    torch.set_default_dtype(torch.float32)
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import config.base as cb
    N, W = cb.NUM_ASSETS, cb.WINDOW_SIZE             # the constructor's shape: config/base.py:28-29
    TradingEnv = load_reference(W, N)
    rng = np.random.default_rng(seed)
    cc = close_channel(F)
    test = make_series(rng, N, T_eval + W, F)
    train = make_series(rng, N, T_roll + W, F)
    out = {"test_series": test, "train_series": train}

    def actions(T):
        a = make_actions(rng, "simplex", T, N)
        mixed = make_actions(rng, "mixed", T, N)
        a[7::7] = mixed[7::7]
        return a

    def prices_of(series, T):
        c = series[:, :, cc]
        p = np.zeros((T + 1, N), np.float32)
        for i in range(1, T + 1):
            p[i] = c[:, i + W - 1] / c[:, i + W - 2]
        return p

    def tname(x):
        return type(x).__name__ + ("" if not hasattr(x, "dtype") else ":" + str(x.dtype).replace("torch.", "")) + \
            ("" if not hasattr(x, "shape") else ":" + "x".join(map(str, tuple(x.shape))))

    env = TradingEnv()
    out["init_info_types"] = np.array(json.dumps({k: [tname(x) for x in v] for k, v in env.info.items()}))
    out["init_value"] = np.array(float(env.value))
    for phase, series, T in (("eval0", test, T_eval), ("rollout", train, T_roll), ("eval1", test, T_eval)):
        acts, prices = actions(T), prices_of(series, T)
        rewards = np.full(T + 1, np.nan)
        values = np.zeros(T + 1)
        buf_v = np.full(T + 1, np.nan)
        s = None
        for step in range(T + 1):
            data = torch.tensor(series[:, step:step + W, :])
            if step == 0:
                s = env.reset(data)
                assert s is data
            else:
                a = torch.tensor(acts[step]).reshape(N, 1)
                r, s_ = env.step(a, data, torch.tensor(prices[step]))
                assert s_ is data
                rewards[step] = float(r)
                if phase == "rollout":
                    buf_v[step] = float(np.array(env.value))     # RolloutBuffer.add: np.array(v)
                s = s_
            values[step] = float(env.value)
        info = env.info
        assert list(info.keys()) == ["values", "actions", "rewards", "returns"]
        out[f"{phase}_actions_in"], out[f"{phase}_prices"] = acts, prices
        out[f"{phase}_rewards"], out[f"{phase}_values"], out[f"{phase}_buffer_value"] = rewards, values, buf_v
        out[f"{phase}_info_values"] = np.array([float(x) for x in info["values"]])
        out[f"{phase}_info_actions"] = np.array(info["actions"], dtype=np.float64)   # eval.py:33
        out[f"{phase}_info_rewards"] = np.array([float(x) for x in info["rewards"]])
        out[f"{phase}_info_returns"] = np.array([float(x) for x in info["returns"]])
        out[f"{phase}_info_types"] = np.array(json.dumps({k: [tname(x) for x in v[:2]] for k, v in info.items()}))
        out[f"{phase}_chan"] = s[:, :, -1].numpy().astype(np.float64)
        assert np.array_equal(s[:, :, :-1].numpy(), series[:, T:T + W, :-1])
    meta = dict(N=N, W=W, F=F, close_channel=cc, T_eval=T_eval, T_roll=T_roll, seed=seed, dtype="f32",
                reference="zachramsey/pm-rl @ 2025-03-04 train/on_policy.py + env/sim/trading_env.py",
                torch=torch.__version__)
    out["meta"] = np.array(json.dumps(meta))
    np.savez_compressed(os.path.join(OUT, "onpolicy_driver.npz"), **out)


CASES = [
    # name, N, W, T, dtype, kind, resets, chan_steps
    ("simplex_n5_w50_t64_f64", 5, 50, 64, "f64", "simplex", (), None),
    ("simplex_n5_w50_t64_f32", 5, 50, 64, "f32", "simplex", (), None),
    ("simplex_n30_w50_t256_f64", 30, 50, 256, "f64", "simplex", (), [0, 1, 2, 47, 48, 49, 50, 51, 100, 255, 256]),
    ("simplex_n30_w50_t256_f32", 30, 50, 256, "f32", "simplex", (), [0, 1, 2, 48, 49, 50, 51, 256]),
    ("mixed_n30_w50_t64_f64", 30, 50, 64, "f64", "mixed", (), [0, 1, 49, 50, 64]),
    ("mixed_n30_w50_t64_f32", 30, 50, 64, "f32", "mixed", (), [0, 1, 49, 50, 64]),
    ("rawpos_n30_w50_t48_f64", 30, 50, 48, "f64", "rawpos", (), [0, 1, 48]),
    ("rawpos_n30_w50_t48_f32", 30, 50, 48, "f32", "rawpos", (), [0, 1, 48]),
    ("negsum1_n5_w8_t24_f64", 5, 8, 24, "f64", "negsum1", (), None),
    ("negsum1_n5_w8_t24_f32", 5, 8, 24, "f32", "negsum1", (), None),
    ("wrap_n5_w8_t40_f64", 5, 8, 40, "f64", "simplex", (), None),
    ("wrap_n5_w4_t12_f32", 5, 4, 12, "f32", "simplex", (), None),
    ("reset_n5_w8_t40_f64", 5, 8, 40, "f64", "simplex", (13, 29), None),
    ("reset_n7_w6_t30_f32", 7, 6, 30, "f32", "mixed", (5, 6, 20), None),
    ("simplex_n129_w50_t16_f64", 129, 50, 16, "f64", "simplex", (), [0, 1, 16]),
]

# F != 5: the reference's windows carry len(pool.features) channels (data/data_loader.py:48)
FEAT_CASES = [
    # name, N, W, T, dtype, kind, resets, chan_steps, F
    ("feat12_n30_w50_t64_f64", 30, 50, 64, "f64", "simplex", (), [0, 1, 49, 50, 64], 12),
    ("feat12_n30_w50_t64_f32", 30, 50, 64, "f32", "mixed", (), [0, 1, 49, 50, 64], 12),
    ("feat3_n7_w10_t30_f32", 7, 10, 30, "f32", "mixed", (11,), None, 3),
    ("feat8_n32_w32_t80_f64", 32, 32, 80, "f64", "simplex", (40,), [0, 1, 31, 32, 33, 40, 41, 80], 8),
]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="comma list: env (F = 5 cases), feat, driver, reward, trainer")
    only = set(filter(None, ap.parse_args().only.split(","))) or {"env", "feat", "driver", "reward", "trainer"}
    if "env" in only:
        for i, (name, N, W, T, dt, kind, resets, cs) in enumerate(CASES):
            m = run_case(name, N, W, T, dt, kind, resets, cs, seed=1000 + i)
            print("wrote", m["name"])
    if "feat" in only:
        for i, (name, N, W, T, dt, kind, resets, cs, F) in enumerate(FEAT_CASES):
            m = run_case(name, N, W, T, dt, kind, resets, cs, seed=2000 + i, F=F)
            print("wrote", m["name"])
    if "driver" in only:
        driver_vectors()
        print("wrote onpolicy_driver")
    if "reward" in only:
        reward_module_vectors()
        print("wrote reward_module")
    if "trainer" in only:
        trainer_vectors()
        print("wrote trainer_reward")


if __name__ == "__main__":
    main()
