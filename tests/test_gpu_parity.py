"""HIP path (libpmenv.so through the C ABI) vs the reference's golden vectors and
vs the CPU oracle; full-size properties at BASELINE sizes. Needs an MI355X."""
import zlib

import numpy as np
import pytest
import torch

import golden_util as gu
from test_oracle_golden import compare
from oracle import OracleEnv, gae as or_gae, moments as or_moments, synth_series, synth_actions

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    torch.cuda.set_device(DEV)


def _t(x, dtype=torch.float32):
    return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=DEV)


def replay_gpu(g, mode, host=False, impl="auto", direct=True):
    """host=True: the reference's own call shape with CPU tensors (train/on_policy.py:59-67
    hands the env host tensors): surface steps through pmenv_step_host (direct=False: the
    whole window staged through the GPU, round 4's path), advance steps staged. impl: the
    advance step's implementation (TradingEnv.set_step_impl)."""
    from pmenv import TradingEnv
    m = g["meta"]
    N, W, F, T = m["N"], m["W"], m["F"], m["T"]
    env = TradingEnv(num_envs=1, num_assets=N, window=W, features=F, device=DEV, track_info=True, step_impl=impl,
                     close_channel=gu.close_channel(g))
    env._HOST_DIRECT = direct
    _t = (lambda x, dtype=torch.float32: torch.as_tensor(np.ascontiguousarray(x), dtype=dtype)) if host else \
        globals()["_t"]
    out = {"rewards": np.full(T + 1, np.nan), "values": np.zeros(T + 1), "rets": np.full(T + 1, np.nan),
           "wpost": np.full((T + 1, N), np.nan), "chans": {}, "market_ok": True}
    obs = None
    for i in range(T + 1):
        if g["ops"][i]:
            obs = _t(gu.window(g, i)[0])             # unbatched [N, W, F] like the reference
            env.reset(obs)
        else:
            if mode == "surface":
                obs = _t(gu.window(g, i)[0])
                r, obs2 = env.step(_t(g["actions"][i]).reshape(N, 1), obs, _t(g["prices"][i]))
            else:
                r, obs2 = env.step(_t(g["actions"][i]).reshape(N, 1), obs, bar=_t(gu.bar(g, i)))
                out["market_ok"] &= np.array_equal(obs[..., :-1].cpu().numpy(), gu.window(g, i)[0, ..., :-1])
            assert obs2 is obs and r.dim() == 0 and r.device == obs.device
            out["rewards"][i] = float(r)
            if host:                   # the reference's entry types: 0-dim / [N] numpy arrays
                out["rets"][i] = float(env.info["returns"][-1])
                out["wpost"][i] = env.info["actions"][-1]
            else:
                out["rets"][i] = float(env.info["returns"][-1][0])
                out["wpost"][i] = env.info["actions"][-1][0].cpu().numpy()
        out["values"][i] = float(env.value)
        out["chans"][i] = obs[:, :, -1].cpu().numpy().copy()     # host windows advance in place
    return out


@pytest.mark.parametrize("name", gu.cases())
@pytest.mark.parametrize("mode", ["surface", "advance"])
def test_gpu_matches_reference_goldens(name, mode):
    g = gu.load(name)
    out = replay_gpu(g, mode)
    assert out["market_ok"]
    compare(g, out)


@pytest.mark.parametrize("name", gu.cases())
@pytest.mark.parametrize("impl", ["flat", "one_launch", "two_launch", "relay"])
def test_gpu_every_step_path_matches_reference_goldens(name, impl):
    """The reference's recorded outputs replayed through each advance-step implementation
    forced (AUTO takes one_launch at one env). A path refuses exactly the shapes its
    contract excludes (include/pmenv.h: the one-launch forms need N <= 64 and 16-B
    granular env windows; two launches take F != 5 through the generic stream); those cases
    check the refusal instead."""
    from pmenv import TradingEnv
    m = gu.load(name)["meta"]
    N, W, F = m["N"], m["W"], m["F"]
    # the shape rules of pmenv_set_step_path (include/pmenv.h)
    granular = F == 5 and (N * W * F) % 4 == 0
    # F != 5: the generic stream (2 <= F <= 16, 16-B granular, the workgroup's rows fit)
    generic = F != 5 and 2 <= F <= 16 and (N * W * F) % 4 == 0 and 4 * 1024 // (W * F) + 2 <= 256
    misfit = {"two_launch": not (granular or generic),
              "one_launch": not (granular and W >= 2 and N <= 64 and N * W * F * 4 <= 64 * 1024),
              "flat": not (granular and W >= 2 and N <= 64 and N * W * F // 4 >= 148),
              "relay": not (granular and W >= 2 and N <= 512)}[impl]
    try:
        env = TradingEnv(num_envs=1, num_assets=N, window=W, features=F, device=DEV, step_impl=impl)
    except ValueError:
        assert misfit, f"{impl} refused N={N} W={W} F={F}"
        return
    assert not misfit, f"{impl} accepted N={N} W={W} F={F}"
    kern = {"flat": "step_flat_kernel", "one_launch": "step_env_kernel", "relay": "step_relay_kernel",
            "two_launch": "+"}[impl]
    assert kern in env.step_path.split(" | ")[1], env.step_path      # the in-place path is the one forced
    g = gu.load(name)
    out = replay_gpu(g, "advance", impl=impl)
    assert out["market_ok"]
    compare(g, out)


HOST_LEGS = {"surface_direct": ("surface", "auto", True), "surface_staged": ("surface", "auto", False),
             "advance_relay": ("advance", "relay", True), "advance_auto": ("advance", "auto", True)}


@pytest.mark.parametrize("name", ["simplex_n30_w50_t256_f64", "mixed_n30_w50_t64_f32", "wrap_n5_w8_t40_f64",
                                  "reset_n5_w8_t40_f64", "simplex_n5_w50_t64_f32", "feat8_n32_w32_t80_f64"])
@pytest.mark.parametrize("leg", list(HOST_LEGS))
def test_gpu_reference_goldens_with_host_tensors(name, leg):
    """The reference's callers drive the env with CPU tensors, unchanged: features,
    actions and prices on the host in, reward and value back on the host, the
    features mutated in place and returned (trading_env.py:102-105). Surface steps run
    through pmenv_step_host (direct) and through round 4's whole-window staging; advance
    steps with host tensors through the relayed step and AUTO's."""
    if name not in gu.cases():
        pytest.skip("golden case absent")
    mode, impl, direct = HOST_LEGS[leg]
    g = gu.load(name)
    m = g["meta"]
    if impl == "relay" and not (m["F"] == 5 and (m["N"] * m["W"] * 5) % 4 == 0 and m["W"] >= 2):
        pytest.skip("relay refuses this shape (checked in test_gpu_every_step_path_matches_reference_goldens)")
    out = replay_gpu(g, mode, host=True, impl=impl, direct=direct)
    compare(g, out)


def _run_both(cfg_kw, B, N, W, T, kind="simplex", seed=0, F=5, resets=None, mode="advance", double_buffer=False,
              impl="auto"):
    """Drive pmenv and the oracle side by side on identical inputs (impl: the advance
    step's implementation, TradingEnv.set_step_impl)."""
    from pmenv import TradingEnv
    from pmenv.config import EnvConfig
    rng = np.random.default_rng(seed)
    Fm = F - 1
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((W + T, B, N)), axis=0))
    ser = np.empty((W + T, B, N, Fm), np.float32)
    for f in range(Fm):
        ser[..., f] = closes * np.exp(0.002 * rng.standard_normal(closes.shape))
    ser[..., cfg_kw.get("close_channel", min(3, Fm - 1))] = closes
    obs0 = np.zeros((B, N, W, F), np.float32)
    obs0[..., :Fm] = ser[:W].transpose(1, 2, 0, 3)
    if kind == "simplex":
        z = rng.standard_normal((T, B, N))
        act = np.exp(z) / np.exp(z).sum(-1, keepdims=True)
    elif kind == "mixed":
        act = rng.standard_normal((T, B, N))
    else:
        act = rng.uniform(0, 1, (T, B, N)) / N * 2
    act = act.astype(np.float32)
    cfg = EnvConfig(num_envs=B, num_assets=N, window=W, features=F, **cfg_kw)
    genv = TradingEnv(config=cfg, device=DEV, track_info=True, step_impl=impl)
    cenv = OracleEnv(cfg)
    gobs = _t(obs0)
    cobs = obs0.copy()
    genv.reset(gobs)
    cenv.reset(cobs)
    for t in range(T):
        if resets is not None and t in resets:
            mask = resets[t]
            genv.reset(gobs, mask=_t(mask, torch.bool))
            cenv.reset(cobs, mask=mask)
        y = None
        if mode == "surface":
            y = (ser[W + t, ..., cfg.close_channel] / ser[W + t - 1, ..., cfg.close_channel]).astype(np.float32)
            win = np.zeros_like(cobs)
            win[..., :Fm] = ser[t + 1:t + 1 + W].transpose(1, 2, 0, 3)
            cobs[...] = win
            gobs.copy_(_t(win))
            gr, _ = genv.step(_t(act[t]), gobs, prices=_t(y))
            cr, cret, cw = cenv.step(act[t], cobs, prices=y)
        elif double_buffer:
            nxt = torch.full_like(gobs, float("nan"))
            prev = gobs.clone()
            gr, got = genv.step(_t(act[t]), gobs, bar=_t(ser[W + t]), out=nxt)
            assert got is nxt and torch.equal(gobs, prev)        # the input window is untouched
            gobs = nxt
            cr, cret, cw = cenv.step(act[t], cobs, bar=ser[W + t])
        else:
            gr, _ = genv.step(_t(act[t]), gobs, bar=_t(ser[W + t]))
            cr, cret, cw = cenv.step(act[t], cobs, bar=ser[W + t])
        g_r = gr.cpu().numpy()
        both_nan = np.isnan(g_r) & np.isnan(cr)
        err = np.where(both_nan, 0, np.abs(g_r.astype(np.float64) - cr))
        tol = np.where(both_nan, 0, 1e-6 * np.abs(np.nan_to_num(cr)) + 1e-9)   # SHARPE: NaN at t=1 (numpy ddof=1)
        assert np.all(err <= tol), f"step {t}: reward err {np.nanmax(err):.3e}"
        np.testing.assert_allclose(genv.info["returns"][-1].cpu().numpy(), cret, rtol=1e-12)
        gv = genv.value.cpu().numpy()
        np.testing.assert_allclose(gv, cenv.value, rtol=1e-12)
        np.testing.assert_allclose(genv.info["actions"][-1].cpu().numpy(), cw, rtol=2e-7, atol=1e-12)
        go = gobs.cpu().numpy()
        assert np.array_equal(go[..., :Fm], cobs[..., :Fm]), f"market channels differ at step {t}"
        np.testing.assert_allclose(go[..., Fm], cobs[..., Fm], rtol=2e-7, atol=1e-12)
    assert np.array_equal(genv._counter.cpu().numpy(), cenv.k)
    np.testing.assert_allclose(genv._ring.cpu().numpy(), cenv.ring, rtol=2e-7, atol=1e-12)
    np.testing.assert_allclose(genv._stat_a.cpu().numpy(), cenv.stat_a, rtol=1e-9, atol=1e-14)
    return genv, cenv


MODES = [
    dict(),
    dict(ring="chrono"),
    dict(reward="returns"),
    dict(reward="sharpe_ratio"),
    dict(reward="diff_sharpe", sharpe_eta=0.05),
    dict(commission=0.0025),
    dict(commission=0.01, ret="net", reward="diff_sharpe"),
    dict(commission=0.0025, reward="returns"),                  # default GROSS: info["returns"] as :88
    dict(commission=0.0025, ret="auto", reward="sharpe_ratio"),  # opt-in AUTO: net for reward.py kinds
    dict(norm="or"),
    dict(reward_scale=100.0, init_cash=1e6),
]


@pytest.mark.parametrize("kw", MODES, ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
@pytest.mark.parametrize("kind", ["simplex", "mixed", "rawpos"])
def test_gpu_vs_oracle_modes(kw, kind):
    _run_both(kw, B=67, N=30, W=50, T=70, kind=kind, seed=zlib.crc32(f"{kw}{kind}".encode()))


@pytest.mark.parametrize("mode", ["surface", "advance"])
def test_gpu_vs_oracle_surface_and_advance(mode):
    _run_both({}, B=33, N=30, W=12, T=30, kind="mixed", mode=mode, seed=3)


@pytest.mark.parametrize("N,W,F,B", [
    (30, 50, 5, 40),      # 7,500 floats per env: 16-B chunks, the tail past 8,192 floats not reached
    (30, 50, 8, 5),       # 12,000 floats: chunks past the prefetched 8,192
    (64, 16, 8, 3),       # exactly 8,192 floats
    (7, 6, 4, 9),         # F = 4: one weight float per chunk, at its end
    (9, 8, 3, 11),        # F = 3: two weight floats in some chunks
    (5, 50, 5, 7),        # 1,250 floats: not 16-B granular, the dword path
])
@pytest.mark.parametrize("kw", [{}, {"ring": "chrono"}, {"commission": 0.0025, "reward": "diff_sharpe"}],
                         ids=["storage", "chrono", "commission"])
def test_gpu_surface_step_vs_oracle(N, W, F, B, kw):
    """The reference surface contract with device windows (channel F-1 rebuilt from the ring):
    16-B-granular env blocks are rewritten in whole chunks, others float by float; past the
    ring's wrap, against the oracle."""
    kw = dict(kw, **({} if F == 5 else {"close_channel": F - 2}))
    _run_both(kw, B=B, N=N, W=W, T=W + 5, kind="mixed", F=F, mode="surface", seed=N * 7 + W + F)


@pytest.mark.parametrize("N,W,F,B,T,kw", [
    (30, 50, 5, 9000, 53, {}),                                      # 270 MB: past the Infinity Cache
    (16, 12, 8, 44000, 15, {"ring": "chrono", "commission": 0.0025}),
    (4, 5, 4, 850000, 8, {"ring": "chrono"}),                      # 206 rows of 51 envs per workgroup
])
def test_gpu_surface_stream_vs_oracle(N, W, F, B, T, kw):
    """The surface contract on windows past the Infinity Cache: the scalar step, then
    surface_stream_kernel (the window's 16-B chunks with their weight floats replaced from the
    ring columns staged in LDS), past the ring's wrap, against the oracle."""
    kw = dict(kw, **({} if F == 5 else {"close_channel": F - 2}))
    _run_both(kw, B=B, N=N, W=W, T=T, kind="simplex", F=F, mode="surface", seed=B + F)


@pytest.mark.parametrize("N,W,F", [(30, 50, 5), (129, 50, 5), (5, 50, 5), (7, 6, 3)])
def test_gpu_double_buffered_advance(N, W, F):
    kw = {} if F == 5 else {"close_channel": F - 2}
    _run_both(kw, B=9, N=N, W=W, T=W + 7, kind="mixed", F=F, seed=N, double_buffer=True)


@pytest.mark.parametrize("kw", MODES, ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
@pytest.mark.parametrize("kind", ["simplex", "mixed"])
def test_gpu_flat_obs_out_vs_oracle_modes(kw, kind):
    """The two-launch step double-buffered (scalar_step_vec_kernel, then the flat
    stream advance_flat_wg_kernel: the obs_out path for N > 64) against the oracle in
    every reward / ring / norm / commission mode, through the ring wrap."""
    from pmenv import TradingEnv
    e = TradingEnv(num_envs=3, num_assets=30, window=50, device=DEV, step_impl="two_launch")
    assert "advance_flat_wg_kernel" in e.step_path.split(" | ")[0]
    _run_both(kw, B=67, N=30, W=50, T=70, kind=kind, seed=zlib.crc32(f"flat{kw}{kind}".encode()),
              double_buffer=True, impl="two_launch")


@pytest.mark.parametrize("kw", MODES, ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
@pytest.mark.parametrize("kind", ["simplex", "mixed"])
def test_gpu_flat_inplace_vs_oracle_modes(kw, kind):
    """The two-launch step in place (the scalar step copying the halo, then
    advance_flat_inplace_kernel: the in-place path for N > 64 and for cache-resident
    windows of 3,072+ envs) against the oracle."""
    from pmenv import TradingEnv
    e = TradingEnv(num_envs=3, num_assets=30, window=50, device=DEV, step_impl="two_launch")
    assert "advance_flat_inplace_kernel" in e.step_path.split(" | ")[1]
    _run_both(kw, B=67, N=30, W=50, T=70, kind=kind, seed=zlib.crc32(f"flatip{kw}{kind}".encode()),
              impl="two_launch")


@pytest.mark.parametrize("N,W,B", [
    (30, 50, 37),     # env = 1875 chunks: waves straddle envs and rows
    (5, 4, 13),       # rows of 20 floats: several rows per wave, chunks straddle rows
    (4, 2, 7),        # W = 2 (the smallest flat window): every other day is a last day
    (1, 4, 9),        # one asset, envs of 5 chunks
    (64, 16, 3),      # grid tail: chunk count not a multiple of 64
    (129, 50, 2),     # long envs
    (12, 10, 1),      # single env
])
def test_gpu_flat_obs_out_shapes(N, W, B):
    impl = "two_launch" if N * W * 5 % 4 == 0 else "auto"    # not 16-B granular: the LDS fallback
    _run_both({}, B=B, N=N, W=W, T=W + 9, kind="mixed", seed=N * 7 + W, double_buffer=True, impl=impl)
    _run_both({"ring": "chrono"}, B=B, N=N, W=W, T=W + 3, kind="simplex", seed=N + W, double_buffer=True,
              impl=impl)


@pytest.mark.parametrize("N,W,B", [(30, 50, 37), (5, 4, 13), (4, 2, 7), (1, 4, 9), (64, 16, 3), (129, 50, 2),
                                   (12, 10, 1), (30, 50, 600)])
def test_gpu_flat_inplace_shapes(N, W, B):
    """Workgroup seams (the halo) at every alignment against rows, envs and the
    tensor's end; (30, 50, 600): hundreds of workgroups, each seam's halo exercised."""
    impl = "two_launch" if N * W * 5 % 4 == 0 else "auto"    # not 16-B granular: the LDS fallback
    _run_both({}, B=B, N=N, W=W, T=W + 9, kind="mixed", seed=N * 5 + W, impl=impl)
    _run_both({"ring": "chrono"}, B=B, N=N, W=W, T=W + 3, kind="simplex", seed=N + 3 * W, impl=impl)


def test_gpu_auto_path_rule():
    """AUTO: windows up to 24 MiB take the one-workgroup-per-env step (launch-latency
    bound); N <= 64 in place from 24 to 256 MiB the relayed one-launch step (step_relay_kernel)
    — except up to 48 MiB where the one-workgroup-per-env step holds the env with >= 90 %
    occupancy (N = 30) — and double-buffered from 48 to 128 MiB; above, env windows of
    >= 1,000 chunks take the flat one-launch step (step_flat_kernel) — double-buffered from
    128 MiB, in place from 256 MiB, with or without commission — and the rest the two-launch
    stream; wide envs (64 < N <= 128) take step_flat_vec_kernel in place above 1 GiB.
    Checked against the oracle at the band's shapes."""
    from pmenv import TradingEnv

    def parts(e):
        db, ip = e.step_path.split(" | ")
        return db, ip
    small = TradingEnv(num_envs=800, num_assets=8, window=50, device=DEV)            # 6 MB
    assert small.step_path.count("step_env_kernel") == 2
    db, ip = parts(TradingEnv(num_envs=1500, num_assets=30, window=50, device=DEV))   # 45 MB
    assert db.startswith("step_env_kernel") and ip.startswith("step_env_kernel")
    db, ip = parts(TradingEnv(num_envs=1700, num_assets=30, window=50, device=DEV))   # 51 MB
    assert db.startswith("step_relay_kernel") and ip.startswith("step_relay_kernel")
    db, ip = parts(TradingEnv(num_envs=3000, num_assets=30, window=50, device=DEV))   # 90 MB
    assert db.startswith("step_relay_kernel") and ip.startswith("step_relay_kernel")
    db, ip = parts(TradingEnv(num_envs=4096, num_assets=30, window=50, device=DEV))   # 123 MB: config 2
    assert db.startswith("step_relay_kernel") and ip.startswith("step_relay_kernel")
    db, ip = parts(TradingEnv(num_envs=8192, num_assets=30, window=50, device=DEV))   # 246 MB: config 4's share
    assert db.startswith("step_flat_kernel") and ip.startswith("step_relay_kernel")
    db, ip = parts(TradingEnv(num_envs=4096, num_assets=16, window=50, device=DEV))   # 66 MB, 78 % fill
    assert ip.startswith("step_relay_kernel")
    db, ip = parts(TradingEnv(num_envs=4096, num_assets=8, window=50, device=DEV))    # 33 MB, 65 % fill
    assert ip.startswith("step_relay_kernel") and db.startswith("step_env_kernel")
    huge = TradingEnv(num_envs=9000, num_assets=30, window=50, device=DEV)           # 270 MB
    assert huge.step_path.count("step_flat_kernel") == 2
    db, ip = parts(TradingEnv(num_envs=9000, num_assets=8, window=50, device=DEV))    # 72 MB, 500 chunks per env
    assert db.startswith("step_relay_kernel") and ip.startswith("step_relay_kernel")
    thin = TradingEnv(num_envs=18000, num_assets=8, window=50, device=DEV)           # 144 MB
    db, ip = parts(thin)
    assert ip.startswith("step_relay_kernel") and "step_flat_kernel" not in db and "step_env_kernel" not in db
    wide = TradingEnv(num_envs=2000, num_assets=65, window=50, device=DEV)           # N > 64
    assert "step_flat_kernel" not in wide.step_path
    comm = TradingEnv(num_envs=9000, num_assets=30, window=50, device=DEV, commission=0.0025)
    assert comm.step_path.count("step_flat_kernel") == 2                            # the fixed point per tile
    comm.set_step_impl("two_launch")                                                # forced: still available
    assert "step_flat_kernel" not in comm.step_path
    wide_big = TradingEnv(num_envs=16384, num_assets=100, window=50, device=DEV)     # 1.6 GB
    db, ip = wide_big.step_path.split(" | ")
    assert ip.startswith("step_flat_vec_kernel") and not db.startswith("step_flat")
    wide_500 = TradingEnv(num_envs=8192, num_assets=500, window=50, device=DEV)      # config 5: two launches
    assert "step_flat" not in wide_500.step_path
    _run_both({}, B=1700, N=30, W=50, T=9, kind="mixed", seed=31)
    _run_both({"ring": "chrono"}, B=1700, N=30, W=50, T=5, kind="simplex", seed=32, double_buffer=True)
    _run_both({}, B=4096, N=8, W=50, T=53, kind="mixed", seed=34)
    _run_both({"ring": "chrono", "commission": 0.0025}, B=4096, N=16, W=50, T=6, kind="rawpos", seed=35)
    _run_both({}, B=9000, N=30, W=50, T=7, kind="mixed", seed=33)


@pytest.mark.parametrize("impl", ["one_launch", "two_launch"])
def test_gpu_flat_resident_series_obs_out(impl):
    """Day-indexed bars (resident series) double-buffered == the bar batch, bit for
    bit; an out-of-range day reads NaN market channels, counted, not read."""
    from pmenv import TradingEnv, MarketSeries
    rng = np.random.default_rng(5)
    T, N, W, B, S = 200, 30, 20, 41, 30
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((T, N)), axis=0))
    bars = np.stack([closes * np.exp(0.002 * rng.standard_normal((T, N))) for _ in range(3)] + [closes], -1)
    m = MarketSeries(bars.astype(np.float32), device=DEV)
    start = m.random_starts(B, W, S + 1, generator=torch.Generator().manual_seed(3))
    obs_a = m.initial_window(start, W)
    obs_b = obs_a.clone()
    ea = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl)
    eb = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl)
    ea.reset(obs_a)
    eb.reset(obs_b)
    act = torch.softmax(torch.randn(S, B, N, device=DEV), -1)
    for t in range(S):
        day = start + W + t
        ra, obs_a = ea.step(act[t], obs_a, series=m, day=day, out=torch.empty_like(obs_a))
        rb, obs_b = eb.step(act[t], obs_b, bar=m.bars[day.long()].contiguous(), out=torch.empty_like(obs_b))
        assert torch.equal(ra, rb)
    assert torch.equal(obs_a, obs_b) and torch.equal(ea.value, eb.value)
    bad = start + W + S
    bad[7] = -3
    _, nxt = ea.step(act[0], obs_a, series=m, day=bad, out=torch.empty_like(obs_a))
    assert ea.nonfinite_count() == 1
    assert bool(torch.isnan(nxt[7, :, -1, :4]).all()) and not bool(torch.isnan(nxt[6]).any())


@pytest.mark.parametrize("N,W,B", [(1, 4, 9), (4, 6, 13), (8, 10, 21), (9, 4, 5), (16, 8, 33), (17, 4, 7),
                                   (33, 4, 11), (64, 16, 3), (65, 4, 6), (129, 8, 5), (256, 4, 3), (300, 8, 4),
                                   (500, 50, 4), (512, 2, 3)])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_k1_packed_asset_counts(N, W, B, db):
    """The two-launch step's packed scalar-step shape per asset count (partial last
    lane, group edges at 8 / 16 / 32 / 64 lanes, N up to 512) through both window
    modes, against the oracle."""
    _run_both({}, B=B, N=N, W=W, T=W + 5, kind="mixed", seed=N * 31 + W, double_buffer=db, impl="two_launch")
    _run_both({"commission": 0.0025, "norm": "or"}, B=B, N=N, W=W, T=W + 2, kind="rawpos", seed=N + 7 * W,
              double_buffer=db, impl="two_launch")


@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
@pytest.mark.parametrize("kw", MODES[:1] + MODES[4:8], ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
def test_gpu_one_and_two_launch_agree(db, kw):
    """The two implementations of the advance step on identical inputs agree bit for
    bit (N <= 64: the two-launch path's register-form scalar step reduces in the same
    order as the one-launch step's), so a run sharded over ranks — whose path can
    differ from the unsharded run's by env count — gives the same bits."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 37, 30, 50, 56
    ser = synth.series(W + T, B, N, seed=zlib.crc32(f"{kw}{db}".encode()), device=DEV)
    act = synth.actions(T, B, N, seed=7, device=DEV)
    envs, obs = [], []
    for impl in ("one_launch", "two_launch"):
        e = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl, **kw)
        o = synth.window_from_series(ser, W)
        e.reset(o)
        envs.append(e)
        obs.append(o)
    for t in range(T):
        rs = []
        for i, e in enumerate(envs):
            if db:
                r, obs[i] = e.step(act[t], obs[i], bar=ser[W + t], out=torch.empty_like(obs[i]))
            else:
                r, _ = e.step(act[t], obs[i], bar=ser[W + t])
            rs.append(r)
        assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
        assert torch.equal(rs[0].nan_to_num(7.0), rs[1].nan_to_num(7.0)), f"step {t}: rewards"
        assert torch.equal(envs[0].value, envs[1].value), f"step {t}: values"


@pytest.mark.parametrize("N", [1, 5, 8, 9, 16])
@pytest.mark.parametrize("kw", [MODES[0], MODES[2], MODES[6], MODES[8], MODES[9]],
                         ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_small_n_paths_agree(N, kw, db):
    """N <= 16: the two-launch step's packed scalar step (8 / 16 lanes per env) gives the
    bits of the one-launch steps' register-form scalar part (flat, per-env) in every
    path, in place and double-buffered, including the signed-zero corners — all-zero and
    all -0.0 action rows, whose sums the register form's padding lanes turn into +0.0."""
    from pmenv import TradingEnv, synth
    B = 41
    W = -(-max(8, -(-592 // (5 * N))) // 4) * 4             # flat: >= 148 16-B chunks per env window
    T = W + 4                                                  # through the storage-ring wrap
    ser = synth.series(W + T, B, N, seed=zlib.crc32(f"small{N}{kw}".encode()), device=DEV)
    act = synth.actions(T, B, N, seed=N + 3, device=DEV).clone()
    act[:, 1::3] = act[:, 1::3] * 3.0 - 0.4                  # off-simplex rows, some negative weights
    act[:, 3] = 0.0
    act[:, 5] = -0.0
    act[2:, 7] = -0.0
    act[::2, 9, : (N + 1) // 2] = -0.0
    impls = ("flat", "one_launch", "two_launch")
    envs, obs = [], []
    for impl in impls:
        e = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl, **kw)
        o = synth.window_from_series(ser, W)
        e.reset(o)
        envs.append(e)
        obs.append(o)
    assert "scalar_step_vec_kernel" in envs[2].step_path
    for t in range(T):
        rs = []
        for i, e in enumerate(envs):
            if db:
                r, obs[i] = e.step(act[t], obs[i], bar=ser[W + t], out=torch.empty_like(obs[i]))
            else:
                r, _ = e.step(act[t], obs[i], bar=ser[W + t])
            rs.append(r)
        for i in (1, 2):
            # bit patterns: the zero rows' w' is 0 / 0 (NaN), the same NaN in every path
            assert torch.equal(obs[0].view(torch.int32), obs[i].view(torch.int32)), f"step {t} {impls[i]}: windows"
            assert torch.equal(rs[0].view(torch.int32), rs[i].view(torch.int32)), f"step {t} {impls[i]}: rewards"
            assert torch.equal(envs[0].value.view(torch.int64), envs[i].value.view(torch.int64)), \
                f"step {t} {impls[i]}: values"


@pytest.mark.parametrize("kind", ["simplex", "mixed", "rawpos"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
@pytest.mark.parametrize("kw", MODES, ids=lambda k: "-".join(f"{a}={b}" for a, b in k.items()) or "reference")
def test_gpu_one_launch_vs_oracle_modes(kind, db, kw):
    """step_env_kernel (one workgroup per env: the scalar step on wave 0 while the
    window is in flight, the window advanced through an LDS image) in every reward /
    ring / norm / commission mode, in place and double-buffered, through the ring wrap."""
    from pmenv import TradingEnv
    assert TradingEnv(num_envs=3, num_assets=30, window=50, device=DEV).step_path.count("step_env_kernel") == 2
    _run_both(kw, B=37, N=30, W=50, T=56, kind=kind, seed=zlib.crc32(f"one{kw}{kind}{db}".encode()),
              double_buffer=db, impl="one_launch")


@pytest.mark.parametrize("N,W,B", [(30, 50, 37), (5, 4, 13), (4, 2, 7), (1, 4, 9), (64, 16, 3), (12, 10, 1),
                                   (33, 20, 5), (8, 50, 11), (4, 50, 600), (64, 47, 3)])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_one_launch_shapes(N, W, B, db):
    """Env windows from 2 to 1,000+ chunks: rows straddling chunks, W = 2, one asset,
    envs starting at every offset inside a 1 KiB block, partial last wave, a
    workgroup of one wave."""
    _run_both({}, B=B, N=N, W=W, T=W + 9, kind="mixed", seed=N * 11 + W, double_buffer=db, impl="one_launch")
    _run_both({"ring": "chrono"}, B=B, N=N, W=W, T=W + 3, kind="simplex", seed=N + 5 * W, double_buffer=db,
              impl="one_launch")


def test_gpu_step_impl_selection_rules():
    """The one-launch step takes F = 5, W >= 2, N <= 64 windows whose 1 KiB blocks fit
    15 waves of 4 chunks (64 KiB of LDS); a forced path that does not fit the shape is
    refused (the handle keeps its path) and AUTO falls back by itself."""
    from pmenv import TradingEnv
    big = TradingEnv(num_envs=2, num_assets=64, window=50, device=DEV)       # 4,000 chunks per env
    assert "step_env_kernel" not in big.step_path
    with pytest.raises(ValueError):
        big.set_step_impl("one_launch")
    assert big.step_impl == "auto"
    assert TradingEnv(num_envs=2, num_assets=64, window=47, device=DEV).step_path.count("step_env_kernel") == 2
    assert "step_env_kernel" not in TradingEnv(num_envs=2, num_assets=65, window=4, device=DEV).step_path
    odd = TradingEnv(num_envs=2, num_assets=5, window=50, device=DEV)           # not 16-B granular
    assert odd.step_path == "step_tiny_kernel"
    for impl in ("one_launch", "two_launch"):
        with pytest.raises(ValueError):
            odd.set_step_impl(impl)
    with pytest.raises(ValueError):
        TradingEnv(num_envs=2, num_assets=5, window=8, device=DEV, step_impl="fastest")


def test_gpu_out_must_not_overlap():
    from pmenv import TradingEnv
    env = TradingEnv(num_envs=2, num_assets=5, window=8, device=DEV)
    buf = torch.ones(3, 5, 8, 5, device=DEV)
    obs = buf[:2]
    env.reset(obs)
    with pytest.raises(Exception):
        env.step(torch.full((2, 5), 0.2, device=DEV), obs, bar=torch.ones(2, 5, 4, device=DEV), out=buf[1:])


@pytest.mark.parametrize("N,W,F,B", [
    (129, 50, 5, 9),      # multi-tile: 129 rows > one 32 KiB LDS tile
    (500, 50, 5, 4),      # config 5 asset count (S&P 500)
    (5, 50, 5, 7),        # env block 1250 floats: not 16-B granular -> scalar path
    (64, 16, 5, 5), (65, 16, 5, 5),   # wave-width edges of the per-asset loop
    (7, 6, 3, 11),        # F = 3 (two market channels)
    (3, 1, 5, 4),         # W = 1: the ring is "full" from the first update
    (1, 4, 2, 3),         # single asset, single market channel
])
def test_gpu_vs_oracle_shapes(N, W, F, B):
    kw = {} if F == 5 else {"close_channel": F - 2}
    _run_both(kw, B=B, N=N, W=W, T=2 * W + 3, kind="mixed", F=F, seed=N * 1000 + W)


@pytest.mark.parametrize("N,W,F,B,path", [
    (5, 50, 5, 3, "step_tiny_kernel"),         # config 1: 250-float rows, staged in LDS
    (8, 50, 8, 3, "step_small_kernel"),        # 3,200 floats: 256 x 16
    (32, 32, 8, 5, "step_small_kernel"),       # config/base.py with F = 8: 8,192 floats, 512 x 16
    (30, 50, 8, 4, "step_small_kernel"),       # 12,000 floats: 1,024 x 16
    (3, 7, 5, 9, "step_tiny_kernel"),          # 105 floats, most lanes idle
    (7, 10, 3, 6, "step_tiny_kernel"),
    (64, 8, 4, 5, "step_tiny_kernel"),         # 2,048 floats: the tiny step's largest, 64 assets
    (64, 4, 8, 3, "step_tiny_kernel"),         # 448 bar floats: more than one per thread
    (64, 3, 9, 2, "step_tiny_kernel"),         # 512 bar floats: two per thread, every thread
    (60, 3, 10, 3, "step_small_kernel"),       # 540 bar floats: past the tiny step's staging
    (40, 3, 16, 2, "step_small_kernel"),       # 600 bar floats, F = 16
    (65, 6, 5, 3, "step_small_kernel"),        # N > 64: the LDS-scratch scalar step
    (30, 50, 12, 3, "step_advance_lds_kernel"),   # 18,000 floats: past the register step
])
@pytest.mark.parametrize("kw", [{}, {"ring": "chrono"}, {"commission": 0.0025, "reward": "diff_sharpe"}],
                         ids=["storage", "chrono", "commission"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_register_step_vs_oracle(N, W, F, B, path, kw, db):
    """step_tiny_kernel (env windows <= 2,048 floats, N <= 64: staged in LDS), step_small_kernel
    (one workgroup per env, the window in VGPRs, any F and alignment) and the LDS fallback past
    its 16,384 floats, against the oracle past the ring's wrap."""
    from pmenv import TradingEnv
    kw = dict(kw, **({} if F == 5 else {"close_channel": F - 2}))
    assert TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, **kw).step_path == path
    _run_both(kw, B=B, N=N, W=W, T=2 * W + 3, kind="mixed", F=F, seed=N * 100 + W * 10 + F, double_buffer=db)


@pytest.mark.parametrize("N,W,F,B", [
    (30, 50, 8, 4),       # 12,000 floats per env: three 4,096-float workgroups per env
    (8, 10, 3, 11),       # 240 floats: many envs per workgroup
    (5, 12, 2, 9),        # one market channel
    (9, 8, 4, 13),        # F = 4: every day a whole chunk
    (3, 20, 6, 7),
    (11, 4, 7, 5),        # W = 4: most chunks span two rows' days
    (64, 16, 8, 3),
    (65, 16, 4, 2),       # N > 64: the packed scalar step
    (100, 10, 8, 3),      # N = 100: the packed scalar step, two-envs-per-tile seams
    (30, 50, 12, 4),      # F = 12 (config/base.py's indicators): four halo chunks, 16-B shifted reads
    (8, 10, 16, 11),      # F = 16: the widest, a shift of four whole chunks
    (9, 8, 9, 13),        # F = 9: dword shifted reads past the two-chunk halo
    (11, 4, 10, 5),       # F = 10, W = 4: 8-B shifted reads, chunks across rows
    (3, 20, 13, 7),
    (65, 16, 14, 2),      # N > 64 with F = 14
])
@pytest.mark.parametrize("kw", [{}, {"ring": "chrono"}, {"commission": 0.0025, "reward": "diff_sharpe"}],
                         ids=["storage", "chrono", "commission"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_generic_stream_vs_oracle(N, W, F, B, kw, db):
    """F != 5 on two launches: the scalar step, then advance_gen_kernel (the window staged in
    LDS, the shift by F floats read dword-wise, the in-place halo copied by the scalar step),
    against the oracle past the ring's wrap, with a masked reset midway."""
    from pmenv import TradingEnv
    kw = dict(kw, close_channel=F - 2)
    e = TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, step_impl="two_launch", **kw)
    assert e.step_path.count("advance_gen_kernel") == 2, e.step_path
    rng = np.random.default_rng(N + W + F)
    _run_both(kw, B=B, N=N, W=W, T=2 * W + 3, kind="mixed", F=F, seed=N * 100 + W * 10 + F, double_buffer=db,
              impl="two_launch", resets={W // 2 + 1: rng.random(B) < 0.4})


@pytest.mark.parametrize("F", [8, 12, 16])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_generic_stream_auto_at_size(db, F):
    """AUTO's generic stream on a window past its 2 MiB threshold (600 x 30 x 50 x F: the
    reference loader's F = 8, and its width with config/base.py's indicators on), commission
    and the differential Sharpe, past the ring's wrap."""
    from pmenv import TradingEnv
    kw = {"commission": 0.0025, "reward": "diff_sharpe", "close_channel": F - 2}
    e = TradingEnv(num_envs=600, num_assets=30, window=50, features=F, device=DEV, **kw)
    assert e.step_path.count("advance_gen_kernel") == 2, e.step_path
    _run_both(kw, B=600, N=30, W=50, T=53, kind="mixed", F=F, seed=600 + F, double_buffer=db)


@pytest.mark.parametrize("kw", [{"commission": 0.0025, "reward": "diff_sharpe"}, {"ring": "chrono", "reward": "sharpe_ratio"}],
                         ids=["commission", "chrono"])
def test_gpu_tiny_step_many_envs_modes(kw):
    """step_tiny_kernel with 2,048 envs of config 1's shape in the other reward / ring modes."""
    from pmenv import TradingEnv
    assert TradingEnv(num_envs=2048, num_assets=5, window=50, device=DEV, **kw).step_path == "step_tiny_kernel"
    _run_both(kw, B=2048, N=5, W=50, T=53, kind="mixed", seed=2048)


def test_gpu_generic_stream_auto_threshold():
    """AUTO gives F != 5 windows above 2 MiB the generic stream (16 MiB over the tiny step's
    windows; past the register step's 16,384 floats too, both modes) and keeps the one-launch
    steps below; F = 5, F > 8 and non-granular windows never take it."""
    from pmenv import TradingEnv
    big = TradingEnv(num_envs=48, num_assets=30, window=50, features=8, close_channel=6, device=DEV)   # 2.3 MB
    assert big.step_path.count("advance_gen_kernel") == 2, big.step_path
    small = TradingEnv(num_envs=40, num_assets=30, window=50, features=8, close_channel=6, device=DEV)  # 1.9 MB
    assert small.step_path == "step_small_kernel"
    assert "advance_gen_kernel" not in TradingEnv(num_envs=4096, num_assets=30, window=50, device=DEV).step_path
    # tiny windows (<= 2,048 floats): 16 MiB
    tiny = TradingEnv(num_envs=2048, num_assets=5, window=50, features=8, close_channel=6, device=DEV)  # 16.4 MB
    assert tiny.step_path == "step_tiny_kernel"
    tiny_big = TradingEnv(num_envs=2100, num_assets=5, window=50, features=8, close_channel=6, device=DEV)
    assert tiny_big.step_path.count("advance_gen_kernel") == 2, tiny_big.step_path
    wide = TradingEnv(num_envs=8, num_assets=30, window=50, features=12, close_channel=10, device=DEV)
    wide.set_step_impl("two_launch")                                  # F <= 16 streams (four halo chunks)
    assert wide.step_path.count("advance_gen_kernel") == 2, wide.step_path
    wider = TradingEnv(num_envs=8, num_assets=30, window=50, features=17, close_channel=15, device=DEV)
    with pytest.raises(ValueError):
        wider.set_step_impl("two_launch")
    # past the register step's 16,384 floats per env: the LDS fallback below 2 MiB
    w8 = TradingEnv(num_envs=16, num_assets=100, window=50, features=8, close_channel=6, device=DEV)   # 2.6 MB
    assert w8.step_path.count("advance_gen_kernel") == 2, w8.step_path
    w6 = TradingEnv(num_envs=8, num_assets=64, window=50, features=6, close_channel=4, device=DEV)     # 0.6 MB
    assert w6.step_path == "step_advance_lds_kernel"


@pytest.mark.parametrize("N,W,F,B,path", [
    (5, 50, 5, 4096, "step_tiny_kernel"),      # config 1's env, 4,096 of them (odd envs 8-B aligned)
    (9, 50, 7, 1024, "step_small_kernel"),     # 3,150 floats (8-B granular: AUTO keeps the register step)
    (30, 49, 7, 96, "step_small_kernel"),      # 10,290 floats: 1,024 x 16
    (7, 10, 3, 2048, "step_tiny_kernel"),
])
def test_gpu_register_step_many_envs(N, W, F, B, path):
    """The one-workgroup-per-env steps with thousands of workgroups in flight, in place,
    against the oracle past the ring's wrap."""
    from pmenv import TradingEnv
    kw = {} if F == 5 else {"close_channel": F - 2}
    assert TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, **kw).step_path == path
    _run_both(kw, B=B, N=N, W=W, T=W + 3, kind="mixed", F=F, seed=B + N * 100 + W * 10 + F)


def test_gpu_masked_reset_mid_run():
    B = 20
    rng = np.random.default_rng(5)
    resets = {7: rng.random(B) < 0.3, 15: rng.random(B) < 0.5, 16: np.ones(B, bool)}
    _run_both({}, B=B, N=9, W=8, T=30, kind="simplex", resets=resets)


def test_gpu_state_roundtrip():
    from pmenv import TradingEnv
    B, N, W = 16, 10, 8
    ser = torch.rand(W + 40, B, N, 4, device=DEV) + 1.0
    act = torch.softmax(torch.randn(40, B, N, device=DEV), -1)
    obs = torch.zeros(B, N, W, 5, device=DEV)
    obs[..., :4] = ser[:W].permute(1, 2, 0, 3)
    e1 = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, reward="diff_sharpe")
    e1.reset(obs)
    for t in range(13):
        e1.step(act[t], obs, bar=ser[W + t])
    sd = e1.state_dict()
    obs_ck = obs.clone()
    r1 = [e1.step(act[t], obs, bar=ser[W + t])[0].clone() for t in range(13, 40)]
    e2 = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, reward="diff_sharpe")
    e2.load_state_dict(sd)
    r2 = [e2.step(act[t], obs_ck, bar=ser[W + t])[0].clone() for t in range(13, 40)]
    assert all(torch.equal(a, b) for a, b in zip(r1, r2))
    assert torch.equal(obs, obs_ck) and torch.equal(e1.value, e2.value)


@pytest.mark.parametrize("impl", ["one_launch", "two_launch"])
def test_gpu_full_size_properties(impl):
    """BASELINE config (65,536 envs x 30 assets x 50 x 5) through past the ring wrap,
    by the one-launch step and by the two-launch path (the default here; the nt flat
    streams):
    market channels are exactly the sliding window of the series, the reward is
    log(sum w*y) with y the fp32 close relative, the value compounds the returns,
    and the weight channel is the ring in the reference's storage order."""
    from pmenv import TradingEnv, synth
    B, N, W, F, T = 65536, 30, 50, 5, 60
    ser = synth.series(W + T, B, N, seed=11, device=DEV)
    act = synth.actions(T, B, N, seed=12, device=DEV)
    obs = synth.window_from_series(ser, W, F)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, step_impl=impl)
    assert env.step_path.count("step_env_kernel") == (2 if impl == "one_launch" else 0)
    env.reset(obs)
    logv = torch.full((B,), float(np.log(25000.0)), dtype=torch.float64, device=DEV)
    spare = torch.empty_like(obs)
    for t in range(T):
        # even steps in place, odd steps double-buffered
        if t % 2:
            r, nxt = env.step(act[t], obs, bar=ser[W + t], out=spare)
            obs, spare = nxt, obs
        else:
            r, _ = env.step(act[t], obs, bar=ser[W + t])
        y = (ser[W + t, ..., 3] / ser[W + t - 1, ..., 3]).double()
        ref = torch.log((act[t].double() * y).sum(-1))
        err = (r.double() - ref).abs()
        assert bool((err <= 1e-6 * ref.abs() + 1e-8).all()), f"step {t}: {float(err.max()):.3e}"
        logv += ref
    assert torch.equal(obs[..., :4], ser[T:T + W].permute(1, 2, 0, 3))
    assert torch.allclose(env.value.log(), logv, rtol=0, atol=1e-9)
    chan = obs[..., 4]                                          # [B, N, W]
    assert torch.equal(chan, env.weights.get_all())
    assert bool(env.weights.is_full.all())
    assert torch.allclose(chan.sum(1), torch.ones_like(chan.sum(1)), atol=1e-5)   # simplex per day
    assert env.nonfinite_count() == 0
    # a sample of envs against the oracle on the same inputs, from a fresh reset
    S = 64
    sub = TradingEnv(num_envs=S, num_assets=N, window=W, features=F, device=DEV, step_impl=impl)
    sobs = synth.window_from_series(ser[:, :S].contiguous(), W, F)
    from pmenv.config import EnvConfig
    cenv = OracleEnv(EnvConfig(num_envs=S, num_assets=N, window=W, features=F))
    cobs = sobs.cpu().numpy().copy()
    sub.reset(sobs)
    cenv.reset(cobs)
    ser_h, act_h = ser[:, :S].cpu().numpy(), act[:, :S].cpu().numpy()
    for t in range(T):
        gr, _ = sub.step(act[t, :S].contiguous(), sobs, bar=ser[W + t, :S].contiguous())
        cr, _, _ = cenv.step(act_h[t], cobs, bar=ser_h[W + t])
        assert np.all(np.abs(gr.cpu().numpy() - cr) <= 1e-6 * np.abs(cr) + 1e-9)
    assert np.array_equal(sobs.cpu().numpy(), cobs)


def test_gpu_synth_matches_oracle():
    from pmenv import synth
    s = synth.series(20, 9, 7, env_offset=5, seed=3, device=DEV).cpu().numpy()
    np.testing.assert_allclose(s, synth_series(20, 9, 7, env_offset=5, seed=3), rtol=1e-6)
    a = synth.actions(6, 9, 7, env_offset=5, seed=4, device=DEV).cpu().numpy()
    np.testing.assert_allclose(a, synth_actions(6, 9, 7, env_offset=5, seed=4), rtol=1e-6)


@pytest.mark.parametrize("T,B,kernel", [(300, 10, "scan"), (257, 63, "scan"), (1, 5, "tile16"), (63, 2, "tile16"),
                                        # tiled: T below / across / not a multiple of the segment, ragged B
                                        (37, 100, "tile16"), (64, 64, "tile16"), (129, 4099, "tile16"),
                                        (300, 130, "tile16"), (256, 65536, "tile8"), (37, 16385, "tile8"),
                                        # from 8,192 envs long horizons take the tile, not the split
                                        (2048, 8192, "tile16"),
                                        # the 64-VGPR tile (B >= 65,536, T >= 256): ragged B, T past a segment
                                        (300, 70001, "tile8_occ8"), (256, 65600, "tile8_occ8")])
def test_gpu_gae_kernels_match_oracle(T, B, kernel):
    """GAE(gamma, lambda) over a [T, B] rollout through the kernel each shape takes
    (chunked wave scan for a handful of envs with long horizons, the tiled scan with
    16- or 8-step lane segments) vs the oracle's sequential recursion (parity unpinned
    by the reference)."""
    from pmenv import rollout
    rng = np.random.default_rng(T + B)
    r = rng.standard_normal((T, B)).astype(np.float32)
    v = rng.standard_normal((T + 1, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.02
    adv, ret = rollout.gae(_t(r), _t(v), _t(d, torch.bool), 0.99, 0.95)
    oadv, oret = or_gae(r, v, d, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), oadv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.cpu().numpy(), oret, rtol=1e-5, atol=1e-5)
    adv2, _ = rollout.gae(_t(r), _t(v), None, 0.99, 1.0)            # no dones, lambda = 1: long carries
    oadv2, _ = or_gae(r, v, np.zeros_like(d), 0.99, 1.0)
    np.testing.assert_allclose(adv2.cpu().numpy(), oadv2, rtol=1e-5, atol=1e-4)


def test_gpu_gae_per_env_loop_beyond_tile_offsets():
    """A rollout whose [T+1, B] value array passes the tiled scan's 2^31-byte offsets
    (T = 1, B = 2^28) takes the per-env loop kernel: vs the oracle's recursion on a
    strided sample of envs, and the closed form adv = r + gamma*(1-d)*v1 - v0 for all."""
    from pmenv import rollout
    T, B = 1, 1 << 28
    g = torch.Generator(device=DEV).manual_seed(9)
    r = torch.randn(T, B, device=DEV, generator=g)
    v = torch.randn(T + 1, B, device=DEV, generator=g)
    d = torch.rand(T, B, device=DEV, generator=g) < 0.02
    adv, ret = rollout.gae(r, v, d, 0.99, 0.95)
    expect = (r.double() + 0.99 * (~d).double() * v[1:].double() - v[:1].double()).float()
    assert torch.allclose(adv, expect, rtol=1e-6, atol=1e-6)
    assert torch.allclose(ret, adv + v[:1], rtol=1e-6, atol=1e-6)
    pick = torch.arange(0, B, 4099, device=DEV)
    oadv, oret = or_gae(r[:, pick].cpu().numpy(), v[:, pick].cpu().numpy(), d[:, pick].cpu().numpy(), 0.99, 0.95)
    np.testing.assert_allclose(adv[:, pick].cpu().numpy(), oadv, rtol=1e-6, atol=1e-6)
    del r, v, d, adv, ret, expect
    torch.cuda.empty_cache()


@pytest.mark.parametrize("T,B", [(512, 64), (4096, 512), (1000, 200), (5000, 3), (2048, 4096), (700, 4099),
                                 (16384, 64), (513, 1), (1024, 8191), (640, 65), (1280, 1600)])
def test_gpu_gae_horizon_split_matches_oracle(T, B):
    """The default wrapper path (pmenv_gae_ex): few envs x long horizons split the
    horizon across workgroups in one pass (gae_lookback_kernel: 64- and 128-day chunks,
    one env, ragged env blocks and horizons, the largest B of the rule) — vs the oracle's
    recursion, with episode ends inside and across the chunk boundaries."""
    from pmenv import _abi, rollout
    lib = _abi.load()
    assert lib.pmenv_gae_workspace(T, B) > 0
    rng = np.random.default_rng(T * 7 + B)
    r = rng.standard_normal((T, B)).astype(np.float32)
    v = rng.standard_normal((T + 1, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.003
    adv, ret = rollout.gae(_t(r), _t(v), _t(d, torch.bool), 0.99, 0.95)
    oadv, oret = or_gae(r, v, d, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), oadv, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(ret.cpu().numpy(), oret, rtol=1e-5, atol=1e-5)
    adv2, _ = rollout.gae(_t(r), _t(v), None, 0.99, 1.0)          # no dones, lambda = 1: long carries
    oadv2, _ = or_gae(r, v, np.zeros_like(d), 0.99, 1.0)
    np.testing.assert_allclose(adv2.cpu().numpy(), oadv2, rtol=1e-5, atol=1e-4)


def test_gpu_gae_and_moments_match_oracle():
    from pmenv import rollout
    rng = np.random.default_rng(1)
    T, B = 64, 1000
    r = rng.standard_normal((T, B)).astype(np.float32)
    v = rng.standard_normal((T + 1, B)).astype(np.float32)
    d = rng.random((T, B)) < 0.05
    adv, ret = rollout.gae(_t(r), _t(v), _t(d, torch.bool), 0.99, 0.95)
    oadv, oret = or_gae(r, v, d, 0.99, 0.95)
    np.testing.assert_allclose(adv.cpu().numpy(), oadv, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(ret.cpu().numpy(), oret, rtol=1e-6, atol=1e-6)
    x = rng.standard_normal(1_000_003).astype(np.float32)
    m = rollout.moments(_t(x)).cpu().numpy()
    om = or_moments(x)
    assert m[0] == om[0]
    np.testing.assert_allclose(m[1:], om[1:], rtol=1e-9)


@pytest.mark.parametrize("n,off", [(0, 0), (1, 0), (3, 1), (5, 2), (1000, 3), (4099, 1), (3_000_001, 2)])
def test_gpu_moments_alignment_and_ragged_sizes(n, off):
    """16-B vector body + scalar head/tail: any start alignment and length."""
    from pmenv import rollout
    rng = np.random.default_rng(n + off)
    x = rng.standard_normal(n + off).astype(np.float32)
    m = rollout.moments(_t(x)[off:]).cpu().numpy()
    om = or_moments(np.ascontiguousarray(x[off:]))
    assert m[0] == om[0] == n
    np.testing.assert_allclose(m[1:], om[1:], rtol=1e-9, atol=1e-9)


def test_gpu_errors_mirror_reference():
    from pmenv import TradingEnv
    env = TradingEnv(num_envs=2, num_assets=5, window=8, device=DEV)
    obs = torch.zeros(2, 5, 8, 5, device=DEV)
    env.reset(obs)
    with pytest.raises(ValueError):               # weight_buffer.py:18-19
        env.step(torch.ones(2, 4, device=DEV), obs, torch.ones(2, 5, device=DEV))
    with pytest.raises(ValueError):
        env.step(torch.ones(2, 5, device=DEV), obs)
    with pytest.raises(ValueError):
        env.step(torch.ones(2, 5, device=DEV), obs.double(), torch.ones(2, 5, device=DEV))


def test_gpu_nonfinite_counter():
    from pmenv import TradingEnv
    env = TradingEnv(num_envs=3, num_assets=4, window=4, device=DEV)
    obs = torch.ones(3, 4, 4, 5, device=DEV)
    env.reset(obs)
    a = torch.full((3, 4), 0.25, device=DEV)
    a[1, 2] = float("nan")
    env.step(a, obs, torch.ones(3, 4, device=DEV))
    assert env.nonfinite_count() == 1


def test_gpu_step_is_graph_capturable():
    from pmenv import TradingEnv, synth
    B, N, W, T = 256, 30, 50, 8
    ser = synth.series(W + T, B, N, device=DEV)
    act = synth.actions(T, B, N, device=DEV)
    obs_a = synth.window_from_series(ser, W)
    obs_b = obs_a.clone()
    ea = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    eb = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    ea.reset(obs_a)
    eb.reset(obs_b)
    torch.cuda.synchronize()
    from pmenv import _abi
    import ctypes
    lib = _abi.load()
    rew = torch.empty(T, B, device=DEV)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(T):
            _abi.check(lib.pmenv_step(eb._h, ctypes.c_void_p(act[t].data_ptr()), None,
                                      ctypes.c_void_p(ser[W + t].data_ptr()), ctypes.c_void_p(obs_b.data_ptr()),
                                      ctypes.c_void_p(rew[t].data_ptr()), s), eb._h)
    eb.reset(obs_b)            # capture does not execute; start both from reset
    obs_b.copy_(synth.window_from_series(ser, W))
    eb.reset(obs_b)
    g.replay()
    ref = torch.stack([ea.step(act[t], obs_a, bar=ser[W + t])[0] for t in range(T)])
    torch.cuda.synchronize()
    assert torch.equal(ref, rew) and torch.equal(obs_a, obs_b)


@pytest.mark.parametrize("impl", ["one_launch", "two_launch"])
def test_gpu_resident_series_equals_bar_batch(impl):
    """Resident-series data path (env b reads series[day[b]]) == stepping with the
    gathered bar batch, bit for bit; windows initialised from per-env start days."""
    from pmenv import TradingEnv, MarketSeries
    rng = np.random.default_rng(2)
    T, N, W, B, S = 300, 30, 50, 97, 40
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((T, N)), axis=0))
    bars = np.stack([closes * np.exp(0.002 * rng.standard_normal((T, N))) for _ in range(3)] + [closes], -1)
    m = MarketSeries(bars.astype(np.float32), device=DEV)
    start = m.random_starts(B, W, S, generator=torch.Generator().manual_seed(0))
    obs_a = m.initial_window(start, W)
    ref = np.stack([bars[int(s):int(s) + W].transpose(1, 0, 2) for s in start.cpu()]).astype(np.float32)
    assert np.array_equal(obs_a[..., :4].cpu().numpy(), ref)
    obs_b = obs_a.clone()
    ea = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl)
    eb = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=impl)
    ea.reset(obs_a)
    eb.reset(obs_b)
    act = torch.softmax(torch.randn(S, B, N, device=DEV), -1)
    for t in range(S):
        day = start + W + t
        ra, _ = ea.step(act[t], obs_a, series=m, day=day)
        rb, _ = eb.step(act[t], obs_b, bar=m.bars[day.long()].contiguous())
        assert torch.equal(ra, rb)
    assert torch.equal(obs_a, obs_b) and torch.equal(ea.value, eb.value)
    # a day outside the series is reported, not read
    bad = start + W + S
    bad[3] = T + 5
    ea.step(act[0], obs_a, series=m, day=bad)
    assert ea.nonfinite_count() == 1


@pytest.mark.parametrize("N,W,F,B,impl,path", [
    (30, 50, 8, 512, "auto", "advance_gen_kernel"),     # 24.6 MB: AUTO's generic stream
    (8, 10, 3, 33, "two_launch", "advance_gen_kernel"),
    (30, 50, 8, 4, "auto", "step_small_kernel"),
    (5, 50, 5, 9, "auto", "step_tiny_kernel"),          # config 1's env
    (8, 10, 3, 600, "auto", "step_tiny_kernel"),
])
def test_gpu_resident_series_any_F_equals_bar_batch(N, W, F, B, impl, path):
    """The resident-series data path (env b reads series[day[b]], the day read on the device)
    through the F != 5 and small-window kernels == stepping with the gathered bar batch, bit for
    bit, both in place; a day outside the series gives NaN bars and is reported."""
    from pmenv import TradingEnv, MarketSeries
    rng = np.random.default_rng(N + W + F)
    T, S = 3 * W + 40, 2 * W + 3
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((T, N)), axis=0))
    chans = [closes * np.exp(0.002 * rng.standard_normal((T, N))) for _ in range(F - 2)] + [closes]
    bars = np.stack(chans, -1).astype(np.float32)                       # [T, N, F - 1], close last
    m = MarketSeries(bars, device=DEV)
    start = m.random_starts(B, W, S, generator=torch.Generator().manual_seed(F))
    obs_a = m.initial_window(start, W)
    obs_b = obs_a.clone()
    kw = dict(num_envs=B, num_assets=N, window=W, features=F, close_channel=F - 2, device=DEV, step_impl=impl)
    ea, eb = TradingEnv(**kw), TradingEnv(**kw)
    assert path in ea.step_path.split(" | ")[-1], ea.step_path
    ea.reset(obs_a)
    eb.reset(obs_b)
    act = torch.softmax(torch.randn(S, B, N, device=DEV), -1)
    for t in range(S):
        day = start + W + t
        ra, _ = ea.step(act[t], obs_a, series=m, day=day)
        rb, _ = eb.step(act[t], obs_b, bar=m.bars[day.long()].contiguous())
        assert torch.equal(ra.view(torch.int32), rb.view(torch.int32)), f"step {t}"
    assert torch.equal(obs_a.view(torch.int32), obs_b.view(torch.int32)) and torch.equal(ea.value, eb.value)
    bad = start + W + S                   # the day after the horizon: past the series for the latest starts
    bad[B // 2] = T + 5
    ea.step(act[0], obs_a, series=m, day=bad)
    outside = (bad >= T).cpu().numpy()
    assert ea.nonfinite_count() == int(outside.sum())
    nan_rows = torch.isnan(obs_a[:, :, W - 1, :F - 1]).all(-1).all(-1).cpu().numpy()
    assert np.array_equal(nan_rows, outside)


@pytest.mark.parametrize("T,N,W,B,H,S", [
    (200, 30, 12, 33, 40, 64),     # F = 5 vector staging (4 pairs per thread), persistent gather
    (300, 30, 50, 17, 80, 64),     # F = 5, 8 pairs per thread (BASELINE shape)
    (200, 30, 12, 33, 40, 1301),   # persistent loop: several samples per workgroup, ragged tail
    (60, 3, 5, 4, 9, 64),          # LDS-staged, sample block not 16-B granular
    (120, 300, 50, 3, 60, 16)])    # staged days > 64 KiB: per-float kernel
def test_gpu_replay_gather_matches_restatement(T, N, W, B, H, S):
    """replay/buffer.py:39-79 sample on device vs the numpy restatement
    (the reference module is not importable: parity restated from its text)."""
    from pmenv import MarketSeries
    from pmenv.replay import DeviceReplay
    from oracle import replay_gather
    rng = np.random.default_rng(4)
    bars = (100 * np.exp(0.01 * rng.standard_normal((T, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    rb = DeviceReplay(B, N, W, H, m)
    for h in range(H + 17):                      # wraps the ring; some windows run off the series ends
        rb.add(torch.full((B,), (W + h) % (T + 3) - 2, dtype=torch.int32, device=DEV),
               torch.rand(B, N, device=DEV), torch.randn(B, device=DEV))
    h0, env = rb.indices(S, generator=torch.Generator().manual_seed(1))
    s, a, r, s2 = rb.gather(h0, env)
    es, ea, er, es2 = replay_gather(bars, rb.days.cpu().numpy(), rb.actions.cpu().numpy(), rb.rewards.cpu().numpy(),
                                    h0.cpu().numpy(), env.cpu().numpy(), W)
    assert np.array_equal(s.cpu().numpy(), es, equal_nan=True)
    assert np.array_equal(s2.cpu().numpy(), es2, equal_nan=True)
    assert np.array_equal(a.cpu().numpy()[..., 0], ea) and np.array_equal(r.cpu().numpy()[:, 0, 0], er)


def test_gpu_replay_gather_full_size_persistent():
    """The replay at the f4 bench shape (4,096 envs x 256 recorded steps, 8,192 samples
    of 30 assets x 50 days): the persistent gather (one workgroup per CU, ~32 samples
    each, the next sample's loads in flight) vs the restatement on 512 of the samples."""
    from pmenv import MarketSeries
    from pmenv.replay import DeviceReplay
    from oracle import replay_gather
    B, N, W, H, S, T = 4096, 30, 50, 256, 8192, 700
    rng = np.random.default_rng(11)
    bars = (100 * np.exp(0.01 * rng.standard_normal((T, N, 4)).cumsum(0))).astype(np.float32)
    m = MarketSeries(bars, device=DEV)
    rb = DeviceReplay(B, N, W, H, m)
    g = torch.Generator(device=DEV).manual_seed(5)
    day0 = torch.randint(W, T - H - 2, (B,), device=DEV, generator=g, dtype=torch.int32)
    for h in range(H + 40):                      # wraps the ring
        rb.add(day0 + h % H, torch.rand(B, N, device=DEV, generator=g), torch.randn(B, device=DEV, generator=g))
    h0, env = rb.indices(S, generator=torch.Generator().manual_seed(6))
    s, a, r, s2 = rb.gather(h0, env)
    pick = np.sort(np.random.default_rng(7).choice(S, 512, replace=False))
    es, ea, er, es2 = replay_gather(bars, rb.days.cpu().numpy(), rb.actions.cpu().numpy(), rb.rewards.cpu().numpy(),
                                    h0.cpu().numpy()[pick], env.cpu().numpy()[pick], W)
    assert np.array_equal(s.cpu().numpy()[pick], es, equal_nan=True)
    assert np.array_equal(s2.cpu().numpy()[pick], es2, equal_nan=True)
    assert np.array_equal(a.cpu().numpy()[pick, :, 0], ea) and np.array_equal(r.cpu().numpy()[pick, 0, 0], er)


@pytest.mark.parametrize("B,N,W,T", [(300, 30, 20, 80), (5, 300, 4, 9), (70, 1, 3, 2), (9, 257, 2, 5),
                                     (4097, 30, 10, 252)])
def test_gpu_trajectory_metrics_match_restatement(B, N, W, T):
    """util/eval.py:14-37 metrics over an env trajectory vs the numpy restatement
    (quantstats is absent: parity unpinned by the reference)."""
    from pmenv import TradingEnv, synth
    from pmenv.replay import trajectory_metrics
    from oracle import trajectory_metrics as ref_metrics
    ser = synth.series(W + T, B, N, device=DEV)
    act = synth.actions(T, B, N, device=DEV)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, track_info=True)
    env.reset(obs)
    for t in range(T):
        env.step(act[t], obs, bar=ser[W + t])
    rets = torch.stack(env.info["returns"][1:]) - 1.0
    vals = torch.stack(env.info["values"])
    wts = torch.stack(env.info["actions"])
    got = trajectory_metrics(rets, vals, wts)
    exp = ref_metrics(rets.cpu().numpy(), vals.cpu().numpy(), wts.cpu().numpy())
    for i, k in enumerate(("sharpe", "sortino", "max_drawdown", "average_turnover", "final_value")):
        np.testing.assert_allclose(got[k].cpu().numpy(), exp[:, i], rtol=1e-6, atol=1e-9, err_msg=k)


def test_gpu_beyond_flat_index_range_in_place():
    """A window past the flat stream's 32-bit chunk index (1.2 M envs x 30 x 50 x 5 =
    36 GB, 2.25e9 chunks): the one-launch step (64-bit env offsets) and the two-launch
    fallback (the row kernel) each step in place, shifting every sampled env's window
    by one day, appending its bar and writing a finite reward (start, middle and end
    of the tensor)."""
    from pmenv import TradingEnv
    B, N, W = 1_200_000, 30, 50
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV)
    assert env.step_path.split(" | ")[1].startswith("step_env_kernel")     # AUTO: no flat stream here
    g = torch.Generator(device=DEV).manual_seed(3)
    obs = torch.rand(B, N, W, 5, device=DEV, generator=g) + 0.5
    env.reset(obs)
    pick = torch.tensor([0, 1, B // 2, B - 2, B - 1], device=DEV)
    for impl in ("one_launch", "two_launch"):
        env.set_step_impl(impl)
        if impl == "two_launch":
            assert "advance_rows_kernel" in env.step_path.split(" | ")[1]
        bar = torch.rand(B, N, 4, device=DEV, generator=g) + 0.5
        act = torch.softmax(torch.randn(B, N, device=DEV, generator=g), -1)
        before = obs[pick].clone()
        r, out = env.step(act, obs, bar=bar)
        assert out is obs
        after = obs[pick]
        assert torch.equal(after[:, :, :-1, :], before[:, :, 1:, :])
        assert torch.equal(after[:, :, -1, :4], bar[pick])
        assert torch.isfinite(r).all() and env.nonfinite_count() == 0
        del bar, act
    del obs, env
    torch.cuda.empty_cache()
