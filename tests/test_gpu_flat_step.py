"""step_flat_kernel: the whole advance step in ONE launch over fixed 16 KiB tiles of the
flat window (the scalar step run by every workgroup an env straddles, the env's state
written by its owner, a per-step snapshot and in-place halo by parity; step_flat.h).

Checked against the CPU oracle in every mode, bit for bit against the two-launch path
(and so against every other path) across resets, masked resets, checkpoint restores,
path switches, resident-series days and hipGraph capture, and at the BASELINE shape.
Needs an MI355X."""
import zlib

import numpy as np
import pytest
import torch

from test_gpu_parity import DEV, MODES, _gpu, _run_both  # noqa: F401  (_gpu: autouse fixture)

pytestmark = pytest.mark.gpu

# (N, W, B): envs of 150 .. 3,760 chunks, i.e. 1 .. 8 envs per 1,024-chunk tile, rows
# straddling chunks, envs at every offset in a tile, a partial last tile
SHAPES = [(30, 50, 37), (4, 50, 600), (4, 30, 301), (12, 10, 97), (64, 47, 3), (8, 50, 11), (64, 16, 5),
          (33, 20, 5), (2, 60, 130), (1, 600, 9), (64, 2, 50), (40, 3, 21)]   # W = 2, 3: most days are last days


def _mode_id(k):
    return "-".join(f"{a}={b}" for a, b in k.items()) or "reference"


@pytest.mark.parametrize("kind", ["simplex", "mixed", "rawpos"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
@pytest.mark.parametrize("kw", MODES, ids=_mode_id)
def test_gpu_flat_vs_oracle_modes(kind, db, kw):
    """Every reward / ring / norm / commission mode, in place and double-buffered, past
    the ring wrap, against the oracle."""
    _run_both(kw, B=37, N=30, W=50, T=56, kind=kind, seed=zlib.crc32(f"flat{kw}{kind}{db}".encode()),
              double_buffer=db, impl="flat")


@pytest.mark.parametrize("N,W,B", SHAPES)
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_flat_shapes_vs_oracle(N, W, B, db):
    _run_both({}, B=B, N=N, W=W, T=W + 7, kind="mixed", seed=N * 13 + W, double_buffer=db, impl="flat")
    _run_both({"ring": "chrono"}, B=B, N=N, W=W, T=W + 3, kind="simplex", seed=N + 7 * W, double_buffer=db,
              impl="flat")


def _state(e):
    return (e._value.clone(), e._counter.clone(), e._ring.clone(), e._w_new.clone(), e._last_close.clone(),
            e._stat_a.clone(), e._stat_b.clone())


def _same(ga, gb, what):
    for i, (x, y) in enumerate(zip(ga, gb)):
        assert torch.equal(x.nan_to_num(7.0), y.nan_to_num(7.0)), f"{what}: state field {i}"


@pytest.mark.parametrize("N,W,B", [(30, 50, 37), (4, 30, 301), (64, 47, 3)])
@pytest.mark.parametrize("kw", [dict(), dict(commission=0.0025, reward="sharpe_ratio"),
                                dict(ring="chrono", reward="diff_sharpe")], ids=_mode_id)
def test_gpu_flat_bitwise_vs_two_launch_through_state_changes(N, W, B, kw):
    """The flat one-launch step and the two-launch path, driven with the same inputs
    through everything that invalidates the snapshot / halo — full and masked resets,
    a checkpoint restore, a switch to another path and back, a different window buffer,
    in place and double-buffered steps, prices given, resident-series days — agree on
    every window, reward, returned weight and state field, bit for bit."""
    from pmenv import TradingEnv, synth
    T = W + 24
    ser = synth.series(W + T, B, N, seed=zlib.crc32(f"{N}{W}{kw}".encode()), device=DEV)
    act = synth.actions(T, B, N, seed=5, device=DEV)
    kind_mixed = torch.randn(T, B, N, device=DEV, generator=torch.Generator(DEV).manual_seed(3))
    res = synth.series(T + W + 8, 1, N, seed=9, device=DEV)[:, 0].contiguous()
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i, track_info=True, **kw)
            for i in ("flat", "two_launch")]
    assert "step_flat_kernel" in envs[0].step_path and "step_flat_kernel" not in envs[1].step_path
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
            if mask9 is not None:                         # masked reset mid-run
                e.reset(obs[i], mask=mask9)
            if t == 14:                                   # checkpoint (state and window)
                cks[i], obs_cks[i] = e.state_dict(), obs[i].clone()
            if t == 20 and i == 0:
                e.set_step_impl("two_launch")             # another path writes the state...
            if t == 22 and i == 0:
                e.set_step_impl("flat")                   # ...and the flat step re-primes
            if t == 26:                                   # restore the t = 14 checkpoint
                e.load_state_dict(cks[i])
                obs[i].copy_(obs_cks[i])
            wo = torch.empty(B, N, device=DEV)
            if t % 4 == 1:                                # double-buffered
                r, obs[i] = e.step(a, obs[i], bar=ser[W + t], out=torch.empty_like(obs[i]), weights_out=wo)
            elif t % 7 == 5:                              # a fresh window buffer, in place
                obs[i] = obs[i].clone()
                r, _ = e.step(a, obs[i], bar=ser[W + t], weights_out=wo)
            elif t % 6 == 2:                              # resident-series days
                day = torch.full((B,), t + W, dtype=torch.int32, device=DEV)
                day[::3] += 2
                r, _ = e.step(a, obs[i], series=res, day=day, weights_out=wo)
            elif t % 9 == 4:                              # caller prices
                r, _ = e.step(a, obs[i], bar=ser[W + t], prices=ser[W + t, ..., 3] / ser[W + t - 1, ..., 3],
                              weights_out=wo)
            else:
                r, _ = e.step(a, obs[i], bar=ser[W + t], weights_out=wo)
            outs.append((r.clone(), wo, e.info["returns"][-1]))
        assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
        assert torch.equal(outs[0][0].nan_to_num(7.0), outs[1][0].nan_to_num(7.0)), f"step {t}: rewards"
        assert torch.equal(outs[0][1], outs[1][1]), f"step {t}: weights"
        assert torch.equal(outs[0][2].nan_to_num(7.0), outs[1][2].nan_to_num(7.0)), f"step {t}: returns"
        _same(_state(envs[0]), _state(envs[1]), f"step {t}")


def test_gpu_flat_masked_reset_same_mask():
    """Masked resets every sixth step on both paths, state compared after each step."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 300, 4, 30, 40
    ser = synth.series(W + T, B, N, seed=1, device=DEV)
    act = synth.actions(T, B, N, seed=2, device=DEV)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("flat", "two_launch")]
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    g = torch.Generator(DEV).manual_seed(4)
    for t in range(T):
        mask = torch.rand(B, device=DEV, generator=g) < 0.2 if t % 6 == 5 else None
        rs = []
        for e, o in zip(envs, obs):
            if mask is not None:
                e.reset(o, mask=mask)
            rs.append(e.step(act[t], o, bar=ser[W + t])[0])
        assert torch.equal(obs[0], obs[1]) and torch.equal(rs[0], rs[1]), f"step {t}"
        _same(_state(envs[0]), _state(envs[1]), f"step {t}")


def test_gpu_flat_graph_capture_and_replay():
    """Flat steps captured into a hipGraph (an odd count, so a host-chosen parity would
    go wrong on the second replay): the handle switches to the device-sequenced form and
    graph replays interleave with eager steps, a full reset, a masked reset and a
    checkpoint restore — every reward, value and window equal to an eager two-launch env
    on the same inputs, bit for bit."""
    import ctypes
    from pmenv import TradingEnv, synth, _abi
    B, N, W, T, D = 2048, 30, 50, 5, 48
    ser = synth.series(W + D, B, N, seed=7, device=DEV)
    act = synth.actions(D, B, N, seed=8, device=DEV)
    ea = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="two_launch")
    eb = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="flat")
    obs_a = synth.window_from_series(ser, W)
    obs_b = obs_a.clone()
    ea.reset(obs_a)
    eb.reset(obs_b)
    day = 0

    def eager(n):
        nonlocal day
        for _ in range(n):
            ra, _ = ea.step(act[day], obs_a, bar=ser[W + day])
            rb, _ = eb.step(act[day], obs_b, bar=ser[W + day])
            assert torch.equal(ra, rb) and torch.equal(obs_a, obs_b), f"eager day {day}"
            day += 1

    eager(3)                                               # host-sequenced flat steps first
    lib = _abi.load()
    act_buf = torch.empty(T, B, N, device=DEV)
    bar_buf = torch.empty(T, B, N, 4, device=DEV)
    rew_b = torch.empty(T, B, device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(T):
            _abi.check(lib.pmenv_step(eb._h, ctypes.c_void_p(act_buf[t].data_ptr()), None,
                                      ctypes.c_void_p(bar_buf[t].data_ptr()), ctypes.c_void_p(obs_b.data_ptr()),
                                      ctypes.c_void_p(rew_b[t].data_ptr()), s), eb._h)
    assert "device-sequenced" in eb.step_path

    def replay():
        nonlocal day
        act_buf.copy_(act[day:day + T])
        bar_buf.copy_(ser[W + day:W + day + T])
        g.replay()
        ref = torch.stack([ea.step(act[day + t], obs_a, bar=ser[W + day + t])[0] for t in range(T)])
        torch.cuda.synchronize()
        assert torch.equal(ref, rew_b), f"replay from day {day}: rewards"
        assert torch.equal(obs_a, obs_b) and torch.equal(ea.value, eb.value), f"replay from day {day}"
        day += T

    replay()
    replay()                                               # the same graph: parity from the device
    eager(2)                                               # eager, device-sequenced
    replay()
    fresh = synth.window_from_series(ser[day:day + W + 1].contiguous(), W)
    obs_a.copy_(fresh)
    obs_b.copy_(fresh)
    ea.reset(obs_a)
    eb.reset(obs_b)                                        # invalidates on the device
    replay()
    mask = torch.rand(B, device=DEV, generator=torch.Generator(DEV).manual_seed(1)) < 0.3
    ea.reset(obs_a, mask=mask)
    eb.reset(obs_b, mask=mask)
    eager(1)
    ck_a, ck_b, ck_obs = ea.state_dict(), eb.state_dict(), obs_a.clone()
    replay()
    ea.load_state_dict(ck_a)
    eb.load_state_dict(ck_b)
    obs_a.copy_(ck_obs)
    obs_b.copy_(ck_obs)
    day -= T
    replay()                                               # from the restored checkpoint
    eager(2)
    assert day <= D


def test_gpu_flat_graph_captures_a_reset_before_its_steps():
    """A hipGraph whose first node is a reset (masked) followed by flat steps, captured on a
    handle that was host-sequenced until then: the captured reset clears the snapshot's
    valid word, so every replay re-primes from the reset state — replays 2, 3, ... included,
    where a validity left at 1 by the previous replay would compose straddling envs from
    the pre-reset snapshot. Equal to an eager two-launch env doing the same, bit for bit."""
    import ctypes
    from pmenv import TradingEnv, synth, _abi
    B, N, W, T, D = 2048, 30, 50, 3, 40
    ser = synth.series(W + D, B, N, seed=17, device=DEV)
    act = synth.actions(D, B, N, seed=18, device=DEV)
    ea = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="two_launch")
    eb = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="flat")
    obs_a = synth.window_from_series(ser, W)
    obs_b = obs_a.clone()
    ea.reset(obs_a)
    eb.reset(obs_b)
    for day in range(2):                                   # host-sequenced flat steps first
        ea.step(act[day], obs_a, bar=ser[W + day])
        eb.step(act[day], obs_b, bar=ser[W + day])
    assert torch.equal(obs_a, obs_b)
    lib = _abi.load()
    mask = (torch.rand(B, device=DEV, generator=torch.Generator(DEV).manual_seed(2)) < 0.5).to(torch.uint8)
    act_buf = torch.empty(T, B, N, device=DEV)
    bar_buf = torch.empty(T, B, N, 4, device=DEV)
    rew_b = torch.empty(T, B, device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    p = lambda x: ctypes.c_void_p(x.data_ptr())  # noqa: E731
    with torch.cuda.graph(g):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _abi.check(lib.pmenv_reset(eb._h, p(obs_b), p(mask), s), eb._h)
        for t in range(T):
            _abi.check(lib.pmenv_step(eb._h, p(act_buf[t]), None, p(bar_buf[t]), p(obs_b), p(rew_b[t]), s), eb._h)
    assert "device-sequenced" in eb.step_path
    day = 2
    for rep in range(4):
        act_buf.copy_(act[day:day + T])
        bar_buf.copy_(ser[W + day:W + day + T])
        g.replay()
        ea.reset(obs_a, mask=mask)
        ref = torch.stack([ea.step(act[day + t], obs_a, bar=ser[W + day + t])[0] for t in range(T)])
        torch.cuda.synchronize()
        assert torch.equal(ref, rew_b), f"replay {rep}: rewards"
        assert torch.equal(obs_a, obs_b) and torch.equal(ea.value, eb.value), f"replay {rep}: windows / values"
        assert torch.equal(ea._counter, eb._counter), f"replay {rep}: counters"
        day += T
    ra, _ = ea.step(act[day], obs_a, bar=ser[W + day])     # eager after the replays
    rb, _ = eb.step(act[day], obs_b, bar=ser[W + day])
    assert torch.equal(ra, rb) and torch.equal(obs_a, obs_b)


def test_gpu_flat_caller_edits_between_steps():
    """The features are the caller's (trading_env.py:102-105: the reference keeps no copy
    and honours every edit). At the BASELINE shape the caller, between steps and without a
    reset, rescales the market channels of the in-place window, writes env.value, and hands
    in the window as a new tensor at the old one's address: the flat one-launch step (tile
    halo and state snapshot from the previous step) equals the two-launch path (which
    keeps nothing) bit for bit, because TradingEnv tells the handle what changed
    (pmenv_window_written / pmenv_state_written). The wrapper's check costs well under a
    microsecond of host time per step."""
    import time
    from pmenv import TradingEnv, synth
    B, N, W, T = 65536, 30, 50, 12
    ser = synth.series(W + T, B, N, seed=31, device=DEV)
    act = synth.actions(T, B, N, seed=32, device=DEV)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("flat", "two_launch")]
    assert envs[0].step_path.endswith("step_flat_kernel (in place)")
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    reused = 0
    for t in range(T):
        for i, e in enumerate(envs):
            if t in (2, 7):                                # edit the window in place (every tile seam)
                obs[i][..., :4].mul_(1.0009765625)
            if t == 8:                                     # and its weight channel
                obs[i][..., 4].mul_(0.5)
            if t in (3, 9):                                # write the state through .value
                e.value.mul_(0.75)
            if t == 5:                                     # a new tensor, likely at the same address
                keep = obs[i].clone()
                keep[..., 3].mul_(0.998046875)
                old = obs[i].data_ptr()
                obs[i] = None
                obs[i] = torch.empty_like(keep)
                obs[i].copy_(keep)
                del keep
                reused += obs[i].data_ptr() == old
        rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
        assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
        assert torch.equal(envs[0].value, envs[1].value), f"step {t}: values"
    print(f"new window at the old address: {reused} of 2")
    e, o = envs[0], obs[0]
    st = e._stream()
    n = 20000
    t0 = time.perf_counter()
    for _ in range(n):
        e._edits(o, st)
        e._watch(o)
    per = (time.perf_counter() - t0) / n
    print(f"edit check + watch: {per * 1e6:.3f} us per step")
    assert per < 2e-5             # host timing on a shared box: a generous bound, not a benchmark


def test_gpu_flat_announced_writes_that_bypass_version_counters():
    """Writes torch's version counters do not see (through `.data` here; DLPack, raw kernels
    and edits between graph replays alike) are announced with TradingEnv.window_written /
    state_written: the flat step (halo and snapshot kept from the previous step) then equals
    the two-launch path (which keeps nothing) bit for bit."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 16384, 30, 50, 8
    ser = synth.series(W + T, B, N, seed=41, device=DEV)
    act = synth.actions(T, B, N, seed=42, device=DEV)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("flat", "two_launch")]
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    for t in range(T):
        for e, o in zip(envs, obs):
            if t in (2, 5):
                v = o._version
                o.data[..., :4].mul_(1.0009765625)           # invisible to o's version counter
                assert o._version == v
                e.window_written(o)
            if t == 4:
                e._value.data.mul_(0.75)                   # invisible to the state's counter
                e.state_written()
        rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
        assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
        assert torch.equal(envs[0].value, envs[1].value), f"step {t}: values"


def test_gpu_flat_path_rules():
    """FLAT takes F = 5, W >= 2, N <= 64 windows of >= 148 chunks (at most one env per
    wave of a tile: 256 x 4 from 511 chunks, 512 x 2 below); a forced FLAT that does not
    fit is refused and the handle keeps its path."""
    from pmenv import TradingEnv
    ok = TradingEnv(num_envs=5, num_assets=30, window=50, device=DEV, step_impl="flat")
    assert ok.step_path == "step_flat_kernel (obs_out) | step_flat_kernel (in place)"
    for n, w in [(1, 4), (4, 20), (65, 50)]:           # 5 / 100 chunks per env; N > 64
        e = TradingEnv(num_envs=5, num_assets=n, window=w, device=DEV)
        before = e.step_path
        with pytest.raises(ValueError):
            e.set_step_impl("flat")
        assert e.step_path == before


def test_gpu_flat_full_size_properties():
    """BASELINE config (65,536 envs x 30 x 50 x 5) by the flat one-launch step, through
    the ring wrap, alternating in place and double-buffered: the market channels are the
    sliding series, the reward log(sum w*y), the value compounds the returns, the weight
    channel is get_all(); and a 64-env sample against the oracle."""
    from oracle import OracleEnv
    from pmenv import TradingEnv, synth
    from pmenv.config import EnvConfig
    B, N, W, F, T = 65536, 30, 50, 5, 60
    ser = synth.series(W + T, B, N, seed=21, device=DEV)
    act = synth.actions(T, B, N, seed=22, device=DEV)
    obs = synth.window_from_series(ser, W, F)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, features=F, device=DEV, step_impl="flat")
    env.reset(obs)
    logv = torch.full((B,), float(np.log(25000.0)), dtype=torch.float64, device=DEV)
    spare = torch.empty_like(obs)
    for t in range(T):
        if t % 3 == 2:
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
    assert torch.equal(obs[..., 4], env.weights.get_all())
    assert env.nonfinite_count() == 0
    S = 64
    cenv = OracleEnv(EnvConfig(num_envs=S, num_assets=N, window=W, features=F))
    cobs = synth.window_from_series(ser[:, :S].contiguous(), W, F).cpu().numpy().copy()
    cenv.reset(cobs)
    ser_h, act_h = ser[:, :S].cpu().numpy(), act[:, :S].cpu().numpy()
    for t in range(T):
        cr, _, _ = cenv.step(act_h[t], cobs, bar=ser_h[W + t])
    np.testing.assert_allclose(env.value[:S].cpu().numpy(), cenv.value, rtol=1e-12)
    assert np.array_equal(obs[:S, ..., :4].cpu().numpy(), cobs[..., :4])
    np.testing.assert_allclose(obs[:S, ..., 4].cpu().numpy(), cobs[..., 4], rtol=2e-7, atol=1e-12)


def test_gpu_flat_long_run_bitwise_at_baseline_size():
    """400 steps at the BASELINE shape (65,536 envs x 30 x 50) on a resident series, the
    flat one-launch step against the two-launch path: in place with a double-buffered
    step every 7th day and masked resets (a fifth of the envs, fresh windows) every 50
    days; windows, rewards, values and counters compared bit for bit every 20 steps and
    at the end. A rare ordering fault in the snapshot / halo sequencing would surface
    here."""
    from pmenv import TradingEnv, MarketSeries
    B, N, W, T = 65536, 30, 50, 400
    rng = np.random.default_rng(11)
    days = W + T + 64
    closes = 100 * np.exp(np.cumsum(0.01 * rng.standard_normal((days, N)), axis=0))
    bars = np.stack([closes * np.exp(0.002 * rng.standard_normal((days, N))) for _ in range(3)] + [closes], -1)
    m = MarketSeries(bars.astype(np.float32), device=DEV)
    g = torch.Generator().manual_seed(5)
    start = m.random_starts(B, W, T, generator=g)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("flat", "two_launch")]
    obs = [m.initial_window(start, W) for _ in envs]
    spare = [torch.empty_like(obs[0]) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    day = start.clone()
    gd = torch.Generator(DEV).manual_seed(6)
    for t in range(T):
        a = torch.softmax(torch.randn(B, N, device=DEV, generator=gd), -1)
        d = day + W + t
        if t and t % 50 == 0:
            mask = torch.rand(B, device=DEV, generator=gd) < 0.2
            fresh = m.initial_window(torch.where(mask, start, d - W).to(torch.int32), W)
            for i, e in enumerate(envs):
                obs[i][mask] = fresh[mask]
                e.reset(obs[i], mask=mask)
        rs = []
        for i, e in enumerate(envs):
            if t % 7 == 3:
                r, nxt = e.step(a, obs[i], series=m, day=d, out=spare[i])
                obs[i], spare[i] = nxt, obs[i]
            else:
                r, _ = e.step(a, obs[i], series=m, day=d)
            rs.append(r)
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
        if t % 20 == 19 or t == T - 1:
            assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
            assert torch.equal(envs[0].value, envs[1].value), f"step {t}: values"
            assert torch.equal(envs[0]._counter, envs[1]._counter), f"step {t}: counters"
    assert envs[0].nonfinite_count() == 0


def test_gpu_flat_counts_a_nonfinite_env_once():
    """An env whose tiles straddle several workgroups is still counted once when its reward
    turns non-finite (only the owner writes the env's outputs), and its NaN stays in it."""
    from pmenv import TradingEnv, synth
    B, N, W = 37, 30, 50                                    # 1,875 chunks per env: 2-3 tiles each
    ser = synth.series(W + 2, B, N, seed=3, device=DEV)
    obs = synth.window_from_series(ser, W)
    env = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="flat")
    env.reset(obs)
    a = torch.full((B, N), 1.0 / N, device=DEV)
    a[5, 7] = float("nan")
    r, _ = env.step(a, obs, bar=ser[W])
    assert env.nonfinite_count() == 1
    assert torch.isnan(r[5]) and torch.isfinite(r[torch.arange(B, device=DEV) != 5]).all()
    assert torch.isfinite(obs[torch.arange(B, device=DEV) != 5]).all()


def test_gpu_flat_two_handles_on_two_streams():
    """One handle per stream: two envs stepped on two HIP streams with their launches
    interleaved (each handle's snapshot / halo parities are its own) give the bits of
    each env stepped alone."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 4096, 30, 50, 12
    ser = [synth.series(W + T, B, N, env_offset=k * B, seed=5, device=DEV) for k in range(2)]
    act = [synth.actions(T, B, N, env_offset=k * B, seed=6, device=DEV) for k in range(2)]

    def run(streams):
        envs, obs, rews = [], [], []
        for k in range(2):
            with torch.cuda.stream(streams[k]):
                e = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="flat")
                o = synth.window_from_series(ser[k], W)
                e.reset(o)
                envs.append(e)
                obs.append(o)
                rews.append([])
        for t in range(T):
            for k in range(2):
                with torch.cuda.stream(streams[k]):
                    r, _ = envs[k].step(act[k][t], obs[k], bar=ser[k][W + t])
                    rews[k].append(r.clone())
        torch.cuda.synchronize()
        return [(obs[k], torch.stack(rews[k]), envs[k].value.clone()) for k in range(2)]

    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    both = run([s1, s2])
    alone = run([s1, s1])
    for k in range(2):
        for x, y in zip(both[k], alone[k]):
            assert torch.equal(x, y), k
