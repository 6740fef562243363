"""step_relay_kernel: the two-launch path's scalar step and window stream in ONE launch,
the scalar workgroups relaying w' and the counter to the stream tiles through epoch-tagged
words (step_relay.h).

Checked against the CPU oracle in every mode, bit for bit against the two-launch path
(whose scalar step it runs) across resets, masked resets, checkpoint restores, path
switches, fresh window buffers, double-buffered steps, resident-series days and caller
prices, at every scalar-step form (N <= 16 packed, register form, 64 < N <= 512 packed
strided), and at the cache-resident and BASELINE shapes. Needs an MI355X."""
import zlib

import numpy as np
import pytest
import torch

from test_gpu_parity import DEV, MODES, _gpu, _run_both  # noqa: F401  (_gpu: autouse fixture)
from test_gpu_flat_step import _same, _state

pytestmark = pytest.mark.gpu

# (N, W, B): every scalar-step form (N <= 8 / <= 16 packed, 32 / 64 lanes, 64 < N <= 512
# packed strided), W = 2 (every day a last day), envs of a few chunks to many tiles
SHAPES = [(30, 50, 37), (5, 48, 211), (8, 12, 301), (16, 20, 97), (33, 20, 23), (64, 47, 9), (100, 20, 13),
          (130, 14, 7), (300, 10, 5), (500, 50, 3), (30, 2, 400), (1, 600, 9)]   # N W F 16-B granular


def _mode_id(k):
    return "-".join(f"{a}={b}" for a, b in k.items()) or "reference"


@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
@pytest.mark.parametrize("kw", MODES, ids=_mode_id)
def test_gpu_relay_vs_oracle_modes(db, kw):
    """Every reward / ring / norm / commission mode, past the ring wrap, against the oracle."""
    _run_both(kw, B=37, N=30, W=50, T=56, kind="mixed", seed=zlib.crc32(f"relay{kw}{db}".encode()),
              double_buffer=db, impl="relay")


@pytest.mark.parametrize("N,W,B", SHAPES)
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_relay_shapes_vs_oracle(N, W, B, db):
    _run_both({}, B=B, N=N, W=W, T=W + 5, kind="mixed", seed=N * 17 + W, double_buffer=db, impl="relay")


@pytest.mark.parametrize("N,W,B", [(30, 50, 37), (8, 30, 301), (64, 47, 3), (200, 20, 5)])
@pytest.mark.parametrize("kw", [dict(), dict(commission=0.0025, reward="sharpe_ratio"),
                                dict(ring="chrono", reward="diff_sharpe")], ids=_mode_id)
def test_gpu_relay_bitwise_vs_two_launch_through_state_changes(N, W, B, kw):
    """The relayed step and the two-launch path, driven with the same inputs through
    everything that invalidates the relay halo — full and masked resets, a checkpoint
    restore, a switch to another path and back, a fresh window buffer, double-buffered
    steps, caller prices, resident-series days — agree on every window, reward, returned
    weight and state field, bit for bit."""
    from pmenv import TradingEnv, synth
    T = W + 24
    ser = synth.series(W + T, B, N, seed=zlib.crc32(f"relay{N}{W}{kw}".encode()), device=DEV)
    act = synth.actions(T, B, N, seed=5, device=DEV)
    kind_mixed = torch.randn(T, B, N, device=DEV, generator=torch.Generator(DEV).manual_seed(3))
    res = synth.series(T + W + 8, 1, N, seed=9, device=DEV)[:, 0].contiguous()
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i, track_info=True, **kw)
            for i in ("relay", "two_launch")]
    assert envs[0].step_path == "step_relay_kernel (obs_out) | step_relay_kernel (in place)"
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
                e.set_step_impl("relay")
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
                day[1::7] = 10 ** 6                       # outside the series: NaN bar, as every path
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


def test_gpu_relay_caller_edits_between_steps():
    """The in-place halo is the previous step's output: caller edits of the window (seen by
    the version counter, or announced with window_written) and of the state re-prime it."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 2048, 30, 50, 10
    ser = synth.series(W + T, B, N, seed=21, device=DEV)
    act = synth.actions(T, B, N, seed=22, device=DEV)
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i) for i in ("relay", "two_launch")]
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    for t in range(T):
        for i, e in enumerate(envs):
            if t in (2, 6):
                obs[i][..., :4].mul_(1.0009765625)          # every tile seam
            if t == 4:
                obs[i].data[..., 3].mul_(0.998046875)       # invisible to the version counter...
                e.window_written(obs[i])                    # ...announced
            if t == 7:
                e.value.mul_(0.75)
        rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
        assert torch.equal(obs[0], obs[1]), f"step {t}: windows"
        assert torch.equal(envs[0].value, envs[1].value), f"step {t}: values"


def _capture(fn):
    """fn() captured into a CUDA/HIP graph on a side stream."""
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream(DEV))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        out = fn()
    torch.cuda.current_stream(DEV).wait_stream(s)
    return g, out


@pytest.mark.parametrize("B,W", [(512, 20), (8192, 50)], ids=["256x2", "256x4"])
@pytest.mark.parametrize("db", [False, True], ids=["inplace", "obs_out"])
def test_gpu_relay_graph_capture_replays_the_relay_step(db, B, W):
    """A captured RELAY step stays step_relay_kernel: its epoch and parity come from the
    launch counter on the device (the ordered ticket), and the validity of its counter copy
    and halo from device words the captured invalidations clear. Eager relay steps, replays
    of a one-step graph and replays of a [reset, step, step] graph interleave, each bitwise
    equal to an eager two-launch env driven with the same inputs. 8,192 x 30 x 50 is the
    window AUTO gives 256 x 4 tiles (in place)."""
    from pmenv import TradingEnv, synth
    N, T = 30, 16
    ser = synth.series(W + T + 8, B, N, seed=31, device=DEV)
    act = synth.actions(T + 8, B, N, seed=32, device=DEV)
    er = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="relay")
    et = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="two_launch")
    o_r, o_t = synth.window_from_series(ser, W), synth.window_from_series(ser, W)
    nx_r, nx_t = torch.empty_like(o_r), torch.empty_like(o_t)
    er.reset(o_r)
    et.reset(o_t)

    def step(e, a, o, bar, nx):
        if db:
            r, _ = e.step(a, o, bar=bar, out=nx)
            o.copy_(nx)
            return r
        return e.step(a, o, bar=bar)[0]

    a_buf, b_buf = act[0].clone(), ser[W].clone()
    for t in range(3):                                   # eager relay steps
        step(er, act[t], o_r, ser[W + t], nx_r)
        step(et, act[t], o_t, ser[W + t], nx_t)
    g1, r_cap = _capture(lambda: step(er, a_buf, o_r, b_buf, nx_r))
    assert "step_relay_kernel" in er.step_path and "relay steps device-sequenced" in er.step_path, er.step_path
    w_buf = synth.window_from_series(ser, W)             # graph 2's reset window

    def reset_and_two():
        er.reset(o_r)
        step(er, a_buf, o_r, b_buf, nx_r)
        return step(er, a_buf, o_r, b_buf, nx_r)
    g2, r2_cap = _capture(reset_and_two)
    # the capture ran nothing: re-sync the relay env to the two-launch env's state and window
    er.load_state_dict(et.state_dict())
    o_r.copy_(o_t)
    for t in range(3, T):
        a_buf.copy_(act[t])
        b_buf.copy_(ser[W + t])
        if t % 4 == 0:                                   # graph 2: reset, then two steps (same inputs)
            o_r.copy_(w_buf)
            o_t.copy_(w_buf)
            g2.replay()
            et.reset(o_t)
            step(et, act[t], o_t, ser[W + t], nx_t)
            rt = step(et, act[t], o_t, ser[W + t], nx_t)
            rr = r2_cap
        elif t % 4 == 1:                                 # eager relay step
            rr = step(er, act[t], o_r, ser[W + t], nx_r)
            rt = step(et, act[t], o_t, ser[W + t], nx_t)
        else:                                            # graph 1: one relay step
            g1.replay()
            rr = r_cap
            rt = step(et, act[t], o_t, ser[W + t], nx_t)
        torch.cuda.synchronize(DEV)
        assert torch.equal(rr, rt), f"t {t}: rewards"
        assert torch.equal(o_r, o_t), f"t {t}: windows"
        assert torch.equal(er.value, et.value), f"t {t}: values"


def test_gpu_relay_after_replays_of_another_path():
    """A handle captured while another path was current, its graph replayed (state and window
    written where the host does not see it), then switched to RELAY: the relay step re-primes
    its copies from the device words the replays cleared (no stale host flag), bitwise equal
    to a two-launch env throughout."""
    from pmenv import TradingEnv, synth
    B, N, W, T = 1024, 30, 20, 14
    ser = synth.series(W + T, B, N, seed=41, device=DEV)
    act = synth.actions(T, B, N, seed=42, device=DEV)
    er = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="relay")
    et = TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl="two_launch")
    o_r, o_t = synth.window_from_series(ser, W), synth.window_from_series(ser, W)
    er.reset(o_r)
    et.reset(o_t)
    for t in range(2):                                   # eager relay steps: the host flags hold
        er.step(act[t], o_r, bar=ser[W + t])
        et.step(act[t], o_t, bar=ser[W + t])
    er.set_step_impl("two_launch")
    a_buf, b_buf = act[0].clone(), ser[W].clone()
    snap = er.state_dict(), o_r.clone()
    g, r_cap = _capture(lambda: er.step(a_buf, o_r, bar=b_buf)[0])
    er.load_state_dict(snap[0])
    o_r.copy_(snap[1])
    er.set_step_impl("relay")
    for t in range(2, T):
        a_buf.copy_(act[t])
        b_buf.copy_(ser[W + t])
        if t in (5, 6, 9):                               # replays of the captured two-launch step
            g.replay()
            rr = r_cap
        else:
            rr = er.step(act[t], o_r, bar=ser[W + t])[0]
        rt = et.step(act[t], o_t, bar=ser[W + t])[0]
        torch.cuda.synchronize(DEV)
        assert torch.equal(rr, rt), f"t {t}: rewards"
        assert torch.equal(o_r, o_t), f"t {t}: windows"


@pytest.mark.parametrize("B,N", [(8192, 30), (4096, 30), (65536, 30), (8192, 500)])
def test_gpu_relay_full_size_bitwise(B, N):
    """The BASELINE shapes (config 2, config 4's 8-GPU share, the whole config 4, config 5)
    in place, relay against two launches, bit for bit, past the ring wrap."""
    from pmenv import TradingEnv, synth
    W, T = 50, 54 if N == 30 else 6
    ser = synth.series(W + T, B, N, seed=B + N, device=DEV)
    act = synth.actions(T, B, N, seed=N, device=DEV)
    kw = dict(reward="diff_sharpe") if N == 500 else {}
    envs = [TradingEnv(num_envs=B, num_assets=N, window=W, device=DEV, step_impl=i, **kw)
            for i in ("relay", "two_launch")]
    obs = [synth.window_from_series(ser, W) for _ in envs]
    for e, o in zip(envs, obs):
        e.reset(o)
    for t in range(T):
        rs = [e.step(act[t], o, bar=ser[W + t])[0] for e, o in zip(envs, obs)]
        assert torch.equal(rs[0], rs[1]), f"step {t}: rewards"
    assert torch.equal(obs[0], obs[1])
    _same(_state(envs[0]), _state(envs[1]), "end")
    del envs, obs
    torch.cuda.empty_cache()
