"""On-device synthetic market data — replaces the reference's
network data path (data/load_yf.py, data/instrument.py:79, :339-356) for benchmarks.

Counter-based Philox4x32-10 keyed by (seed, global env id, asset, day), so a
sharded run generates exactly its slice of the unsharded data.
"""
import ctypes

import torch

from . import _abi

MARKET_CHANNELS = 4  # open, high, low, close


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def series(T, B, N, env_offset=0, seed=42, sigma=0.015, device=None):
    """OHLC random walk, [T, B, N, 4] float32 (time-major: one day's bars contiguous)."""
    lib = _abi.load()
    device = torch.device(device or "cuda")
    out = torch.empty(T, B, N, MARKET_CHANNELS, dtype=torch.float32, device=device)
    _abi.check(lib.pmenv_synth_series(ctypes.c_void_p(out.data_ptr()), T, B, N, env_offset, seed, sigma,
                                      _stream(out.device)), None, "pmenv_synth_series")
    return out


def actions(T, B, N, env_offset=0, seed=43, device=None):
    """Softmax-of-N(0,1) simplex actions, [T, B, N] float32."""
    lib = _abi.load()
    device = torch.device(device or "cuda")
    out = torch.empty(T, B, N, dtype=torch.float32, device=device)
    _abi.check(lib.pmenv_synth_actions(ctypes.c_void_p(out.data_ptr()), T, B, N, env_offset, seed,
                                       _stream(out.device)), None, "pmenv_synth_actions")
    return out


def window_from_series(series_t, W, F=5):
    """Initial obs [B, N, W, F] from the first W days of a [T, B, N, 4] series."""
    lib = _abi.load()
    T, B, N, C = series_t.shape
    if C != MARKET_CHANNELS or F != 5 or T < W:
        raise ValueError("window_from_series needs a [T>=W, B, N, 4] series and F == 5")
    obs = torch.empty(B, N, W, F, dtype=torch.float32, device=series_t.device)
    _abi.check(lib.pmenv_window_init(ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(series_t.data_ptr()),
                                     B, N, W, F, _stream(obs.device)), None, "pmenv_window_init")
    return obs
