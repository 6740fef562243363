"""HBM-resident market data path.

The reference builds every day's window on the host (`data/instrument.py:339-356`
materialises all T-W+1 windows, W× the series) and feeds one per step through a
`DataLoader(batch_size=1)` (`data/instrument_pool.py:464-477`), with price relatives
precomputed as close_t / close_{t-1} (`instrument.py:79`). Here the series lives in
HBM once, [T, N, F-1] shared by all envs; each env trades it from its own start day,
the initial windows are gathered on device, and each step reads the day's bar
straight from the series inside the fused step (no per-step copy, no host traffic).
"""
import ctypes

import numpy as np
import torch

from . import _abi


class MarketSeries:
    def __init__(self, bars, device=None):
        """bars: [T, N, F-1] market channels (e.g. [open, high, low, close]) as numpy or torch."""
        t = torch.as_tensor(np.asarray(bars) if not torch.is_tensor(bars) else bars)
        if t.dim() != 3:
            raise ValueError("bars must be [T, N, F-1]")
        self.bars = t.to(device=device or "cuda", dtype=torch.float32).contiguous()
        self.days, self.num_assets, self.channels = self.bars.shape
        self.device = self.bars.device

    def initial_window(self, start, window):
        """obs [B, N, W, F] with obs[b, :, t, :F-1] = bars[start[b] + t]; channel F-1 = 0 (reset fills it)."""
        lib = _abi.load()
        start = torch.as_tensor(start, device=self.device).to(torch.int32).contiguous()
        B = start.numel()
        F = self.channels + 1
        obs = torch.empty(B, self.num_assets, window, F, dtype=torch.float32, device=self.device)
        s = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        _abi.check(lib.pmenv_window_init_days(ctypes.c_void_p(obs.data_ptr()), ctypes.c_void_p(self.bars.data_ptr()),
                                              self.days, self.num_assets, F, ctypes.c_void_p(start.data_ptr()), B,
                                              window, s), None, "pmenv_window_init_days")
        return obs

    def random_starts(self, num_envs, window, horizon, generator=None):
        """Uniform start days leaving room for `window` + `horizon` days."""
        hi = self.days - window - horizon + 1
        if hi < 1:
            raise ValueError("series too short for window + horizon")
        return torch.randint(0, hi, (num_envs,), generator=generator, device="cpu").to(self.device, torch.int32)
