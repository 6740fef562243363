"""pmenv — MI355X-native vectorised portfolio environment (hot path of zachramsey/pm-rl).

The compute path is libpmenv.so (HIP kernels for gfx950 behind include/pmenv.h);
this package is the host-side mirror of the reference's Python interface
(env/sim/trading_env.py TradingEnv) plus the data/rollout helpers around it.
"""
from .config import EnvConfig  # noqa: F401
from .trading_env import TradingEnv, RingView  # noqa: F401
from . import synth, rollout, parallel, trainer, data, replay, rollout_buffer, on_policy, off_policy  # noqa: F401
from .data import MarketSeries  # noqa: F401
from .rollout_buffer import DeviceRolloutBuffer  # noqa: F401

__all__ = ["EnvConfig", "TradingEnv", "RingView", "synth", "rollout", "parallel", "trainer", "data", "MarketSeries", "replay",
           "DeviceRolloutBuffer", "rollout_buffer", "on_policy", "off_policy"]
