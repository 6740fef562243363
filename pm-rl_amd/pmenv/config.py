"""Env configuration — the reference's module constants as an explicit struct.

The reference binds these at import time from config/base.py (WINDOW_SIZE :28,
NUM_ASSETS :29, INITIAL_CASH :47, COMISSION :48, REWARD :51, REWARD_SCALE :52,
RISK_FREE_RATE :53, SEED :3); here they are per-env-object fields passed to
pmenv_create (include/pmenv.h pmenv_cfg).
"""
from dataclasses import dataclass, field, asdict

from . import _abi

# config/base.py defaults
SEED = 42
WINDOW_SIZE = 32
NUM_ASSETS = 32
INITIAL_CASH = 25000
COMISSION = 0.0
REWARD = "log_returns"
REWARD_SCALE = 1
RISK_FREE_RATE = 0.04


@dataclass
class EnvConfig:
    num_envs: int = 1
    num_assets: int = NUM_ASSETS
    window: int = WINDOW_SIZE
    features: int = 5                 # [open, high, low, close, weight]
    close_channel: int = 3
    reward: str = REWARD              # log_returns | returns | sharpe_ratio | diff_sharpe
    norm: str = "and"                 # and (trading_env.py:58) | or (pg.py:52)
    ring: str = "storage"             # storage (weight_buffer.py:38-39) | chrono
    ret: str = "gross"                # gross: trading_env.py:88 for every reward kind (info["returns"] as
                                      # the reference records it) | net: reward.py:20-31 over info["values"]
                                      # (commission included) | auto: gross for log_returns, net otherwise
    init_cash: float = float(INITIAL_CASH)
    commission: float = COMISSION
    reward_scale: float = float(REWARD_SCALE)
    risk_free_rate: float = RISK_FREE_RATE
    sharpe_eta: float = 0.01
    mu_tol: float = 1e-10
    mu_max_iter: int = 100
    extra: dict = field(default_factory=dict)

    def validate(self):
        if self.reward not in _abi.REWARD_KINDS:
            raise ValueError(f"unknown reward {self.reward!r}; one of {sorted(_abi.REWARD_KINDS)}")
        if self.norm not in _abi.NORM_MODES:
            raise ValueError(f"unknown norm mode {self.norm!r}")
        if self.ring not in _abi.RING_MODES:
            raise ValueError(f"unknown ring mode {self.ring!r}")
        if self.ret not in _abi.RET_MODES:
            raise ValueError(f"unknown ret mode {self.ret!r}")
        for k in ("num_envs", "num_assets", "window"):
            if int(getattr(self, k)) < 1:
                raise ValueError(f"{k} must be >= 1")
        if self.features < 2:
            raise ValueError("features must be >= 2 (market channels + the weight channel)")
        if not 0 <= self.close_channel < self.features - 1:
            raise ValueError("close_channel must index a market channel (0 .. F-2)")
        if not 0.0 <= self.commission < 1.0:
            raise ValueError("commission must be in [0, 1)")
        return self

    def to_c(self):
        self.validate()
        c = _abi.PmenvCfg()
        c.num_envs, c.num_assets, c.window, c.features = (int(self.num_envs), int(self.num_assets),
                                                           int(self.window), int(self.features))
        c.close_channel = int(self.close_channel)
        c.reward_kind = _abi.REWARD_KINDS[self.reward]
        c.norm_mode = _abi.NORM_MODES[self.norm]
        c.ring_mode = _abi.RING_MODES[self.ring]
        c.ret_mode = _abi.RET_MODES[self.ret]
        c.mu_max_iter = int(self.mu_max_iter)
        c.init_cash = float(self.init_cash)
        c.commission = float(self.commission)
        c.reward_scale = float(self.reward_scale)
        c.risk_free_rate = float(self.risk_free_rate)
        c.sharpe_eta = float(self.sharpe_eta)
        c.mu_tol = float(self.mu_tol)
        return c

    def as_dict(self):
        return asdict(self)
