"""step_relay_kernel's forward progress without dispatch order (step_relay.h head): a tile
that still misses a relay word after its polls defers — appends itself to the step's
deferral list, re-checks once, exits — and a deferred tile runs exactly once, by itself or
by a scalar block, with the tile's own code.

The product's order never exercises that path, so the tools build forces it
(tools/libpmenv_ab.so, step_relay_kernel<..., ANY = 1>): PMENV_RELAY_SPIN=0 (every tile
defers on its first missing word) and PMENV_RELAY_TILES_FIRST=1 (blockIdx rotated so every
tile is dispatched before every scalar block: most tiles are run by scalar blocks). Each
forced handle must give the product handle's bits — rewards, windows, values — step for step
past the ring wrap. Needs an MI355X."""
import ctypes
import os

import pytest
import torch

from test_gpu_parity import DEV, _gpu  # noqa: F401  (_gpu: autouse fixture)

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS_LIB = os.path.join(ROOT, "tools", "libpmenv_ab.so")
RELAY = 4


def _load(path):
    from pmenv import _abi
    lib = ctypes.CDLL(path)
    for name, res, args in _abi.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


class _Env:
    def __init__(self, lib, B, N, W, knobs):
        from pmenv import _abi
        self.lib = lib
        c = _abi.PmenvCfg()
        lib.pmenv_cfg_default(ctypes.byref(c), B, N, W, 5)
        h = ctypes.c_void_p()
        old = {k: os.environ.get(k) for k in knobs}
        os.environ.update(knobs)                 # the tools build reads its knobs at create
        try:
            rc = lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(h))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        assert rc == 0, lib.pmenv_last_error(None)
        self.h = h
        assert lib.pmenv_set_step_path(h, RELAY) == 0, lib.pmenv_last_error(h)

    def path(self):
        return self.lib.pmenv_step_path(self.h).decode()

    def close(self):
        torch.cuda.synchronize()
        self.lib.pmenv_destroy(self.h)


@pytest.mark.parametrize("B,N,W", [(512, 30, 50), (301, 8, 30), (97, 64, 20)])
def test_gpu_relay_forced_deferral_gives_the_product_bits(B, N, W):
    from pmenv import _abi, synth
    if not os.path.exists(TOOLS_LIB):
        pytest.fail(f"{TOOLS_LIB} missing: build it with `python pm-rl_amd/build.py`")
    prod = _abi.load()
    tools = _load(TOOLS_LIB)
    variants = [({}, prod), ({"PMENV_RELAY_SPIN": "0"}, tools), ({"PMENV_RELAY_TILES_FIRST": "1"}, tools),
                ({"PMENV_RELAY_SPIN": "0", "PMENV_RELAY_TILES_FIRST": "1"}, tools)]
    T = W + 12
    ser = synth.series(W + T, B, N, seed=B * 7 + N, device=DEV)
    act = synth.actions(T, B, N, seed=B + W, device=DEV)
    stream = ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)
    envs, obs, rew = [], [], []
    for knobs, lib in variants:
        e = _Env(lib, B, N, W, knobs)
        assert e.path() == "step_relay_kernel (obs_out) | step_relay_kernel (in place)", e.path()
        o = synth.window_from_series(ser, W)
        assert lib.pmenv_reset(e.h, ctypes.c_void_p(o.data_ptr()), None, stream) == 0
        envs.append(e)
        obs.append(o)
        rew.append(torch.empty(T, B, device=DEV))
    try:
        for t in range(T):
            for i, e in enumerate(envs):
                a = _abi.PmenvStepArgs()
                a.action, a.bar, a.obs = act[t].data_ptr(), ser[W + t].data_ptr(), obs[i].data_ptr()
                a.reward = rew[i][t].data_ptr()
                assert e.lib.pmenv_step_ex(e.h, ctypes.byref(a), stream) == 0, e.lib.pmenv_last_error(e.h)
            torch.cuda.synchronize()
            for i in range(1, len(envs)):
                assert torch.equal(obs[i].view(torch.int32), obs[0].view(torch.int32)), \
                    f"step {t}: window differs under {variants[i][0]}"
        for i in range(1, len(envs)):
            assert torch.equal(rew[i].view(torch.int32), rew[0].view(torch.int32)), f"rewards differ under {variants[i][0]}"
    finally:
        for e in envs:
            e.close()
