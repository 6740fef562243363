"""A/B two builds of libpmenv.so in ONE process, interleaved rounds (cdna_hip_programming.md
§5.4 rule 24): the same inputs, each library's own handle, the step timed per round with
HIP events on the current stream. Bitwise equality of rewards / values / windows between
the builds is checked on the first rounds' outputs (the builds must give the same bits).

    python tools/ab_libs.py --libs tools/libpmenv_base.so,pm-rl_amd/pmenv/libpmenv.so \
        --envs 8192 --assets 30 --path auto --commission 0 --reward log_returns
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--libs", required=True)
ap.add_argument("--envs", type=int, default=8192)
ap.add_argument("--assets", type=int, default=30)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--features", type=int, default=5, help="F (the bar has F - 1 channels, close at 3)")
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--H", type=int, default=48, help="distinct days of bars / actions (cycled)")
ap.add_argument("--path", default="auto", help="auto | one_launch | two_launch | flat | walk (comma list: per lib)")
ap.add_argument("--commission", type=float, default=0.0)
ap.add_argument("--reward", default="log_returns")
ap.add_argument("--out", action="store_true", help="double-buffered (obs -> obs_out)")
ap.add_argument("--attribute", action="store_true",
                help="synchronise after every step of the bits phase and name the build on stderr "
                     "first (a fault is then reported against the build and step that raised it)")
a = ap.parse_args()

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
B, N, W, F = a.envs, a.assets, a.window, a.features
# "lib.so+KNOB=VAL+...": tools-build knobs set while that variant's handle is created
specs = [x.split("+") for x in a.libs.split(",")]
libs = [sp[0] if os.path.isabs(sp[0]) else os.path.join(ROOT, sp[0]) for sp in specs]
knobs = [dict(kv.split("=", 1) for kv in sp[1:]) for sp in specs]
paths = a.path.split(",")
if len(paths) == 1:
    paths = paths * len(libs)
STEP_PATHS = _abi.STEP_PATHS

g = torch.Generator(device=dev).manual_seed(7)
# a positive OHLC random walk (the values only need to be plausible prices)
close = torch.exp(torch.cumsum(torch.randn(a.H + W, B, N, 1, generator=g, device=dev) * 0.015, 0))
ser = torch.cat([close * 1.001, close * 1.01, close * 0.99, close] +
                [close * (1.0 + 0.001 * c) for c in range(F - 5)], dim=3)[..., :F - 1].contiguous()
del close
act = torch.softmax(torch.randn(a.H, B, N, generator=g, device=dev), dim=-1)
obs0 = torch.empty(B, N, W, F, device=dev)
obs0[..., :F - 1] = ser[:W].permute(1, 2, 0, 3)
obs0[..., F - 1] = 0.0


def bind(path):
    lib = ctypes.CDLL(path)
    for name, res, args in _abi.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


class Env:
    def __init__(self, lib, path):
        self.lib = lib
        cfg = _abi.PmenvCfg()
        lib.pmenv_cfg_default(ctypes.byref(cfg), B, N, W, F)
        cfg.commission = a.commission
        cfg.reward_kind = _abi.REWARD_KINDS[a.reward]
        h = ctypes.c_void_p()
        _abi.check(lib.pmenv_create(ctypes.byref(cfg), 0, ctypes.byref(h)), None, "create")
        self.h = h
        rc = lib.pmenv_set_step_path(h, STEP_PATHS[path])
        if rc:
            raise SystemExit(f"{path}: {lib.pmenv_last_error(h).decode()}")
        self.obs = obs0.clone()
        self.obs2 = torch.empty_like(self.obs) if a.out else None
        self.rew = torch.empty(B, device=dev)
        self.t = 0
        self.reset()

    def reset(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        self.obs.copy_(obs0)
        _abi.check(self.lib.pmenv_reset(self.h, ctypes.c_void_p(self.obs.data_ptr()), None, s), self.h, "reset")
        self.t = 0

    def step(self):
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        d = self.t % a.H
        args = _abi.PmenvStepArgs()
        args.action = act[d].data_ptr()
        args.bar = ser[W + d].data_ptr()
        args.obs = self.obs.data_ptr()
        args.obs_out = self.obs2.data_ptr() if a.out else None
        args.reward = self.rew.data_ptr()
        _abi.check(self.lib.pmenv_step_ex(self.h, ctypes.byref(args), s), self.h, "step")
        if a.out:
            self.obs, self.obs2 = self.obs2, self.obs
        self.t += 1


envs = []
for p, path, kn in zip(libs, paths, knobs):
    os.environ.update(kn)
    envs.append(Env(bind(p), path))
    for k in kn:
        os.environ.pop(k, None)
names = [f"{os.path.basename(p)}{''.join('+' + k + '=' + v for k, v in kn.items())}:{path}"
         for p, path, kn in zip(libs, paths, knobs)]
kernels = [e.lib.pmenv_step_path(e.h).decode() for e in envs]

# bits: the first 2 * W steps (past the ring wrap) from one reset, every build
ref = None
same = []
for name, e in zip(names, envs):
    if a.attribute:
        print(f"# bits: {name} [{e.lib.pmenv_step_path(e.h).decode()}]", file=sys.stderr, flush=True)
    e.reset()
    rs = []
    for i in range(2 * W + 3):
        e.step()
        rs.append(e.rew.clone())
        if a.attribute:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    got = (torch.stack(rs), e.obs.clone())
    if ref is None:
        ref = got
        same.append(True)
    else:
        same.append(bool(torch.equal(got[0].nan_to_num(7.0), ref[0].nan_to_num(7.0)) and
                         torch.equal(got[1].nan_to_num(7.0), ref[1].nan_to_num(7.0))))

times = {n: [] for n in names}
for r in range(a.rounds):
    order = list(range(len(envs))) if r % 2 == 0 else list(reversed(range(len(envs))))
    for i in order:
        e = envs[i]
        for _ in range(5):
            e.step()
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s0.record()
        for _ in range(a.steps):
            e.step()
        s1.record()
        s1.synchronize()
        times[names[i]].append(s0.elapsed_time(s1) * 1000.0 / a.steps)
res = {"B": B, "N": N, "W": W, "commission": a.commission, "reward": a.reward, "out": a.out,
       "variants": {n: {"median_us": statistics.median(times[n]), "min_us": min(times[n]), "rounds": times[n],
                        "kernel": k, "bits_equal_first": s}
                    for n, k, s in zip(names, kernels, same)}}
print(json.dumps(res))
for n in names:
    v = res["variants"][n]
    print(f"# {B}x{N} c={a.commission} {a.reward} out={a.out} {n:45s} {v['median_us']:9.2f} us "
          f"(min {v['min_us']:.2f}) bits_equal={v['bits_equal_first']} [{v['kernel']}]", file=sys.stderr)
