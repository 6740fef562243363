"""A/B of the F != 5 step: the two-launch generic stream (scalar step + advance_gen_kernel,
the product's AUTO above 2 MiB, or forced with PMENV_STEP_PATH_TWO_LAUNCH) against the
register step (step_small_kernel: the tools build with PMENV_GEN_OFF=1 keeps AUTO there),
in ONE process, interleaved, per shape: us per step (HIP events over K steps, median of R),
env-steps/s and the fraction of the 8 TB/s spec for the step's algorithmic bytes
(tools/bench_shapes.py's count), and whether the two give the same windows and rewards.
With PMENV_GEN_PERELEM=1 the other leg is advance_gen_kernel's per-element compose (tools);
with AB_GEN_BASE=<path> another product build (e.g. an earlier commit's), forced alike.

    PMENV_GEN_OFF=1 python tools/ab_gen.py      # prints one JSON object
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import ab_r05 as ab  # noqa: E402
from pmenv import _abi  # noqa: E402

K = int(os.environ.get("AB_K", "50"))
R = int(os.environ.get("AB_R", "5"))
PEAK = 8.0e12
# (B, N, W, F, in place)
SHAPES = [(65536, 30, 50, 8, True), (65536, 30, 50, 8, False), (16384, 30, 50, 8, True), (4096, 30, 50, 8, True),
          (2048, 30, 50, 8, True), (1024, 30, 50, 8, True), (512, 30, 50, 8, True), (256, 30, 50, 8, True),
          (65536, 30, 50, 3, True), (16384, 30, 50, 3, True), (4096, 30, 50, 3, True), (1024, 30, 50, 3, True),
          (65536, 30, 50, 4, True), (16384, 64, 50, 6, True)]
if os.environ.get("AB_GEN_SHAPES") == "wide":     # windows past the register step's 16,384 floats
    SHAPES = [(16384, 64, 50, 6, True), (8192, 100, 50, 8, True), (4096, 64, 50, 8, True), (16384, 64, 50, 6, False),
              (2048, 128, 50, 4, True)]
elif os.environ.get("AB_GEN_SHAPES") == "few":    # around AUTO's threshold against the register step
    SHAPES = [(64, 30, 50, 8, True), (128, 30, 50, 8, True), (256, 30, 50, 8, True), (128, 30, 50, 3, True),
              (256, 30, 50, 3, True), (512, 30, 50, 3, True), (256, 30, 50, 4, True), (256, 30, 50, 6, True),
              (256, 30, 50, 8, False), (512, 30, 50, 3, False), (32, 64, 50, 8, True), (128, 16, 32, 8, True),
              (64, 30, 50, 3, True), (96, 30, 50, 4, True), (64, 16, 32, 8, True),
              # windows of <= 2,048 floats (step_tiny_kernel's)
              (1024, 5, 50, 8, True), (4096, 5, 50, 8, True), (16384, 5, 50, 8, True), (4096, 8, 32, 6, True),
              (16384, 8, 32, 6, False), (4096, 10, 50, 4, True), (65536, 5, 50, 8, True),
              # past the register step's 16,384 floats (the LDS fallback's)
              (64, 100, 50, 8, True), (64, 100, 50, 8, False), (128, 64, 50, 6, True), (128, 64, 50, 6, False),
              (256, 128, 50, 4, True), (8192, 100, 50, 8, False), (2048, 128, 50, 4, False)]
elif os.environ.get("AB_GEN_SHAPES") == "big":    # in place past 128 MiB (the nt tiles; PMENV_GEN_ABL legs)
    SHAPES = [(65536, 30, 50, 3, True), (65536, 30, 50, 4, True), (65536, 30, 50, 8, True)]


def step_bytes(N, W, F):
    return 4 * (N * (W - 1) * F + N * (F - 1) + N + N * W * F) + 20


class Env:
    def __init__(self, lib, B, N, W, F, ip, force_two):
        self.lib = lib
        c = _abi.PmenvCfg()
        lib.pmenv_cfg_default(ctypes.byref(c), B, N, W, F)
        c.close_channel = F - 2
        h = ctypes.c_void_p()
        assert lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(h)) == 0, lib.pmenv_last_error(None)
        self.h = h
        if force_two:
            assert lib.pmenv_set_step_path(h, 2) == 0, lib.pmenv_last_error(h)
        g = torch.Generator(ab.DEV).manual_seed(B + N + W + F)
        H = 8
        self.obs = [torch.rand(B, N, W, F, device=ab.DEV, generator=g) + 0.5, torch.empty(B, N, W, F, device=ab.DEV)]
        self.bars = torch.rand(H, B, N, F - 1, device=ab.DEV, generator=g) + 0.5
        self.acts = torch.softmax(torch.randn(H, B, N, device=ab.DEV, generator=g), -1)
        self.rew = torch.empty(B, device=ab.DEV)
        assert lib.pmenv_reset(h, ctypes.c_void_p(self.obs[0].data_ptr()), None, ab.stream()) == 0
        self.args = []
        for t in range(H):
            a = _abi.PmenvStepArgs()
            a.action, a.bar, a.reward = self.acts[t].data_ptr(), self.bars[t].data_ptr(), self.rew.data_ptr()
            a.obs = self.obs[0 if ip else t % 2].data_ptr()
            a.obs_out = None if ip else self.obs[(t + 1) % 2].data_ptr()
            self.args.append(a)
        self.t, self.H, self.ip = 0, H, ip

    def step(self):
        rc = self.lib.pmenv_step_ex(self.h, ctypes.byref(self.args[self.t % self.H]), ab.stream())
        assert rc == 0, self.lib.pmenv_last_error(self.h)
        self.t += 1

    def window(self):
        return self.obs[0] if self.ip else self.obs[self.t % 2]

    def close(self):
        torch.cuda.synchronize()
        self.lib.pmenv_destroy(self.h)


def main():
    base = os.environ.get("AB_GEN_BASE")            # another product build, forced to two launches too
    perelem = (base is not None or os.environ.get("PMENV_GEN_PERELEM") == "1" or os.environ.get("PMENV_GEN_POL0") == "1"
               or os.environ.get("AB_GEN_FORCE") == "1" or os.environ.get("PMENV_GEN_ABL") is not None)     # the tools leg forced to two launches (e.g. PMENV_GEN_GEOM)
    assert perelem or os.environ.get("PMENV_GEN_OFF") == "1", \
        "run with PMENV_GEN_OFF=1 (against the register step) or PMENV_GEN_PERELEM=1 (against the per-element compose)"
    torch.cuda.set_device(ab.DEV)
    libs = {"gen": ab.load(ab.LIBS["r05"]),
            "small": ab.load(os.path.join(ROOT, base) if base else os.path.join(ROOT, "tools", "libpmenv_ab.so"))}
    other = (f"{base} (two launches)" if base else
             f"tools build, PMENV_GEN_GEOM={os.environ.get('PMENV_GEN_GEOM')}" if os.environ.get("AB_GEN_FORCE") == "1" else
             f"advance_gen_kernel ablation PMENV_GEN_ABL={os.environ.get('PMENV_GEN_ABL')} (tools, timing only)"
             if os.environ.get("PMENV_GEN_ABL") is not None else
             "advance_gen_kernel, default cache policy (tools)" if os.environ.get("PMENV_GEN_POL0") == "1" else
             "advance_gen_kernel per-element (tools)" if perelem else "register step (tools)")
    out = {"K": K, "R": R, "other": other}
    for (B, N, W, F, ip) in SHAPES:
        if perelem and (B, N, W, F) == (16384, 64, 50, 6):
            continue
        key = f"{B}x{N}x{W}x{F}{'_ip' if ip else '_db'}"
        envs = {"gen": Env(libs["gen"], B, N, W, F, ip, True), "small": Env(libs["small"], B, N, W, F, ip, perelem)}
        paths = {n: e.lib.pmenv_step_path(e.h).decode() for n, e in envs.items()}
        res = {n: [] for n in envs}
        for e in envs.values():
            for _ in range(5):
                e.step()
        for _ in range(R):
            for n, e in envs.items():
                res[n].append(ab.timed(e.step, K))
        torch.cuda.synchronize()
        by = step_bytes(N, W, F) * B
        o = {}
        for n in envs:
            us = statistics.median(res[n])
            o[n] = {"us": us, "env_steps_per_s": B / us * 1e6, "frac": by / (us * 1e-6) / PEAK,
                    "path": paths[n].split(" | ")[-1 if ip else 0]}
        o["gen_vs_small_pct"] = 100.0 * (o["gen"]["us"] / o["small"]["us"] - 1.0)
        a, b = envs["gen"], envs["small"]
        o["same_steps"] = a.t == b.t
        o["windows_equal"] = bool(torch.equal(a.window().view(torch.int32), b.window().view(torch.int32)))
        o["market_equal"] = bool(torch.equal(a.window()[..., :F - 1].contiguous().view(torch.int32),
                                             b.window()[..., :F - 1].contiguous().view(torch.int32)))
        o["rewards_equal"] = bool(torch.equal(a.rew.view(torch.int32), b.rew.view(torch.int32)))   # bit patterns (NaN too)
        out[key] = o
        print(key, json.dumps(o), file=sys.stderr, flush=True)
        for e in envs.values():
            e.close()
        del envs, a, b
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
