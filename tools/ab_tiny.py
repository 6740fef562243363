"""A/B of the smallest windows' step: step_tiny_kernel (the product: the env block staged
in LDS by 16-B loads, the reward computed before the barrier) against step_small_kernel
(the tools build with PMENV_TINY_OFF=1), in ONE process, interleaved, per shape: us per
step (HIP events over K back-to-back steps, median of R; launch-rate bound at one env — run
under `rocprofv3 --kernel-trace --stats` for the kernels' own durations) and whether the two
give the same windows and rewards after the same steps.

    PMENV_TINY_OFF=1 python tools/ab_tiny.py      # prints one JSON object
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import ab_gen  # noqa: E402
import ab_r05 as ab  # noqa: E402

K = int(os.environ.get("AB_K", "500"))
R = int(os.environ.get("AB_R", "5"))
# (B, N, W, F, in place): config 1, config 1 at 64 / 4,096 envs, F = 3 and 8 tiny windows, N = 64
SHAPES = [(1, 5, 50, 5, True), (1, 5, 50, 5, False), (64, 5, 50, 5, True), (4096, 5, 50, 5, True),
          (16, 7, 10, 3, True), (8, 8, 25, 8, False), (4, 64, 8, 4, True)]


def main():
    assert os.environ.get("PMENV_TINY_OFF") == "1", "run with PMENV_TINY_OFF=1 (read by the tools build only)"
    torch.cuda.set_device(ab.DEV)
    libs = {"tiny": ab.load(ab.LIBS["r05"]), "small": ab.load(os.path.join(ROOT, "tools", "libpmenv_ab.so"))}
    out = {"K": K, "R": R}
    for (B, N, W, F, ip) in SHAPES:
        key = f"{B}x{N}x{W}x{F}{'_ip' if ip else '_db'}"
        envs = {n: ab_gen.Env(lib, B, N, W, F, ip, False) for n, lib in libs.items()}
        paths = {n: e.lib.pmenv_step_path(e.h).decode() for n, e in envs.items()}
        res = {n: [] for n in envs}
        for e in envs.values():
            for _ in range(20):
                e.step()
        for _ in range(R):
            for n, e in envs.items():
                res[n].append(ab.timed(e.step, K))
        torch.cuda.synchronize()
        o = {n: {"us": statistics.median(res[n]), "path": paths[n]} for n in envs}
        a, b = envs["tiny"], envs["small"]
        o["windows_equal"] = bool(torch.equal(a.window().view(torch.int32), b.window().view(torch.int32)))
        o["rewards_equal"] = bool(torch.equal(a.rew.view(torch.int32), b.rew.view(torch.int32)))   # bit patterns (NaN too)
        out[key] = o
        print(key, json.dumps(o), file=sys.stderr, flush=True)
        for e in envs.values():
            e.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
