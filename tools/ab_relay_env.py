"""A/B of the relayed step's tiles: the product's fixed 8 KiB tiles of the flat window
(step_relay_kernel) against one tile per env (step_relay_env_kernel, the tools build with
PMENV_RELAY_ENV=1), in ONE process, interleaved, on the cache-resident shapes AUTO gives the
relay step — plus a bitwise check of the two after the timed steps (same inputs, same steps).

    PMENV_RELAY_ENV=1 python tools/ab_relay_env.py     # prints one JSON object
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

import ab_r05 as ab  # noqa: E402

SHAPES = [(4096, 30, False), (8192, 30, False), (2048, 30, False), (6144, 30, False), (4096, 30, True),
          (8192, 16, False), (4096, 64, False), (16384, 8, False)]


def main():
    assert os.environ.get("PMENV_RELAY_ENV") == "1", "run with PMENV_RELAY_ENV=1 (read by the tools build only)"
    torch.cuda.set_device(ab.DEV)
    libs = {"flat_tiles": ab.load(ab.LIBS["r05"]), "env_tiles": ab.load(os.path.join(ROOT, "tools", "libpmenv_ab.so"))}
    out = {"K": ab.K, "R": ab.R}
    for (B, N, db) in SHAPES:
        key = f"{B}x{N}{'_db' if db else '_ip'}"
        envs = {n: ab.Env(lib, B, N, 50, 4, db) for n, lib in libs.items()}     # PMENV_STEP_PATH_RELAY
        path = libs["env_tiles"].pmenv_step_path(envs["env_tiles"].h).decode()
        res = {n: [] for n in envs}
        for e in envs.values():
            for _ in range(20):
                e.step()
        for _ in range(ab.R):
            for n, e in envs.items():
                res[n].append(ab.timed(e.step, ab.K))
        o = {n: statistics.median(v) for n, v in res.items()}
        o["env_vs_flat_pct"] = 100.0 * (o["env_tiles"] / o["flat_tiles"] - 1.0)
        torch.cuda.synchronize()
        a, b = envs["flat_tiles"], envs["env_tiles"]
        same = a.t == b.t and all(torch.equal(x, y) for x, y in zip(a.obs, b.obs)) and torch.equal(a.rew, b.rew)
        o["bitwise_equal"] = bool(same)
        o["path"] = path
        out[key] = o
        print(key, json.dumps(o), file=sys.stderr, flush=True)
        for e in envs.values():
            e.close()
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
