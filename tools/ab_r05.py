"""Round 5 A/B: the relayed step (round 5: device-sequenced epoch / parity under capture; its
first form, an ordered ticket per workgroup, is the run in profiles/ab_r05/ticket_r05b.*)
and the look-back GAE with its forward-progress fallback, against the round-4 library
(tools/libpmenv_r04.so, built from commit 0ea79d4's pm-rl_amd/csrc by hipcc with the
product's flags), in ONE process, interleaved; plus a hipGraph-replayed relay step against
eager. Raw C ABI calls on prebuilt arguments (the structs are the same in ABI 2 and 3).

Prints JSON: per shape, us per step (HIP events on the current stream over K steps,
median of R interleaved repetitions) for each library."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402

from pmenv import _abi, synth  # noqa: E402

DEV = torch.device("cuda:0")
K = int(os.environ.get("AB_K", "200"))
R = int(os.environ.get("AB_R", "7"))
LIBS = {"r05": os.path.join(ROOT, "pm-rl_amd", "pmenv", "libpmenv.so"),
        "r04": os.path.join(ROOT, "tools", "libpmenv_r04.so")}


def load(path):
    lib = ctypes.CDLL(path)
    for name, res, args in _abi.SIGNATURES:
        fn = getattr(lib, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    return lib


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream(DEV).cuda_stream)


class Env:
    def __init__(self, lib, B, N, W, path, db):
        self.lib = lib
        c = _abi.PmenvCfg()
        lib.pmenv_cfg_default(ctypes.byref(c), B, N, W, 5)
        h = ctypes.c_void_p()
        assert lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(h)) == 0, lib.pmenv_last_error(None)
        self.h = h
        assert lib.pmenv_set_step_path(h, path) == 0
        H = 64
        self.ser = synth.series(W + H, B, N, seed=B + N, device=DEV)
        self.act = synth.actions(H, B, N, seed=7, device=DEV)
        self.obs = [synth.window_from_series(self.ser, W), torch.empty(B, N, W, 5, device=DEV)]
        self.rew = torch.empty(B, device=DEV)
        assert lib.pmenv_reset(h, ctypes.c_void_p(self.obs[0].data_ptr()), None, stream()) == 0
        self.args = []
        for t in range(H):
            a = _abi.PmenvStepArgs()
            a.action, a.bar, a.reward = self.act[t].data_ptr(), self.ser[W + t].data_ptr(), self.rew.data_ptr()
            a.obs = self.obs[t % 2 if db else 0].data_ptr()
            a.obs_out = self.obs[(t + 1) % 2].data_ptr() if db else None
            self.args.append(a)
        self.t = 0
        self.H = H
        self.db = db

    def step(self):
        a = self.args[self.t % self.H]
        rc = self.lib.pmenv_step_ex(self.h, ctypes.byref(a), stream())
        assert rc == 0, self.lib.pmenv_last_error(self.h)
        self.t += 1

    def close(self):
        torch.cuda.synchronize()
        self.lib.pmenv_destroy(self.h)


def timed(fn, k):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / k


def relay_ab(libs):
    out = {}
    for (B, N, db) in ((4096, 30, False), (8192, 30, False), (4096, 30, True), (16384, 8, False), (2048, 30, False)):
        key = f"{B}x{N}{'_db' if db else '_ip'}"
        envs = {n: Env(lib, B, N, 50, 4, db) for n, lib in libs.items()}     # PMENV_STEP_PATH_RELAY
        res = {n: [] for n in envs}
        for n, e in envs.items():
            for _ in range(20):
                e.step()
        for _ in range(R):
            for n, e in envs.items():
                res[n].append(timed(e.step, K))
        out[key] = {n: statistics.median(v) for n, v in res.items()}
        out[key]["r05_vs_r04_pct"] = 100.0 * (out[key]["r05"] / out[key]["r04"] - 1.0)
        print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
        for e in envs.values():
            e.close()
    return out


def relay_graph(lib):
    """4,096 x 30 in place: a graph of 10 relay steps replayed, against 10 eager steps."""
    e = Env(lib, 4096, 30, 50, 4, False)
    for _ in range(20):
        e.step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream(DEV)
    s.wait_stream(torch.cuda.current_stream(DEV))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s), torch.cuda.graph(g, stream=s):
        for _ in range(10):
            e.step()
    torch.cuda.current_stream(DEV).wait_stream(s)
    path = lib.pmenv_step_path(e.h).decode()
    eager, graph = [], []
    for _ in range(R):
        eager.append(timed(lambda: [e.step() for _ in range(10)], K // 10) / 10)
        graph.append(timed(g.replay, K // 10) / 10)
    e.close()
    return {"path": path, "eager_us": statistics.median(eager), "graph_us": statistics.median(graph)}


def gae_ab(libs):
    out = {}
    for (T, B) in ((4096, 512), (2048, 4096), (16384, 64), (1000, 200)):
        r = torch.randn(T, B, device=DEV)
        v = torch.randn(T + 1, B, device=DEV)
        adv, ret = torch.empty(T, B, device=DEV), torch.empty(T, B, device=DEV)
        res = {}
        for n, lib in libs.items():
            ws = lib.pmenv_gae_workspace(T, B)
            work = torch.empty(max(ws // 8, 1), dtype=torch.float64, device=DEV)
            P = ctypes.c_void_p

            def call(lib=lib, work=work, ws=ws):
                assert lib.pmenv_gae_ex(P(r.data_ptr()), P(v.data_ptr()), None, P(adv.data_ptr()), P(ret.data_ptr()),
                                        T, B, 0.99, 0.95, P(work.data_ptr()), ws, stream()) == 0
            res[n] = call
        times = {n: [] for n in res}
        for n, f in res.items():
            for _ in range(20):
                f()
        outs = {}
        for _ in range(R):
            for n, f in res.items():
                times[n].append(timed(f, K))
        for n, f in res.items():
            f()
            torch.cuda.synchronize()
            outs[n] = (adv.clone(), ret.clone())
        key = f"{T}x{B}"
        out[key] = {n: statistics.median(t) for n, t in times.items()}
        out[key]["bitwise_equal"] = bool(torch.equal(outs["r05"][0], outs["r04"][0]) and
                                         torch.equal(outs["r05"][1], outs["r04"][1]))
        print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
    return out


def f2_ab(libs):
    """The trainer op at the agents' batch sizes (config/pg.py:7 BATCH_SIZE = 64): forward +
    backward per call (round 5: one workgroup, one launch for B <= 64; round 4: rows + fold)."""
    out = {}
    P = ctypes.c_void_p
    for (B, N, kind) in ((64, 30, 0), (64, 8, 0), (32, 30, 2), (64, 64, 0), (128, 30, 0)):
        g = torch.Generator(DEV).manual_seed(B * 100 + N)
        a = torch.randn(B, N, device=DEV, generator=g)
        v = torch.rand(B, device=DEV, generator=g) + 0.5
        pr = torch.rand(B, N, device=DEV, generator=g) * 0.1 + 0.95
        rew = torch.empty(1, device=DEV)
        ret = torch.empty(B, device=DEV)
        go = torch.ones(1, device=DEV)
        ga = torch.empty(B, N, device=DEV)
        calls, outs = {}, {}
        for n, lib in libs.items():
            work = torch.empty(lib.pmenv_batch_reward_workspace(B) // 8, dtype=torch.float64, device=DEV)

            def call(lib=lib, work=work):
                assert lib.pmenv_batch_reward_forward(P(a.data_ptr()), P(v.data_ptr()), P(pr.data_ptr()), B, N, kind, 0,
                                                      1.0, P(work.data_ptr()), P(rew.data_ptr()), P(ret.data_ptr()),
                                                      stream()) == 0
                assert lib.pmenv_batch_reward_backward(P(a.data_ptr()), P(v.data_ptr()), P(pr.data_ptr()), B, N, kind,
                                                       1.0, P(work.data_ptr()), P(go.data_ptr()), P(ga.data_ptr()),
                                                       stream()) == 0
            calls[n] = call
        times = {n: [] for n in calls}
        for n, f in calls.items():
            for _ in range(20):
                f()
        for _ in range(R):
            for n, f in calls.items():
                times[n].append(timed(f, K))
        for n, f in calls.items():
            f()
            torch.cuda.synchronize()
            outs[n] = (rew.clone(), ret.clone(), ga.clone())
        key = f"{B}x{N}_{['log', 'ret', 'sharpe'][kind]}"
        out[key] = {n: statistics.median(t) for n, t in times.items()}
        out[key]["bitwise_equal"] = all(torch.equal(x, y) for x, y in zip(outs["r05"], outs["r04"]))
        print(key, json.dumps(out[key]), file=sys.stderr, flush=True)
    return out


def main():
    torch.cuda.set_device(DEV)
    libs = {n: load(p) for n, p in LIBS.items()}
    if os.environ.get("AB_ONLY") == "f2":
        print(json.dumps({"K": K, "R": R, "f2": f2_ab(libs)}))
        return
    res = {"K": K, "R": R, "relay": relay_ab(libs), "gae": gae_ab(libs), "graph": relay_graph(libs["r05"]),
           "f2": f2_ab(libs)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
