"""A/B the fused-step kernel variants in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24). Variant = PMENV_ADVANCE at env creation."""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("PMENV_LIB", os.path.join(ROOT, "tools", "libpmenv_ab.so"))  # the A/B knobs: tools build
sys.path.insert(0, os.path.join(ROOT, "pm-rl_amd"))
import torch  # noqa: E402
from pmenv import TradingEnv, synth, _abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--variants", default="lds,reg256,reg512")
ap.add_argument("--envs", type=int, default=65536)
ap.add_argument("--assets", type=int, default=30)
ap.add_argument("--window", type=int, default=50)
ap.add_argument("--rounds", type=int, default=7)
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--H", type=int, default=64)
ap.add_argument("--phases", type=int, default=0, help="pmenv_step_args.phases (1: scalar step only)")
ap.add_argument("--series-days", type=int, default=512, help="resident series length for '+DAY' variants")
ap.add_argument("--commission", type=float, default=0.0)
ap.add_argument("--reward", default="log_returns")
a = ap.parse_args()
dev = torch.device("cuda:0")
B, N, W = a.envs, a.assets, a.window
lib = _abi.load()
ser = synth.series(a.H + W, B, N, device=dev)
act = synth.actions(a.H, B, N, device=dev)
envs = {}
# '+DAY' variants: resident-series mode, one shared [T, N, 4] series and a per-env day index
res_ser = synth.series(a.series_days, 1, N, device=dev)[:, 0].contiguous()
day0 = torch.randint(W, a.series_days - a.H, (B,), generator=torch.Generator().manual_seed(3)).to(dev, torch.int32)
days = [day0 + t for t in range(a.H)]
KNOBS = ("PMENV_ADVANCE", "PMENV_UNIT_ROWS", "PMENV_ABLATE", "PMENV_FUSED", "PMENV_K1_GROUPS",
         "PMENV_STREAM_BLOCK", "PMENV_STREAM_POL", "PMENV_FLAT", "PMENV_FLAT_BLOCK",
         "PMENV_FLAT_INPLACE", "PMENV_FLAT_IP_BLOCK", "PMENV_FLAT_IP_VEC", "PMENV_FLAT_DB_WG", "PMENV_K1",
         "PMENV_ONE", "PMENV_ONE_V", "PMENV_ONE_NOCAP", "PMENV_FLAT_S80", "PMENV_ONE_LDS_PAD", "PMENV_FLAT1", "PMENV_FLAT1_GEOM", "PMENV_FLAT1_XCD", "PMENV_FLAT1_POL", "PMENV_FLAT1_LDS_PAD")
for v in a.variants.split(","):
    # "base+KNOB=val+...": extra env knobs at creation (e.g. "o+PMENV_FUSED=0")
    base, *extra = v.split("+")
    # "lds" -> single-launch LDS kernel, "uR" -> streaming with R rows per unit, else default
    # "uR" -> R rows per unit, "aX" -> ablation X, combinable as "u16a3"; suffix "o" -> double-buffered
    for knob in KNOBS:
        os.environ.pop(knob, None)
    for kv in extra:
        if "=" in kv:
            os.environ[kv.split("=")[0]] = kv.split("=")[1]
    import re
    m = re.fullmatch(r"(?:u(\d+))?(?:a(\d+))?o?", base)
    if base in ("stream", "o", "so"):
        pass
    elif m and (m.group(1) or m.group(2)):
        if m.group(1):
            os.environ["PMENV_UNIT_ROWS"] = m.group(1)
        if m.group(2):
            os.environ["PMENV_ABLATE"] = m.group(2)
    else:
        os.environ["PMENV_ADVANCE"] = base
    obs = synth.window_from_series(ser, W)
    e = TradingEnv(num_envs=B, num_assets=N, window=W, device=dev, commission=a.commission, reward=a.reward)
    e.reset(obs)
    print(v, e.step_path, file=sys.stderr)
    envs[v] = (e, obs, torch.empty(B, device=dev), obs.clone() if base.endswith("o") else None)
for knob in KNOBS:
    os.environ.pop(knob, None)
stream = torch.cuda.current_stream()
sp = ctypes.c_void_p(stream.cuda_stream)
times = {v: [] for v in envs}
t_global = {v: 0 for v in envs}
bytes_step = (8 * N * W * 5 + 20) * B
for r in range(a.rounds):
    for v, (e, obs, rew, obs2) in envs.items():
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s0.record(stream)
        for i in range(a.steps):
            t = t_global[v] % a.H
            t_global[v] += 1
            args = _abi.PmenvStepArgs()
            args.action = act[t].data_ptr()
            args.bar = ser[W + t].data_ptr()
            if "DAY" in v.split("+"):
                args.bar, args.day, args.series_days = res_ser.data_ptr(), days[t].data_ptr(), a.series_days
            src, dst = (obs, obs2) if (obs2 is not None and t_global[v] % 2) else (obs2, obs) if obs2 is not None else (obs, None)
            args.obs = src.data_ptr()
            args.obs_out = dst.data_ptr() if dst is not None else None
            args.reward = rew.data_ptr()
            args.phases = a.phases
            rc = lib.pmenv_step_ex(e._h, ctypes.byref(args), sp)
            assert rc == 0
        s1.record(stream)
        torch.cuda.synchronize()
        if r > 0:
            times[v].append(s0.elapsed_time(s1) / a.steps * 1e3)
# all variants saw identical inputs from identical states: results must agree
ref = None
for v, (e, obs, rew, obs2) in envs.items():
    if obs2 is not None and t_global[v] % 2:
        obs = obs2                    # latest window of a double-buffered run
    if ("a" in v.split("+")[0] and v != "lds") or "DAY" in v.split("+"):
        continue                      # ablation builds compute wrong windows by design; DAY reads other bars
    if ref is None:
        ref = (obs, rew, e.value)
    else:
        # variants of the scalar step's reduction shape (PMENV_K1) differ in the last f64
        # bits of the sums; every other variant must agree bit for bit
        if "PMENV_K1" in v or ("PMENV_ONE" in v) != ("PMENV_ONE" in next(iter(envs))):
            assert torch.equal(obs[..., :4], ref[0][..., :4]), f"{v}: market channels differ"
            assert torch.allclose(obs, ref[0], rtol=2e-7, atol=1e-12), f"{v}: weights differ"
            assert torch.allclose(rew, ref[1], rtol=1e-6, atol=1e-9), f"{v}: reward differs"
            assert torch.allclose(e.value, ref[2], rtol=1e-12), f"{v}: value differs"
        else:
            assert torch.equal(obs, ref[0]), f"{v}: obs differs"
            assert torch.equal(rew, ref[1]), f"{v}: reward differs"
            assert torch.equal(e.value, ref[2]), f"{v}: value differs"
out = {}
for v, ts in times.items():
    med = statistics.median(ts)
    out[v] = {"median_us": med, "min_us": min(ts), "GBs": bytes_step / med / 1e3, "frac_8TBs": bytes_step / med / 1e3 / 8000}
print(json.dumps({"B": B, "N": N, "W": W, "variants": out}, indent=1))
