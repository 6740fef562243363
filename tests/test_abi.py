"""The C-ABI library loads and exports exactly what include/pmenv.h declares
(no compute calls: this runs on CPU-only hosts)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pmenv.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pmenv_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from pmenv import _abi
    lib = _abi.load()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), f"libpmenv.so lacks {n}"
    bound = {s[0] for s in _abi.SIGNATURES}
    assert set(names) == bound, f"ctypes binding drift: {set(names) ^ bound}"
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\b(pmenv_[a-z_]+)\b", out))
    assert exported == set(names), f"exported but undeclared / declared but missing: {exported ^ set(names)}"


def test_library_is_gfx950_code_object():
    from pmenv import _abi
    blob = open(_abi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_abi_version_and_cfg_defaults_match_reference_config():
    from pmenv import _abi
    lib = _abi.load()
    assert lib.pmenv_abi_version() == _abi.PMENV_ABI_VERSION
    c = _abi.PmenvCfg()
    lib.pmenv_cfg_default(ctypes.byref(c), 7, 30, 50, 5)
    assert (c.num_envs, c.num_assets, c.window, c.features, c.close_channel) == (7, 30, 50, 5, 3)
    # config/base.py:47-53
    assert c.init_cash == 25000 and c.commission == 0.0 and c.reward_scale == 1.0
    assert c.risk_free_rate == 0.04 and c.reward_kind == 0
    assert c.norm_mode == 0 and c.ring_mode == 0 and c.ret_mode == 0 and c.mu_tol == 1e-10   # ret: GROSS
    assert ctypes.sizeof(_abi.PmenvCfg) == 88


def test_state_layout_is_consistent():
    from pmenv import _abi
    from pmenv.config import EnvConfig
    lib = _abi.load()
    for B, N, W in [(1, 5, 50), (4096, 30, 50), (3, 7, 6)]:
        c = EnvConfig(num_envs=B, num_assets=N, window=W).to_c()
        off = (ctypes.c_size_t * _abi.STATE_FIELDS)()
        assert lib.pmenv_state_layout(ctypes.byref(c), off) == 0
        up = lambda x: (x + 15) // 16 * 16  # noqa: E731
        assert list(off)[:4] == [0, up(8 * B), 2 * up(8 * B), 3 * up(8 * B)]
        assert all(o % 16 == 0 for o in off)
        assert off[5] - off[4] >= 4 * B * W * N and off[6] - off[5] >= 8 and off[7] - off[6] >= 4 * B * N
        assert lib.pmenv_state_bytes_for(ctypes.byref(c)) >= off[7] + 4 * B * N


def test_create_rejects_bad_config_without_touching_the_gpu():
    from pmenv import _abi
    lib = _abi.load()
    c = _abi.PmenvCfg()
    lib.pmenv_cfg_default(ctypes.byref(c), 4, 30, 50, 5)
    c.close_channel = 4                     # the weight channel is not a price
    h = ctypes.c_void_p()
    assert lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1
    assert b"close_channel" in lib.pmenv_last_error(None)
    c.close_channel = 3
    c.window = 4000                         # W*F beyond the LDS tile
    assert lib.pmenv_create(ctypes.byref(c), 0, ctypes.byref(h)) == -1
    assert not h.value


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    from pmenv import _abi
    monkeypatch.setattr(_abi, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_abi, "_lib", None)
    with pytest.raises(ImportError):
        _abi.load()


def test_product_does_not_reference_the_oracle():
    pkg = os.path.join(ROOT, "pm-rl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")) and f != "build.py":
                txt = open(os.path.join(dirpath, f)).read()
                assert "oracle" not in txt.lower(), f"{f} references the oracle"


def test_product_library_reads_no_knobs_and_has_no_ablation_variants():
    """The product library calls no getenv (nothing in the environment can alter the
    timed path) and carries none of the timing-only variants of the tools build
    (tools/libpmenv_ab.so, linked with tools/ab/pmenv_ab.hip): no work-skipping ABL / SKIP instantiations, no
    80-SGPR twins, no A/B-only geometries."""
    from pmenv import _abi
    undef = subprocess.run(["nm", "-D", "--undefined-only", _abi.LIB_PATH], capture_output=True, text=True).stdout
    assert "getenv" not in undef
    syms = subprocess.run(["nm", "-C", _abi.LIB_PATH], capture_output=True, text=True).stdout
    kernels = set(re.findall(r"__device_stub__(\w+<[^>]*>)", syms))
    assert kernels, "no kernel stubs found"
    for k in kernels:
        args = [a.strip() for a in k[k.index("<") + 1:-1].split(",")]
        name = k[:k.index("<")]
        assert "s80" not in name and "nocap" not in name, k
        if name == "advance_flat_inplace_kernel":                                   # 512 x 2 / 256 x 2, no SKIP bits
            assert args in (["512", "2", "0", "0"], ["512", "2", "1", "0"], ["256", "2", "0", "0"]), k
        if name == "step_env_kernel":
            assert args[0] == "4" and args[3] == "0", k                             # V = 4, ABL = 0
        if name == "advance_rows_kernel":
            assert args[0] == "512" and args[3] == "0" and args[4] == "false", k    # ABL = 0, not fused
        if name == "step_flat_kernel":
            assert args[:2] in (["256", "4"], ["128", "8"], ["512", "2"]), k        # the product geometries
        if name == "step_flat_vec_kernel":
            assert args[0] in ("2", "4", "8") and args[1:3] == ["256", "4"], k      # A, 256 x 4
    assert not any(k.startswith(("gae_tile_vec_kernel", "replay_gather_f5_kernel", "advance_flat_kernel<",
                                 "batch_reward_fwd_"))
                   for k in kernels)


def test_step_path_kinds_match_the_header():
    """pmenv_step_path_kind in include/pmenv.h and the Python wrapper's names agree."""
    from pmenv import _abi
    hdr = open(os.path.join(ROOT, "include", "pmenv.h")).read()
    kinds = dict((m.group(1).lower(), int(m.group(2)))
                 for m in re.finditer(r"PMENV_STEP_PATH_(\w+) = (\d+)", hdr))
    assert kinds == {"auto": 0, "one_launch": 1, "two_launch": 2, "flat": 3, "relay": 4}
    assert _abi.STEP_PATHS == kinds


def test_c_caller_links_the_abi():
    """tests/c_abi/c_abi_step (a plain C caller, built by pm-rl_amd/build.py) resolves
    libpmenv.so from the tree."""
    binary = os.path.join(ROOT, "tests", "c_abi", "c_abi_step")
    if not os.path.exists(binary):
        pytest.skip("not built")
    out = subprocess.run(["ldd", binary], capture_output=True, text=True).stdout
    line = next(l for l in out.splitlines() if "libpmenv.so" in l)
    assert "not found" not in line and os.path.realpath(line.split("=>")[1].split()[0]) == \
        os.path.realpath(os.path.join(ROOT, "pm-rl_amd", "pmenv", "libpmenv.so"))


def test_product_dispatch_has_no_conditional_compilation():
    """The product's host side (pmenv.hip, launch.h, handle.h) reads straight through: no
    #if / #ifdef, no environment variable; the tools build's variants sit in tools/ab/
    behind the pmenv_tools hooks, whose product definitions are weak no-ops."""
    csrc = os.path.join(ROOT, "pm-rl_amd", "csrc")
    for f in ("pmenv.hip", "launch.h", "handle.h"):
        txt = open(os.path.join(csrc, f)).read()
        assert not re.search(r"^\s*#\s*if", txt, re.M), f"{f} has conditional compilation"
        assert "getenv" not in txt, f"{f} reads the environment"
    from pmenv import _abi
    syms = subprocess.run(["nm", "-C", _abi.LIB_PATH], capture_output=True, text=True).stdout
    hooks = [l for l in syms.splitlines() if "pmenv_tools::" in l]
    assert hooks and all(l.split()[1] == "W" for l in hooks), "the product's tools hooks must be the weak no-ops"
