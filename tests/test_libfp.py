"""The PMC-traffic fingerprint (tools/libfp.py): a deterministic hash of the product
library's sources and build script, so a rebuild of unchanged sources keeps bench.py's
roofline.traffic while any source edit drops it."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.libfp import source_sha256  # noqa: E402


def _copy_tree(dst):
    for rel in (os.path.join("pm-rl_amd", "csrc"), "include"):
        shutil.copytree(os.path.join(ROOT, rel), os.path.join(dst, rel))
    shutil.copy(os.path.join(ROOT, "pm-rl_amd", "build.py"), os.path.join(dst, "pm-rl_amd", "build.py"))


def test_source_fingerprint_is_stable_and_sensitive(tmp_path):
    here = source_sha256(ROOT)
    assert here is not None and len(here) == 64
    _copy_tree(str(tmp_path))
    assert source_sha256(str(tmp_path)) == here                 # same sources, another place
    with open(tmp_path / "pm-rl_amd" / "csrc" / "common.h", "a") as f:
        f.write("\n")
    assert source_sha256(str(tmp_path)) != here                 # any edit moves it
    os.remove(tmp_path / "pm-rl_amd" / "build.py")
    assert source_sha256(str(tmp_path)) is None                 # incomplete tree: no claim
