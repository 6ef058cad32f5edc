"""The loaded libfdengine.so is tied to the sources it was built from (fdengine/_buildid.py, fd_build_id()).

A prebuilt library that travels to the GPU box beside newer sources must refuse to load instead of running stale
kernels against newer tests (round 2: `unknown option: small_streams` from a library older than its tests)."""
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
PKG = REPO / "realtime-fraud-detection_amd"
sys.path.insert(0, str(PKG))

from fdengine import _buildid as B  # noqa: E402


def _import_with_sources(pkg_root: Path, repo_root: Path):
    env = dict(os.environ, FDENGINE_SRC_ROOT=str(pkg_root), FDENGINE_SRC_REPO=str(repo_root),
               PYTHONPATH=str(PKG), PYTHONDONTWRITEBYTECODE="1")
    return subprocess.run([sys.executable, "-c", "import fdengine; print('loaded')"], env=env, capture_output=True,
                          text=True, timeout=120)


def _copy_sources(tmp: Path):
    pkg, repo = tmp / "pkg", tmp
    shutil.copytree(PKG / "csrc", pkg / "csrc")
    (repo / "include").mkdir()
    shutil.copy(REPO / "include" / "fdengine.h", repo / "include" / "fdengine.h")
    return pkg, repo


def test_library_matches_tree():
    lib = PKG / "lib" / "libfdengine.so"
    got = B.parse(B.embedded_id(lib) or "")
    assert got.get("src") == B.source_digest(), "the in-tree libfdengine.so was not built from these sources"
    assert "--offload-arch=gfx950" in got.get("flags", "")


def test_unchanged_copy_loads(tmp_path):
    pkg, repo = _copy_sources(tmp_path)
    r = _import_with_sources(pkg, repo)
    assert r.returncode == 0 and "loaded" in r.stdout, r.stderr[-2000:]


@pytest.mark.parametrize("victim", ["csrc/ensemble.hip", "csrc/fd_internal.h", "include/fdengine.h"])
def test_touched_source_refuses_stale_library(tmp_path, victim):
    pkg, repo = _copy_sources(tmp_path)
    path = (pkg if victim.startswith("csrc") else repo) / victim
    path.write_bytes(path.read_bytes() + b"\n// edited after the build\n")
    r = _import_with_sources(pkg, repo)
    assert r.returncode != 0
    assert "ImportError" in r.stderr and "stale" in r.stderr, r.stderr[-2000:]
