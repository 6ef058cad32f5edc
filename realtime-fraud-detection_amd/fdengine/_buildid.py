"""Ties libfdengine.so to the source tree it was built from.

The build (fdengine/build.py) embeds `fd_build_id()` = "fdengine-build-id:src=<digest>;flags=<hipcc flags>" in the
library, where <digest> is a SHA-256 over the HIP sources, the csrc headers and include/fdengine.h (names and
bytes). The loader (fdengine/_native.py) recomputes the digest over the tree it runs from and refuses a library
built from other sources: a prebuilt .so that travelled to the GPU box with newer sources fails at import, naming
both digests, instead of running stale kernels against newer tests. No imports beyond the standard library: the
build loads this file by path before the package (and its library) exists.
"""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parent.parent          # realtime-fraud-detection_amd/
REPO_ROOT = PKG_ROOT.parent
MARK = "fdengine-build-id:"


def source_files(pkg_root: Path = PKG_ROOT, repo_root: Path = REPO_ROOT) -> list:
    csrc = Path(pkg_root) / "csrc"
    return sorted(csrc.glob("*.hip")) + sorted(csrc.glob("*.h")) + [Path(repo_root) / "include" / "fdengine.h"]


def digest_files(files) -> str:
    h = hashlib.sha256()
    for p in files:
        p = Path(p)
        h.update(p.name.encode())
        h.update(b"\0")
        h.update(p.read_bytes())
        h.update(b"\0")
    return h.hexdigest()[:32]


def source_digest(pkg_root: Path = PKG_ROOT, repo_root: Path = REPO_ROOT) -> str:
    return digest_files(source_files(pkg_root, repo_root))


def id_string(digest: str, flags) -> str:
    return f"{MARK}src={digest};flags={' '.join(flags)}"


def parse(build_id: str) -> dict:
    """"fdengine-build-id:src=...;flags=..." -> {"src": ..., "flags": ...}"""
    if not build_id.startswith(MARK):
        return {}
    out = {}
    for part in build_id[len(MARK):].split(";", 1):
        k, _, v = part.partition("=")
        out[k] = v
    return out


def embedded_id(lib_path: Path):
    """The build id string inside a built library (read from its bytes, without loading it); None if absent."""
    try:
        data = Path(lib_path).read_bytes()
    except OSError:
        return None
    i = data.find(MARK.encode())
    if i < 0:
        return None
    j = data.find(b"\0", i)
    return data[i:j].decode(errors="replace")


def check(build_id: str, pkg_root: Path = PKG_ROOT, repo_root: Path = REPO_ROOT) -> None:
    """Raise ImportError unless `build_id` (the loaded library's fd_build_id()) matches the sources under
    pkg_root / repo_root."""
    want = source_digest(pkg_root, repo_root)
    got = parse(build_id or "").get("src")
    if got != want:
        raise ImportError(
            f"libfdengine.so is stale: built from sources with digest {got!r}, the tree at {pkg_root} has {want!r}. "
            "Rebuild it in-tree (`python -c 'import __graft_entry__ as g; g.build()'`) before running.")
