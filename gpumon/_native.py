"""Loader for the in-tree native extensions.

The extensions are built in-tree (``make`` or ``__graft_entry__.build()``) so that they travel with
the repository snapshot to a GPU box. There is no pure-Python fallback for the sampler/renderer/
server: if ``_core`` is missing, importing it fails loudly with the build command.
"""

from __future__ import annotations

import importlib
import os

_BUILD_HINT = "build it in-tree first: `make -C {root}` (or python -c 'import __graft_entry__ as g; g.build()')"


def _root() -> str:
    return os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def core():
    """Return the ``gpumon._core`` C++ extension module (raises ImportError if not built)."""
    try:
        return importlib.import_module("gpumon._core")
    except ImportError as e:  # pragma: no cover - exercised only on unbuilt trees
        raise ImportError("gpumon._core native extension is not built; " + _BUILD_HINT.format(root=_root())) from e


def hip():
    """Return the ``gpumon._hip`` HIP-kernel extension (gfx950). Raises ImportError if not built."""
    try:
        return importlib.import_module("gpumon._hip")
    except ImportError as e:
        raise ImportError("gpumon._hip HIP extension is not built; " + _BUILD_HINT.format(root=_root())) from e


def native_available() -> dict:
    out = {}
    for name in ("_core", "_hip"):
        try:
            importlib.import_module("gpumon." + name)
            out[name] = True
        except ImportError:
            out[name] = False
    return out
