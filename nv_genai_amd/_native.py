"""Loader for the host-side native runtime (``_rt``). It is plain C++ (no HIP), so if the
in-tree build is missing it is compiled on first import (a few seconds with g++)."""
from __future__ import annotations

import importlib


def _load_rt():
    try:
        return importlib.import_module("nv_genai_amd._rt")
    except ImportError:
        from . import _build

        _build.build_runtime()
        return importlib.import_module("nv_genai_amd._rt")


rt = _load_rt()
