"""Weights and snapshot I/O: safetensors only (nothing is ever unpickled).

``load_weights(dir)`` reads every ``*.safetensors`` shard of a directory into one dict (HF
naming, e.g. ``model.layers.0.self_attn.q_proj.weight``); ``save_weights`` writes one shard
atomically (random-init weights can be saved once for reproducible runs).
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Dict

import torch


def load_weights(path: str, device: str = "cpu") -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file

    p = Path(path)
    files = [p] if p.is_file() else sorted(p.glob("*.safetensors"))
    if not files:
        raise FileNotFoundError(f"no .safetensors files under {path}")
    out: Dict[str, torch.Tensor] = {}
    for f in files:
        out.update(load_file(str(f), device=device))
    return out


def save_weights(state: Dict[str, torch.Tensor], path: str, name: str = "model.safetensors") -> str:
    from safetensors.torch import save_file

    p = Path(path)
    p.mkdir(parents=True, exist_ok=True)
    tmp = p / (name + ".tmp")
    save_file({k: v.detach().contiguous().cpu() for k, v in state.items()}, str(tmp))
    os.replace(tmp, p / name)
    return str(p / name)
