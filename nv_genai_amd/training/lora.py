"""LoRA adapters for the Llama projections (NeMo ``peft_scheme=lora``,
``target_modules=[attention_qkv]``, adapter_dim 32, alpha 32 — models/Gemma/lora.ipynb).

y = x Wᵀ + (α/r) · (x Aᵀ) Bᵀ with A ∈ ℝ^{r×in} (Kaiming-uniform), B ∈ ℝ^{out×r} (zeros), so
training starts exactly at the base model. Targets map to the fused serving weights:
``qkv`` → wqkv, ``o`` → wo, ``gate_up`` → wgu, ``down`` → wd. ``merge`` folds the adapter into
the bf16 serving weights (W += α/r·B·A), after which the engine serves the tuned model with no
adapter overhead; ``save``/``load`` use safetensors.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, Sequence, Tuple

import torch

TARGETS = {"qkv": "wqkv", "o": "wo", "gate_up": "wgu", "down": "wd"}


@dataclass
class LoRAConfig:
    r: int = 32
    alpha: float = 32.0
    dropout: float = 0.0
    targets: Sequence[str] = field(default_factory=lambda: ("qkv",))

    @property
    def scale(self) -> float:
        return self.alpha / self.r


class LoRA:
    def __init__(self, model, cfg: LoRAConfig = LoRAConfig(), seed: int = 0):
        self.model, self.cfg = model, cfg
        g = torch.Generator().manual_seed(seed)
        self.A: Dict[Tuple[int, str], torch.Tensor] = {}
        self.B: Dict[Tuple[int, str], torch.Tensor] = {}
        dev = model.embed.device
        for li, L in enumerate(model.layers):
            for t in cfg.targets:
                name = TARGETS[t]
                out_f, in_f = L[name].shape
                bound = 1.0 / math.sqrt(in_f)       # kaiming_uniform(a=sqrt(5)) bound
                a = (torch.rand(cfg.r, in_f, generator=g) * 2 - 1) * bound
                self.A[(li, name)] = a.to(dev).requires_grad_(True)
                self.B[(li, name)] = torch.zeros(out_f, cfg.r, device=dev, requires_grad=True)

    def parameters(self):
        for k in sorted(self.A):
            yield self.A[k]
            yield self.B[k]

    def named_parameters(self):
        for k in sorted(self.A):
            yield f"layers.{k[0]}.{k[1]}.lora_A", self.A[k]
            yield f"layers.{k[0]}.{k[1]}.lora_B", self.B[k]

    def linear(self, x: torch.Tensor, li: int, name: str) -> torch.Tensor:
        y = x @ self.model.layers[li][name].t()
        a = self.A.get((li, name))
        if a is None:
            return y
        h = x
        if self.cfg.dropout and torch.is_grad_enabled():
            h = torch.nn.functional.dropout(h, self.cfg.dropout)
        d = (h.to(torch.bfloat16) @ a.to(torch.bfloat16).t()) @ self.B[(li, name)].to(torch.bfloat16).t()
        return y + d * self.cfg.scale

    @torch.no_grad()
    def merge(self, keep_original: bool = True) -> None:
        """W += α/r·B·A in place. The bf16 originals are kept (unless told otherwise) so
        ``unmerge`` restores them bit-exactly rather than subtracting with rounding error."""
        self._orig = {}
        for k, a in self.A.items():
            w = self.model.layers[k[0]][k[1]]
            if keep_original:
                self._orig[k] = w.clone()
            w.copy_((w.float() + self.cfg.scale * (self.B[k].float() @ a.float())).to(w.dtype))

    @torch.no_grad()
    def unmerge(self) -> None:
        orig = getattr(self, "_orig", {})
        for k, a in self.A.items():
            w = self.model.layers[k[0]][k[1]]
            if k in orig:
                w.copy_(orig[k])
            else:
                w.copy_((w.float() - self.cfg.scale * (self.B[k].float() @ a.float())).to(w.dtype))
        self._orig = {}

    def state_dict(self) -> Dict[str, torch.Tensor]:
        return {n: p.detach().cpu().contiguous() for n, p in self.named_parameters()}

    @torch.no_grad()
    def load_state_dict(self, sd: Dict[str, torch.Tensor]) -> None:
        for n, p in self.named_parameters():
            p.copy_(sd[n].to(p.device, p.dtype))

    def save(self, path: str) -> None:
        from safetensors.torch import save_file

        os.makedirs(path, exist_ok=True)
        save_file(self.state_dict(), os.path.join(path, "adapter_model.safetensors"))
        with open(os.path.join(path, "adapter_config.json"), "w") as f:
            json.dump({**asdict(self.cfg), "targets": list(self.cfg.targets), "peft_type": "LORA"}, f)

    @classmethod
    def load(cls, model, path: str) -> "LoRA":
        from safetensors.torch import load_file

        with open(os.path.join(path, "adapter_config.json")) as f:
            c = json.load(f)
        lora = cls(model, LoRAConfig(r=c["r"], alpha=c["alpha"], dropout=c["dropout"], targets=tuple(c["targets"])))
        lora.load_state_dict(load_file(os.path.join(path, "adapter_model.safetensors")))
        return lora
