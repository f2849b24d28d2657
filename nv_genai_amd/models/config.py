"""Model architecture configs.

Dimensions are the public model-card values the reference's model names imply
(SURVEY.md §2.C): the reference only names the models (``meta/llama3-8b-instruct``,
``meta/llama3-70b-instruct`` — deploy/compose/docker-compose-nim-ms.yaml:4,
rag-app-api-catalog-text-chatbot.yaml:14; ``snowflake/arctic-embed-l`` — compose.env:25-27).
Weights are random-initialised (no checkpoints are reachable), so every benchmark runs the
real architecture on synthetic inputs.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, field, replace
from typing import Optional


@dataclass(frozen=True)
class LlamaConfig:
    name: str = "llama3-8b"
    vocab_size: int = 128256
    hidden: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = None
    eps: float = 1e-5
    max_position: int = 8192
    bos_id: int = 128000
    eos_ids: tuple = (128001, 128009)

    @property
    def qkv_dim(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def num_params(self) -> int:
        per_layer = (self.hidden * self.qkv_dim + self.heads * self.head_dim * self.hidden
                     + 3 * self.hidden * self.ffn + 2 * self.hidden)
        return per_layer * self.layers + 2 * self.vocab_size * self.hidden + self.hidden

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.layers * self.kv_heads * self.head_dim * dtype_bytes

    def to_dict(self):
        return asdict(self)


@dataclass(frozen=True)
class EncoderConfig:
    """BERT-large-class bidirectional encoder (snowflake-arctic-embed-l shape)."""

    name: str = "arctic-embed-l"
    vocab_size: int = 30522
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    ffn: int = 4096
    max_position: int = 512
    type_vocab: int = 2
    eps: float = 1e-12
    pooling: str = "cls"  # "cls" | "mean"
    normalize: bool = True
    query_prefix: str = "Represent this sentence for searching relevant passages: "
    passage_prefix: str = ""
    num_labels: int = 0  # >0: cross-encoder / reranker head on the pooled output

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads

    def to_dict(self):
        return asdict(self)


LLAMA_PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(name="llama3-70b", hidden=8192, layers=80, heads=64, kv_heads=8,
                              ffn=28672),
    # small language model (models/NeMo/slm/slm_pretraining_sft.ipynb#cell 18: 12 layers,
    # hidden 768) in this architecture, for training/pretrain.py
    "slm-125m": LlamaConfig(name="slm-125m", hidden=768, layers=12, heads=12, kv_heads=12,
                            head_dim=64, ffn=2048, rope_theta=10000.0, max_position=2048),
    # small configs with the same structure for CPU tests / smoke runs
    "llama-tiny": LlamaConfig(name="llama-tiny", vocab_size=32768, hidden=256, layers=2, heads=4,
                              kv_heads=2, head_dim=64, ffn=512, max_position=2048,
                              bos_id=1, eos_ids=(2,)),
    "llama-small": LlamaConfig(name="llama-small", vocab_size=32768, hidden=1024, layers=4,
                               heads=8, kv_heads=2, head_dim=128, ffn=2816,
                               max_position=8192, bos_id=1, eos_ids=(2,)),
}

ENCODER_PRESETS = {
    "arctic-embed-l": EncoderConfig(),
    "nv-embed-qa": EncoderConfig(name="nv-embed-qa"),
    "e5-large-v2": EncoderConfig(name="e5-large-v2", pooling="mean", query_prefix="query: ",
                                 passage_prefix="passage: "),
    "all-minilm-l6-v2": EncoderConfig(name="all-minilm-l6-v2", hidden=384, layers=6, heads=12,
                                      ffn=1536, pooling="mean", query_prefix=""),
    "bge-reranker-large": EncoderConfig(name="bge-reranker-large", num_labels=1,
                                        normalize=False, query_prefix=""),
    "encoder-tiny": EncoderConfig(name="encoder-tiny", vocab_size=30522, hidden=128, layers=2,
                                  heads=2, ffn=256, max_position=512),
    "reranker-tiny": EncoderConfig(name="reranker-tiny", vocab_size=30522, hidden=128, layers=2,
                                   heads=2, ffn=256, max_position=512, num_labels=1,
                                   normalize=False, query_prefix=""),
}


def llama_config(name_or_cfg, **overrides) -> LlamaConfig:
    cfg = LLAMA_PRESETS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    return replace(cfg, **overrides) if overrides else cfg


def encoder_config(name_or_cfg, **overrides) -> EncoderConfig:
    cfg = ENCODER_PRESETS[name_or_cfg] if isinstance(name_or_cfg, str) else name_or_cfg
    return replace(cfg, **overrides) if overrides else cfg
