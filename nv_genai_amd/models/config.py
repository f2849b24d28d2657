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
    """Decoder-only LM config. The defaults are Llama-3-8B; the architecture switches below
    cover every decoder family the reference names:

    * ``mistral`` — Llama layout, optional sliding-window attention (Mistral-7B NIM config,
      experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:3);
    * ``mixtral`` — sparse MoE MLP, ``num_experts`` SwiGLU experts, top-``experts_per_tok``
      softmax routing (the reference's default chat model ``ai-mixtral-8x7b-instruct``,
      RetrievalAugmentedGeneration/common/configuration.py:75);
    * ``gemma`` — GeGLU (tanh GELU), RMSNorm with a (1 + w) scale, sqrt(hidden) embedding
      scale, tied embeddings, head_dim 256 (models/Gemma/*.ipynb, models/Codegemma/lora.ipynb);
    * ``starcoder2`` — LayerNorm with bias, biased projections, non-gated tanh-GELU MLP,
      sliding-window attention (models/StarCoder2/*.ipynb)."""

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
    arch: str = "llama"            # llama | mistral | mixtral | gemma | starcoder2
    norm: str = "rms"              # rms | layer (LayerNorm with bias)
    act: str = "silu"              # silu | gelu_tanh
    gated_mlp: bool = True         # act(gate) * up  (False: act(fc(x) + b) -> proj)
    attn_bias: bool = False        # q/k/v/o projection biases
    mlp_bias: bool = False
    embed_scale: float = 1.0       # Gemma multiplies the embedding by sqrt(hidden)
    tie_embeddings: bool = False
    sliding_window: int = 0        # 0: full causal attention; W: key j visible to query i iff i - W < j <= i
    num_experts: int = 0           # > 0: sparse MoE MLP
    experts_per_tok: int = 2
    chat_format: str = "llama3"    # llama3 | mistral | gemma | plain

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def qkv_dim(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def num_params(self) -> int:
        mlp = (3 if self.gated_mlp else 2) * self.hidden * self.ffn
        if self.is_moe:
            mlp = mlp * self.num_experts + self.num_experts * self.hidden
        per_layer = (self.hidden * self.qkv_dim + self.heads * self.head_dim * self.hidden
                     + mlp + 2 * self.hidden)
        heads = 1 if self.tie_embeddings else 2
        return per_layer * self.layers + heads * self.vocab_size * self.hidden + self.hidden

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
    # ---- other decoder families (public model-card dimensions)
    # Mistral-7B-Instruct v0.3 (32768-token vocabulary, full attention, theta 1e6)
    "mistral-7b": LlamaConfig(name="mistral-7b", arch="mistral", vocab_size=32768, rope_theta=1e6,
                              max_position=32768, bos_id=1, eos_ids=(2,), chat_format="mistral"),
    # Mistral-7B v0.1: 4096-token sliding window
    "mistral-7b-v0.1": LlamaConfig(name="mistral-7b-v0.1", arch="mistral", vocab_size=32000,
                                   rope_theta=10000.0, sliding_window=4096, max_position=32768,
                                   bos_id=1, eos_ids=(2,), chat_format="mistral"),
    "mixtral-8x7b": LlamaConfig(name="mixtral-8x7b", arch="mixtral", vocab_size=32000,
                                rope_theta=1e6, max_position=32768, num_experts=8,
                                experts_per_tok=2, bos_id=1, eos_ids=(2,), chat_format="mistral"),
    "gemma-7b": LlamaConfig(name="gemma-7b", arch="gemma", vocab_size=256000, hidden=3072,
                            layers=28, heads=16, kv_heads=16, head_dim=256, ffn=24576,
                            rope_theta=10000.0, eps=1e-6, act="gelu_tanh",
                            embed_scale=3072 ** 0.5, tie_embeddings=True, bos_id=2, eos_ids=(1, 107),
                            chat_format="gemma"),
    "gemma-2b": LlamaConfig(name="gemma-2b", arch="gemma", vocab_size=256000, hidden=2048,
                            layers=18, heads=8, kv_heads=1, head_dim=256, ffn=16384,
                            rope_theta=10000.0, eps=1e-6, act="gelu_tanh",
                            embed_scale=2048 ** 0.5, tie_embeddings=True, bos_id=2, eos_ids=(1, 107),
                            chat_format="gemma"),
    "codegemma-7b": LlamaConfig(name="codegemma-7b", arch="gemma", vocab_size=256000, hidden=3072,
                                layers=28, heads=16, kv_heads=16, head_dim=256, ffn=24576,
                                rope_theta=10000.0, eps=1e-6, act="gelu_tanh",
                                embed_scale=3072 ** 0.5, tie_embeddings=True, bos_id=2,
                                eos_ids=(1, 107), chat_format="gemma"),
    "starcoder2-3b": LlamaConfig(name="starcoder2-3b", arch="starcoder2", vocab_size=49152,
                                 hidden=3072, layers=30, heads=24, kv_heads=2, ffn=12288,
                                 rope_theta=999999.4, norm="layer", act="gelu_tanh",
                                 gated_mlp=False, attn_bias=True, mlp_bias=True,
                                 tie_embeddings=True, sliding_window=4096, max_position=16384,
                                 bos_id=0, eos_ids=(0,), chat_format="plain"),
    "starcoder2-7b": LlamaConfig(name="starcoder2-7b", arch="starcoder2", vocab_size=49152,
                                 hidden=4608, layers=32, heads=36, kv_heads=4, ffn=18432,
                                 rope_theta=1e6, norm="layer", act="gelu_tanh", gated_mlp=False,
                                 attn_bias=True, mlp_bias=True, tie_embeddings=True,
                                 sliding_window=4096, max_position=16384, bos_id=0, eos_ids=(0,),
                                 chat_format="plain"),
    "starcoder2-15b": LlamaConfig(name="starcoder2-15b", arch="starcoder2", vocab_size=49152,
                                  hidden=6144, layers=40, heads=48, kv_heads=4, ffn=24576,
                                  rope_theta=100000.0, norm="layer", act="gelu_tanh",
                                  gated_mlp=False, attn_bias=True, mlp_bias=True,
                                  sliding_window=4096, max_position=16384, bos_id=0, eos_ids=(0,),
                                  chat_format="plain"),
    # nv-rerank-qa-mistral-4b: Mistral-7B v0.1 cut to its first 16 layers (bidirectional)
    "mistral-4b-rerank": LlamaConfig(name="mistral-4b-rerank", arch="mistral", vocab_size=32000,
                                     layers=16, rope_theta=10000.0, max_position=4096, bos_id=1,
                                     eos_ids=(2,), chat_format="mistral"),
    # LLaVA-1.5's language model (Vicuna-7B = Llama-2-7B dims) and the NeVA-22B-class decoder
    "vicuna-7b": LlamaConfig(name="vicuna-7b", vocab_size=32000, hidden=4096, layers=32, heads=32,
                             kv_heads=32, ffn=11008, rope_theta=10000.0, max_position=4096,
                             bos_id=1, eos_ids=(2,), chat_format="plain"),
    "neva-22b-llm": LlamaConfig(name="neva-22b-llm", vocab_size=32768, hidden=6144, layers=40,
                                heads=48, kv_heads=8, ffn=24576, rope_theta=10000.0,
                                max_position=4096, bos_id=1, eos_ids=(2,), chat_format="plain"),
    # small configs with the same structure for CPU tests / smoke runs
    "llama-tiny": LlamaConfig(name="llama-tiny", vocab_size=32768, hidden=256, layers=2, heads=4,
                              kv_heads=2, head_dim=64, ffn=512, max_position=2048,
                              bos_id=1, eos_ids=(2,)),
    # Llama-3-70B's attention layout (64 q : 8 kv heads: at TP=8 one KV head per rank) at tiny width
    "llama70b-tiny": LlamaConfig(name="llama70b-tiny", vocab_size=32768, hidden=256, layers=2, heads=64,
                                 kv_heads=8, head_dim=16, ffn=512, max_position=2048,
                                 bos_id=1, eos_ids=(2,)),
    # Llama-3-70B's attention layout with its real head_dim 128 at a small width: at TP=8 each
    # rank holds 8 q heads and 1 KV head and the q/k/v shard is 1280 wide (as 70B's), so the
    # one-GPU TP=8 rehearsal runs the GPU kernels of a 70B rank; hidden 2048 makes a 256-token
    # step's all-reduce 1 MiB, past the two-shot threshold
    "llama70b-small": LlamaConfig(name="llama70b-small", vocab_size=32768, hidden=2048, layers=2, heads=64,
                                  kv_heads=8, head_dim=128, ffn=4096, max_position=8192, bos_id=1,
                                  eos_ids=(2,)),
    # Llama-3-8B's attention layout (32 q : 8 kv heads of 128) at a small width: the headline's
    # GQA group and work-item counts in step-graph GPU tests
    "llama3-gqa-small": LlamaConfig(name="llama3-gqa-small", vocab_size=32768, hidden=1024, layers=2, heads=32,
                                    kv_heads=8, head_dim=128, ffn=2816, max_position=8192, bos_id=1,
                                    eos_ids=(2,)),
    "llama-small": LlamaConfig(name="llama-small", vocab_size=32768, hidden=1024, layers=4,
                               heads=8, kv_heads=2, head_dim=128, ffn=2816,
                               max_position=8192, bos_id=1, eos_ids=(2,)),
    "mistral-tiny": LlamaConfig(name="mistral-tiny", arch="mistral", vocab_size=32768, hidden=256,
                                layers=2, heads=4, kv_heads=2, head_dim=64, ffn=512,
                                rope_theta=1e6, sliding_window=96, max_position=2048, bos_id=1,
                                eos_ids=(2,), chat_format="mistral"),
    "mixtral-tiny": LlamaConfig(name="mixtral-tiny", arch="mixtral", vocab_size=32768, hidden=256,
                                layers=2, heads=4, kv_heads=2, head_dim=64, ffn=384,
                                rope_theta=1e6, num_experts=4, experts_per_tok=2,
                                max_position=2048, bos_id=1, eos_ids=(2,), chat_format="mistral"),
    "gemma-tiny": LlamaConfig(name="gemma-tiny", arch="gemma", vocab_size=32768, hidden=256,
                              layers=2, heads=2, kv_heads=1, head_dim=256, ffn=512,
                              rope_theta=10000.0, eps=1e-6, act="gelu_tanh", embed_scale=16.0,
                              tie_embeddings=True, max_position=2048, bos_id=1, eos_ids=(2,),
                              chat_format="gemma"),
    "starcoder2-tiny": LlamaConfig(name="starcoder2-tiny", arch="starcoder2", vocab_size=32768,
                                   hidden=256, layers=2, heads=4, kv_heads=2, head_dim=64, ffn=512,
                                   rope_theta=1e5, norm="layer", act="gelu_tanh", gated_mlp=False,
                                   attn_bias=True, mlp_bias=True, tie_embeddings=True,
                                   sliding_window=96, max_position=2048, bos_id=1, eos_ids=(2,),
                                   chat_format="plain"),
    # small models of the real families' shapes for GPU kernel tests (head_dim 128 / 256)
    "mixtral-small": LlamaConfig(name="mixtral-small", arch="mixtral", vocab_size=32768,
                                 hidden=1024, layers=2, heads=8, kv_heads=2, head_dim=128,
                                 ffn=1792, rope_theta=1e6, num_experts=8, experts_per_tok=2,
                                 max_position=8192, bos_id=1, eos_ids=(2,), chat_format="mistral"),
    "mistral-small": LlamaConfig(name="mistral-small", arch="mistral", vocab_size=32768,
                                 hidden=1024, layers=2, heads=8, kv_heads=2, head_dim=128,
                                 ffn=2816, rope_theta=1e6, sliding_window=200, max_position=8192,
                                 bos_id=1, eos_ids=(2,), chat_format="mistral"),
    "starcoder2-small": LlamaConfig(name="starcoder2-small", arch="starcoder2", vocab_size=32768,
                                    hidden=1024, layers=2, heads=8, kv_heads=2, head_dim=128,
                                    ffn=4096, rope_theta=1e5, norm="layer", act="gelu_tanh",
                                    gated_mlp=False, attn_bias=True, mlp_bias=True,
                                    tie_embeddings=True, sliding_window=200, max_position=8192,
                                    bos_id=1, eos_ids=(2,), chat_format="plain"),
    "gemma-small": LlamaConfig(name="gemma-small", arch="gemma", vocab_size=32768, hidden=1024,
                               layers=2, heads=8, kv_heads=1, head_dim=256, ffn=2048,
                               rope_theta=10000.0, eps=1e-6, act="gelu_tanh", embed_scale=32.0,
                               tie_embeddings=True, max_position=8192, bos_id=1, eos_ids=(2,),
                               chat_format="gemma"),
}

# DecoderConfig is the family-neutral name of the same dataclass
DecoderConfig = LlamaConfig

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
