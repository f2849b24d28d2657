"""Multi-attribute reward model (the role of ``nvidia/nemotron-4-340b-reward`` in the KG-RAG
evaluation: experimental/knowledge_graph_rag/pages/evaluation.py:38-56, BASELINE.md's
helpfulness / correctness / coherence / complexity / verbosity table).

A decoder scores a (question, answer) conversation: the pair is rendered with the Llama-3 chat
template (user turn, assistant turn), run causally through the decoder's weights and kernels
(:func:`~nv_genai_amd.models.ranker.packed_hidden`, packed sequences, no KV cache), and the
last token's final hidden row goes through a linear head with one output per attribute; each
attribute is ``4 * sigmoid(logit)``, the 0-4 range of the HelpSteer2 attributes Nemotron-4's
reward model predicts. Weights are random-init unless given (no checkpoints are reachable
here), like the ranker's head.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from ..utils.runtime import capture_guard

from .config import llama_config
from .llama import LlamaModel
from .ranker import packed_hidden

ATTRIBUTES = ("helpfulness", "correctness", "coherence", "complexity", "verbosity")

# served name -> decoder preset
REWARD_MODELS = {
    "nvidia/nemotron-4-340b-reward": "llama3-8b",
    "reward-small": "llama-small",
    "reward-tiny": "llama-tiny",
}


class RewardModel:
    def __init__(self, name: str = "nvidia/nemotron-4-340b-reward", device="cuda", dtype=torch.bfloat16,
                 weights: Optional[Dict[str, torch.Tensor]] = None, seed: int = 0, max_len: int = 4096):
        preset = REWARD_MODELS.get(name, name)
        self.name = name
        cfg = llama_config(preset)
        self.lm = LlamaModel(cfg, device, dtype=dtype, weights=weights, seed=seed)
        self.lm.lm_head = None
        self.cfg = cfg
        self.max_len = max_len
        dev = torch.device(device)
        self.device = dev
        if weights is not None and "reward_head.weight" in weights:
            self.head_w = weights["reward_head.weight"].to(dev, torch.float32)
            self.head_b = weights.get("reward_head.bias", torch.zeros(len(ATTRIBUTES))).to(dev, torch.float32)
        else:
            g = torch.Generator(device=dev).manual_seed(seed + 11)
            self.head_w = torch.empty(len(ATTRIBUTES), cfg.hidden, device=dev).normal_(0, 0.02, generator=g)
            self.head_b = torch.zeros(len(ATTRIBUTES), device=dev)
        self._tok = None
        # one forward at a time (executor threads of a server share the model), and none while
        # another thread captures a hipGraph: a library GEMM's first use beside a capture
        # invalidates it (utils.runtime.capture_guard)
        self.lock = threading.Lock()

    @property
    def tok(self):
        if self._tok is None:
            from ..utils.tokenizer import llm_tokenizer

            self._tok = llm_tokenizer()
        return self._tok

    def encode(self, question: str, answer: str) -> List[int]:
        ids = self.tok.apply_chat_template([{"role": "user", "content": question},
                                            {"role": "assistant", "content": answer}],
                                           add_generation_prompt=False)
        if len(ids) > self.max_len:   # keep the start (question) and the end of the answer
            ids = ids[: self.max_len // 2] + ids[-(self.max_len - self.max_len // 2):]
        V = self.cfg.vocab_size
        return [t % V for t in ids]

    @torch.inference_mode()
    def score_batch(self, pairs: Sequence[Tuple[str, str]]) -> List[Dict[str, float]]:
        """Attribute scores of each (question, answer) pair, one packed forward."""
        if not pairs:
            return []
        seqs = [self.encode(q, a) for q, a in pairs]
        lens = [len(s) for s in seqs]
        dev = self.device
        ids = torch.tensor([t for s in seqs for t in s], dtype=torch.int32, device=dev)
        pos = torch.tensor([i for n in lens for i in range(n)], dtype=torch.int32, device=dev)
        cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0).tolist()), dtype=torch.int32, device=dev)
        with self.lock, capture_guard():
            h = packed_hidden(self.lm, ids, pos, cu, max(lens), causal=True)
            last = h.index_select(0, (cu[1:] - 1).long()).float()
            s = 4.0 * torch.sigmoid(last @ self.head_w.t() + self.head_b)
            s = s.cpu()
        return [{a: round(float(v), 4) for a, v in zip(ATTRIBUTES, row)} for row in s]

    def score(self, question: str, answer: str) -> Dict[str, float]:
        return self.score_batch([(question, answer)])[0]


def format_scores(scores: Dict[str, float]) -> str:
    """The reward endpoint's message content: "helpfulness:3.1,correctness:...", the form the
    reference's get_reward_scores parses (evaluation.py:44-56)."""
    return ",".join(f"{a}:{scores[a]}" for a in ATTRIBUTES)


def parse_scores(content: str) -> Optional[Dict[str, float]]:
    try:
        out = {}
        for item in content.split(","):
            k, v = item.split(":")
            out[k.strip()] = float(v)
        return out if all(a in out for a in ATTRIBUTES) else None
    except (ValueError, AttributeError):
        return None
