"""Embedding / reranking engine.

Service contract kept from the NeMo Retriever microservices the reference calls:
``input_type`` query|passage (asymmetric prefixes — examples/5_mins_rag_no_gpu/main.py:51-52,
experimental/fm-asr-streaming-rag/chain-server/common.py:64-101), ``truncate`` END|START|NONE
(RetrievalAugmentedGeneration/common/utils.py:313), 512-token encoder window.

Batching: requests are tokenised, sorted by length and packed into varlen batches of at most
``max_batch_tokens`` tokens (no padding is computed at all); the serving layer's
:class:`DynamicBatcher` merges concurrent HTTP requests into one such call
(Triton's dynamic batching with queue delay, all-MiniLM-L6-v2_config.pbtxt:25-36).
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence

import torch

from ..utils.runtime import capture_guard
from ..observability.markers import gpu_range

from ..models.config import EncoderConfig, encoder_config
from ..models.encoder import EncoderModel
from ..utils.tokenizer import EmbedTokenizer, embed_tokenizer


def pca_whitening(x: torch.Tensor, eps: float = 1e-4):
    """(mu, W) of PCA whitening over calibration embeddings x [n, d]: y = normalise((x - mu) W)
    with W = C^-1/2 (eigenvalues floored at eps * the largest), fp32 on x's device."""
    x = x.double()
    mu = x.mean(0)
    xc = x - mu
    cov = xc.T @ xc / max(1, x.shape[0] - 1)
    lam, U = torch.linalg.eigh(cov)
    W = U @ torch.diag(1.0 / torch.sqrt(lam.clamp_min(0) + eps * lam.max())) @ U.T
    return mu.float(), W.float()


class EmbeddingEngine:
    def __init__(self, model: str | EncoderConfig = "arctic-embed-l", device: Optional[str] = None,
                 max_batch_tokens: int = 65536, seed: int = 0,
                 tokenizer: Optional[EmbedTokenizer] = None,
                 encoder: Optional[EncoderModel] = None):
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        from ..models.ranker import DECODER_RANKERS

        if isinstance(model, str) and model in DECODER_RANKERS:
            # decoder-based cross-encoder (nv-rerank-qa-mistral-4b): models/ranker.py
            from ..models.ranker import DecoderRanker, ranker_encoder_config

            self.cfg = ranker_encoder_config(model)
            encoder = encoder or DecoderRanker(model, self.device, seed=seed)
        else:
            self.cfg = encoder_config(model) if isinstance(model, str) else model
        self.model = encoder or EncoderModel(self.cfg, self.device, seed=seed)
        self.tok = tokenizer or embed_tokenizer()
        self.tok.max_len = min(self.tok.max_len, self.cfg.max_position)
        self.max_batch_tokens = max_batch_tokens
        self.lock = threading.Lock()
        self.dim = self.cfg.hidden
        self.stats = {"calls": 0, "texts": 0, "tokens": 0}
        self.center: Optional[torch.Tensor] = None
        self.whiten: Optional[torch.Tensor] = None

    def calibrate_center(self, texts: Sequence[str], input_type: str = "query") -> torch.Tensor:
        """Isotropy correction: subtract the mean embedding of a calibration set and
        re-normalise every output. Random-init encoders emit nearly collinear vectors (every
        query would retrieve the same passages); centring restores per-query diversity
        without changing the work done per request."""
        self.center = None
        self.center = self.embed(texts, input_type).mean(0)
        return self.center

    def calibrate_whitening(self, texts: Sequence[str], input_type: str = "query",
                            eps: float = 1e-4) -> None:
        """PCA whitening ("BERT-whitening"): y = normalise((x - mu) W), W = C^-1/2 from a
        calibration set (use >= dim texts for a full-rank estimate). Makes a random-init
        encoder's embeddings isotropic so retrieval over a synthetic index is as diverse as
        with a trained model; one [n, d] x [d, d] GEMM per call."""
        self.center, self.whiten = None, None
        self.center, self.whiten = pca_whitening(self.embed(texts, input_type), eps)

    @property
    def name(self) -> str:
        return self.cfg.name

    def _prefix(self, input_type: str) -> str:
        return self.cfg.query_prefix if input_type == "query" else self.cfg.passage_prefix

    def tokenize(self, texts: Sequence[str], input_type: str = "passage",
                 truncate: str = "END") -> List[List[int]]:
        pre = self._prefix(input_type)
        return self.tok.encode_batch([pre + t for t in texts], truncate=truncate)

    @torch.inference_mode()
    def embed_ids(self, seqs: List[List[int]], type_ids: Optional[List[List[int]]] = None) -> torch.Tensor:
        """Packed forward over token-id lists; returns [n, H] fp32 on the engine device
        (for a reranker config: [n, num_labels] logits)."""
        n = len(seqs)
        out_dim = self.cfg.num_labels or self.cfg.hidden
        out = torch.empty(n, out_dim, dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        order = sorted(range(n), key=lambda i: len(seqs[i]))
        # capture_guard: no library GEMM of ours starts while another thread captures a graph
        with self.lock, capture_guard():
            i = 0
            while i < n:
                batch, tok = [], 0
                while i < n and (not batch or tok + len(seqs[order[i]]) <= self.max_batch_tokens):
                    batch.append(order[i])
                    tok += len(seqs[order[i]])
                    i += 1
                # every host->device input goes through pinned memory: a pageable copy waits
                # for the copy engine to drain this stream, i.e. for the previous batch's
                # encoder forward, which under a concurrent LLM step can take a whole step
                pin = self.device.type == "cuda"
                ids = torch.tensor([t for b in batch for t in seqs[b]], dtype=torch.int32)
                pos = torch.tensor([p for b in batch for p in range(len(seqs[b]))], dtype=torch.int32)
                cu = [0]
                for b in batch:
                    cu.append(cu[-1] + len(seqs[b]))
                cu_t = torch.tensor(cu, dtype=torch.int32)
                rows = torch.tensor(batch, dtype=torch.int64)
                if pin:
                    ids, pos, cu_t, rows = (t.pin_memory() for t in (ids, pos, cu_t, rows))
                tt = None
                if type_ids is not None:
                    tt = torch.tensor([t for b in batch for t in type_ids[b]], dtype=torch.int32)
                    tt = (tt.pin_memory() if pin else tt).to(self.device, non_blocking=True)
                with gpu_range(f"embed n={len(batch)} tok={tok}"):
                    res = self.model.forward(ids.to(self.device, non_blocking=True),
                                             pos.to(self.device, non_blocking=True),
                                             cu_t.to(self.device, non_blocking=True),
                                             max(len(seqs[b]) for b in batch), tt)
                if self.center is not None and not self.cfg.num_labels:
                    res = res - self.center
                    if self.whiten is not None:
                        res = res @ self.whiten
                    res = res / res.norm(dim=-1, keepdim=True).clamp_min(1e-12)
                out.index_copy_(0, rows.to(self.device, non_blocking=True), res.to(out.dtype))
                self.stats["tokens"] += tok
            self.stats["calls"] += 1
            self.stats["texts"] += n
        return out

    def embed(self, texts: Sequence[str], input_type: str = "passage", truncate: str = "END") -> torch.Tensor:
        return self.embed_ids(self.tokenize(texts, input_type, truncate))

    def embed_query(self, text: str) -> List[float]:
        return self.embed([text], "query")[0].tolist()

    def embed_documents(self, texts: Sequence[str]) -> List[List[float]]:
        return self.embed(texts, "passage").tolist()

    # ------------------------------------------------------------------ reranking
    def rerank(self, query: str, passages: Sequence[str], truncate: str = "END") -> List[float]:
        """Cross-encoder logits for (query, passage) pairs (needs num_labels == 1)."""
        if not self.cfg.num_labels:
            # bi-encoder fallback: cosine of query vs passages
            q = self.embed([query], "query", truncate)
            p = self.embed(passages, "passage", truncate)
            return (p @ q[0]).tolist()
        pair = getattr(self.model, "encode_pair", None)
        if pair is not None:   # decoder ranker: its own tokenizer and pair template
            return self.embed_ids([pair(query, p, truncate) for p in passages])[:, 0].tolist()
        seqs, types = [], []
        for p in passages:
            enc = self.tok.tok.encode(query, p)
            ids = self.tok._trunc(enc.ids, truncate)
            seqs.append(ids)
            types.append(enc.type_ids[: len(ids)])
        return self.embed_ids(seqs, types)[:, 0].tolist()
