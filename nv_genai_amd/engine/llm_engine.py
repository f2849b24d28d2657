"""LLM serving engine: continuous batching over a paged KV cache, hipGraph-captured decode.

Replaces NIM / TensorRT-LLM. Components:

* :class:`nv_genai_amd._rt.Scheduler` (C++) — FCFS admission against the KV-block budget,
  chunked prefill under a token budget, preemption-by-recompute when decode runs out of
  blocks, prefix caching of full 64-token pages (shared RAG templates / system prompts hit).
* :class:`nv_genai_amd.models.llama.LlamaModel` — the gfx950 kernel forward.
* Decode steps run from hipGraphs captured per padded batch size (the whole step — 32 layers,
  LM head and the sampling kernel — replays as one graph launch), prefill runs eagerly
  (it is GEMM-bound, launch overhead is noise there).

Engine knobs mirror the TRT-LLM envelope the reference configures
(experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:28-39): max_batch_size ->
``max_num_seqs``, max_input_len/max_output_len -> ``max_model_len``,
kv_cache_free_gpu_mem_fraction -> ``kv_cache_fraction``, tensor_para_size -> ``tp``.
"""
from __future__ import annotations

import collections
import itertools
import logging
import os
import random
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .. import ops
from ..observability.markers import gpu_range
from .._native import rt
from ..models.config import LlamaConfig, llama_config
from ..models.llama import AttnMeta, LlamaModel
from ..parallel.dist import ParallelContext, get_context
from ..utils.faults import FaultInjector
from ..utils.tokenizer import IncrementalDetokenizer, LLMTokenizer, llm_tokenizer
from .beam import BeamGroup, advance
from .replica import ReplicaMixin
from .step_graphs import StepGraphMixin

log = logging.getLogger(__name__)
_KV_SHARE_STATS = os.environ.get("NGA_KV_SHARE_STATS", "0") == "1"


@dataclass
class SamplingParams:
    temperature: float = 0.2        # chain-server defaults (server.py:83-88)
    top_p: float = 0.7
    top_k: int = 0
    max_tokens: int = 1024
    stop: Sequence[str] = ()
    stop_token_ids: Sequence[int] = ()
    ignore_eos: bool = False
    seed: Optional[int] = None
    repetition_penalty: float = 1.0
    logprobs: bool = False
    min_tokens: int = 0
    frequency_penalty: float = 0.0  # OpenAI semantics over generated tokens:
    presence_penalty: float = 0.0   #   logit -= freq * count + presence * (count > 0)
    response_format: Optional[str] = None   # "json_object": grammar-constrained JSON output
    beam_width: int = 1             # > 1: beam search (engine/beam.py); sampling knobs ignored
    length_penalty: float = 1.0     # beam hypotheses score sum_logprob / len ** length_penalty


@dataclass
class Request:
    id: int
    prompt_ids: List[int]
    params: SamplingParams
    output_ids: List[int] = field(default_factory=list)
    logprobs: List[float] = field(default_factory=list)
    text: str = ""
    finished: bool = False
    finish_reason: Optional[str] = None
    arrival: float = 0.0
    first_token_time: Optional[float] = None
    finish_time: Optional[float] = None
    seed: int = 0
    on_token: Optional[Callable[["Request", str], None]] = None
    detok: Optional[IncrementalDetokenizer] = None
    cached_prefix: int = 0
    error: Optional[str] = None    # finish_reason "error": why the engine refused the request
    beams: List[tuple] = field(default_factory=list)   # beam search: (score, token ids, text)
    json_state: Optional[object] = None    # _rt.JsonState of a response_format=json_object request
    # multimodal prompt: (position, features [n, hidden]) — rows whose input embeddings are
    # replaced by projected image features (models/vision.py)
    mm: Optional[list] = None
    _hs: Optional[bool] = field(default=None, repr=False, compare=False)

    @property
    def host_sampling(self) -> bool:
        """Sampling needs host state between steps (penalty history, JSON grammar). Fixed once
        the request is queued (``json_state`` is set in ``add_request``), so it is computed
        once: the step loop asks it for every row several times per step."""
        hs = self._hs
        if hs is None:
            p = self.params
            hs = self._hs = bool(p.repetition_penalty != 1.0 or p.frequency_penalty or p.presence_penalty
                                 or self.json_state is not None)
        return hs

    @property
    def ttft(self) -> Optional[float]:
        return None if self.first_token_time is None else self.first_token_time - self.arrival

    @property
    def latency(self) -> Optional[float]:
        return None if self.finish_time is None else self.finish_time - self.arrival


@dataclass
class EngineConfig:
    model: str = "llama3-8b"
    max_num_seqs: int = 256
    max_batched_tokens: int = 16384
    max_model_len: int = 8192
    block_size: int = 64
    kv_cache_fraction: float = 0.3
    kv_cache_blocks: Optional[int] = None
    enable_prefix_caching: bool = True
    use_graphs: bool = True
    graph_batch_sizes: Sequence[int] = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 224, 256)
    decode_pages_per_part: Optional[int] = None  # None: adapt the KV split to the batch
    seed: int = 0
    detokenize: bool = True
    async_decode: bool = True  # pipeline steps (host work overlaps the GPU)
    mixed_prefill_tokens: int = 4096  # prefill tokens that ride along a decode step (0 = off)
    token_alignment: int = 256   # prefill/mixed steps carry a multiple of this many tokens
    mixed_min_tokens: int = 0     # accumulate this many prompt tokens before a mixed step ...
    mixed_max_wait: int = 4       # ... unless the oldest waiting request waited this many steps
    tuned_gemms: bool = True   # load the per-shape hipBLASLt/rocBLAS table (ops/gemm_tuning.py)
    sequence_parallel: bool = False  # TP prefill >= sp_min_tokens: reduce-scatter/all-gather
    fp8: bool = False   # W8A8 FP8 projections (LlamaModel.quantize_fp8)
    kv_cache_dtype: str = "auto"   # "fp8": e4m3fn KV pages (2x the cached tokens, half the KV reads)
    kv_scales: Tuple[float, float] = (1.0, 1.0)   # fp8 KV: the per-tensor K / V scales
    sp_min_tokens: int = 512
    # prefill / mixed steps as hipGraphs, one per (token bucket, decode-row bucket), captured
    # on first use: the whole step (embedding, every layer, LM head, sampling) is one launch,
    # with the step's layout in device buffers (work-list prefill attention, decode rows
    # past the step's own skipped); graph_eager runs the same body without capture (tests)
    mixed_graphs: bool = True
    graph_eager: bool = False
    graph_token_step: int = 256
    max_graph_tokens: int = 0     # 0: mixed_prefill_tokens + max_num_seqs, rounded up
    # numerics checks: every step's fp32 logits of its sampling rows are copied (before
    # sampling, inside captured graphs too) to ``LLMEngine.d_tap`` for ``step_hook``
    logits_tap: bool = False


_INERT = Request(id=-1, prompt_ids=[0], params=SamplingParams(temperature=0.0))


class LLMEngine(ReplicaMixin, StepGraphMixin):
    def __init__(self, cfg: EngineConfig = EngineConfig(), device: Optional[str] = None,
                 pctx: Optional[ParallelContext] = None, model: Optional[LlamaModel] = None,
                 tokenizer: Optional[LLMTokenizer] = None, model_cfg: Optional[LlamaConfig] = None,
                 weights: Optional[dict] = None):
        self.cfg = cfg
        self.p = pctx or get_context()
        if device is None:
            device = str(self.p.device) if self.p.device.type == "cuda" else (
                "cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        self.mcfg = model_cfg or llama_config(cfg.model, max_position=max(cfg.max_model_len, 256))
        self.model = model or LlamaModel(self.mcfg, self.device, pctx=self.p, seed=cfg.seed,
                                         weights=weights, fp8=cfg.fp8)
        if cfg.fp8 and not self.model.fp8:
            self.model.quantize_fp8()
        self.model.sequence_parallel = cfg.sequence_parallel
        self.model.sp_min_tokens = cfg.sp_min_tokens
        self.tok = tokenizer or llm_tokenizer()
        self.stop_ids = set(self.tok.stop_ids) | set(self.mcfg.eos_ids)
        self.gpu = self.device.type == "cuda"
        if self.gpu and cfg.tuned_gemms:
            from ..ops.gemm_tuning import use_tuned_gemms

            self.tuned_gemms = use_tuned_gemms()
        # ---- KV cache
        nb = cfg.kv_cache_blocks
        if nb is None:
            if self.gpu:
                free, _ = torch.cuda.mem_get_info(self.device)
                nb = int(free * cfg.kv_cache_fraction) // self.model.kv_block_bytes(cfg.block_size,
                                                                                    cfg.kv_cache_dtype)
            else:
                nb = 256
        self.num_blocks = int(nb)
        self.model.allocate_kv_cache(self.num_blocks, cfg.block_size, cfg.kv_cache_dtype, cfg.kv_scales)
        self.max_blocks = (cfg.max_model_len + cfg.block_size - 1) // cfg.block_size
        self.sched = rt.Scheduler(self.num_blocks, cfg.block_size, cfg.max_num_seqs,
                                  cfg.max_batched_tokens, cfg.max_model_len,
                                  cfg.enable_prefix_caching)
        self.sched.set_mixed_prefill_tokens(cfg.mixed_prefill_tokens)
        self.sched.set_token_alignment(cfg.token_alignment)
        self.sched.set_mixed_min_tokens(cfg.mixed_min_tokens, cfg.mixed_max_wait)
        # ---- host step buffers (pinned) filled by the native scheduler
        pin = self.gpu
        T, S = max(cfg.max_batched_tokens, cfg.max_num_seqs), cfg.max_num_seqs

        def hbuf(*shape, dtype=torch.int32):
            return torch.zeros(*shape, dtype=dtype, pin_memory=pin)

        self.h_ids, self.h_pos, self.h_slots = hbuf(T), hbuf(T), hbuf(T)
        self.h_cu, self.h_ctx = hbuf(S + 1), hbuf(S)
        self.h_bt = hbuf(S, self.max_blocks)
        self.h_sid = hbuf(S, dtype=torch.int64)
        self.h_smp = hbuf(S)
        self.h_temp = hbuf(S, dtype=torch.float32)
        self.h_topk = hbuf(S)
        self.h_topp = hbuf(S, dtype=torch.float32)
        self.h_seed = hbuf(S, dtype=torch.int64)
        self.h_step = hbuf(S, dtype=torch.int64)
        self.h_pen = hbuf(S, dtype=torch.float32)
        self._np = [b.numpy() for b in (self.h_ids, self.h_pos, self.h_slots, self.h_cu,
                                         self.h_ctx, self.h_bt, self.h_sid, self.h_smp)]
        (self.n_temp, self.n_topk, self.n_topp, self.n_seed, self.n_step, self.n_pen) = (
            b.numpy() for b in (self.h_temp, self.h_topk, self.h_topp, self.h_seed, self.h_step, self.h_pen))
        dev = self.device

        def dbuf(*shape, dtype=torch.int32):
            return torch.zeros(*shape, dtype=dtype, device=dev)

        self.d_ids, self.d_pos, self.d_slots = dbuf(T), dbuf(T), dbuf(T)
        self.d_cu, self.d_ctx = dbuf(S + 1), dbuf(S)
        self.d_bt = dbuf(S, self.max_blocks)
        self.d_temp = dbuf(S, dtype=torch.float32)
        self.d_topk = dbuf(S)
        self.d_topp = dbuf(S, dtype=torch.float32)
        self.d_seed = dbuf(S, dtype=torch.int64)
        self.d_step = dbuf(S, dtype=torch.int64)
        self.d_pen = dbuf(S, dtype=torch.float32)
        self.d_tok = dbuf(S)
        self.d_lp = dbuf(S, dtype=torch.float32)
        self.d_tap = dbuf(S, self.mcfg.vocab_size, dtype=torch.float32) if cfg.logits_tap else None
        # synchronous steps: step_hook(engine, n, tokens) runs after each step with the
        # sampled tokens of its n rows (d_tap holds their logits when logits_tap); a returned
        # list replaces the tokens (teacher forcing: later steps consume the forced ids)
        self.step_hook: Optional[Callable[["LLMEngine", int, List[int]], Optional[List[int]]]] = None
        self.decode_ws = ops.DecodeWorkspace(S, self.model.hq, self.model.hkv, cfg.max_model_len,
                                             dev, cfg.decode_pages_per_part, D=self.model.D,
                                             kv_fp8=cfg.kv_cache_dtype == "fp8") if self.gpu else None
        if self.gpu and self.mcfg.is_moe:
            # this engine's own routing buffers, sized for its largest step before any
            # hipGraph capture (graphs keep pointing at them for the engine's lifetime)
            self.model.moe_ws = ops.MoEWorkspace(max(T, 64), self.mcfg.experts_per_tok,
                                                 self.model.n_experts, dev)
        self.requests: Dict[int, Request] = {}
        self._has_mm = False   # any multimodal request seen (enables the embedding override pass)
        self._ids = itertools.count(1)
        self._rng = random.Random(cfg.seed)
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.stats = {"prefill_steps": 0, "decode_steps": 0, "mixed_steps": 0, "prefill_tokens": 0,
                      "decode_tokens": 0, "prefill_time": 0.0, "decode_time": 0.0, "unpipelined_steps": 0,
                      "host_sched_s": 0.0, "host_launch_s": 0.0, "host_between_s": 0.0,
                      "host_wait_s": 0.0, "host_finalize_s": 0.0, "graph_steps": 0, "graph_captures": 0,
                      "graph_capture_s": 0.0}
        self.lock = threading.RLock()
        self._inbox: "collections.deque" = collections.deque()   # requests queued while a step held the lock
        self._live_ids: set = set()       # ids queued or running (duplicates refused in add_request)
        self._rejected: List[Request] = []   # refused at admission, reported by the next step()
        self._pending: Optional[dict] = None
        self._tok_flip = 0
        self._up_ev = None  # marks the last host->device upload of the pinned step buffers
        # host-side timestamps of recent pipelined steps: (enter, schedule start, launch start,
        # launch end, between end, wait end, exit) — where the host spends a step (bench.py)
        self._host_steps: Deque[tuple] = collections.deque(maxlen=4096)
        # optional GPU-side step timing (events at each launched step's start and end):
        # ``gpu_step_timing()`` splits the GPU timeline into in-step time and idle gaps
        # between steps
        self.step_timing = False
        self._step_events: Deque[tuple] = collections.deque(maxlen=8192)
        self._timeline = collections.deque(maxlen=4096)
        self._tok_host = [(hbuf(S), hbuf(S, dtype=torch.float32)) for _ in range(2)]
        # pinned staging of the pipelined id gather (token index, row of the in-flight step):
        # a pageable host->device copy is staged synchronously by the HIP runtime and can
        # hold the launching thread while the GPU drains the previous step
        self.h_gidx, self.h_gprev = hbuf(T, dtype=torch.int64), hbuf(T, dtype=torch.int64)
        self.d_gidx = dbuf(T, dtype=torch.int64) if self.gpu else None
        self.d_gprev = dbuf(T, dtype=torch.int64) if self.gpu else None
        self._step_reqs: List[Request] = []
        self._step_host = (-1, False)   # (rows, any needs host sampling) of the current step
        self._faults = FaultInjector(rank=self.p.rank)   # NGA_FAULT (utils/faults.py)
        self._nstep = 0
        self._beam_of: Dict[int, BeamGroup] = {}   # live beam seq id -> its group
        self._beam_rows: List[tuple] = []         # (row, seq id) of beam rows in this step
        self._beam_out = None
        self._chan = None
        self._msg = None
        self._tp_gathers = 0    # follower steps that gathered ids from their own previous step
        self._follower_launch: Deque[float] = collections.deque(maxlen=8192)   # receipt -> launched (s)
        self._launch_t0 = None
        if self.p.mp_size > 1:
            # the replica's step channel: followers rebuild every step from the driver's layout
            # (shared memory on one node: publishing never waits for the driver's GPU, so
            # steps pipeline exactly as on one rank — each follower gathers the ids the
            # in-flight step is still producing from its OWN sampled tokens, which equal the
            # driver's: same gathered logits, same per-row seeds)
            from ..parallel import step_channel

            nbytes = self._step_msg_bytes(T, S)
            self._msg = np.zeros(nbytes, dtype=np.uint8)
            self._chan = step_channel.create(self.p, nbytes)
            over = {}
            if not self._chan.pipelined or self.p.pp_size > 1:
                # a collective channel stages the layout through the driver's stream, and pipeline
                # stages exchange activations with p2p sends: such replicas step synchronously
                over["async_decode"] = False
            if self.p.pp_size > 1:
                over["use_graphs"] = False   # stage-to-stage sends stay out of hipGraphs
            elif self.gpu and not self.model.ipc_collectives_cover(S, S):
                # a graph holds only the IPC collectives: gloo's host-copy collectives cannot be
                # captured, and RCCL inside a capture (a custom all-reduce that failed its
                # self-test) is a path no test has executed, so both replay eagerly
                over["use_graphs"] = False
            if over:
                self.cfg = cfg = type(cfg)(**{**cfg.__dict__, **over})
        # ---- prefill / mixed step graphs (step layout in device buffers)
        self.mgraphs: Dict[tuple, torch.cuda.CUDAGraph] = {}
        # step-graph launches by token bucket and by real token count (128-token bins):
        # which GEMM sizes a workload actually runs (bench.py reports them)
        self.bucket_hist: collections.Counter = collections.Counter()
        self.ntok_hist: collections.Counter = collections.Counter()
        self._graph_pool = None
        self._cap_stream = None
        self._mg_ok = self._mixed_graphs_eligible()
        if self._mg_ok:   # (may turn False below: collectives the graphs could not hold)
            step = max(1, cfg.graph_token_step)
            mx = cfg.max_graph_tokens or (cfg.mixed_prefill_tokens + cfg.max_num_seqs)
            self._mg_max_tokens = min(-(-mx // step) * step, T // step * step)
            if self.p.mp_size > 1 and not self.model.ipc_collectives_cover(S, self._mg_max_tokens):
                self._mg_ok = False
            self._nd_buckets = sorted({b for b in (8, 16, 32, 64, 128, 256, 512) if b < S} | {S})
            cap = self._mg_max_tokens // 32 + S + 16     # >= row blocks (32 or 64 rows) of any step
            self.h_ctxd, self.d_ctxd = hbuf(S), dbuf(S)
            self.h_sidx, self.d_sidx = hbuf(S, dtype=torch.int64), dbuf(S, dtype=torch.int64)
            self.h_items, self.d_items = hbuf(cap, 2), dbuf(cap, 2)
            self.h_nitems, self.d_nitems = hbuf(1), dbuf(1)
        # every step's inputs in one pinned -> device copy + one scatter kernel (ops/staging.py)
        self._stager = None
        self._staged_src = None
        if self.gpu and os.environ.get("NGA_PACKED_UPLOAD", "1") != "0":   # 0: per-buffer copies (A/B)
            from ..ops.staging import PackedUpload

            bufs = [self.h_ids, self.h_pos, self.h_slots, self.h_cu, self.h_ctx, self.h_bt, self.h_temp,
                    self.h_topk, self.h_topp, self.h_seed, self.h_step, self.h_pen, self.h_gidx, self.h_gprev]
            if self._mg_ok:
                bufs += [self.h_ctxd, self.h_items, self.h_nitems, self.h_sidx]
            self._stager = PackedUpload(self.device, sum(b.numel() * b.element_size() + 16 for b in bufs))
        if self.gpu and cfg.use_graphs:
            self._capture_graphs()

    # ------------------------------------------------------------------ requests
    def apply_chat_template(self, messages, add_generation_prompt: bool = True) -> List[int]:
        """Prompt ids of a chat in this model family's format (``LlamaConfig.chat_format``)."""
        return self.tok.apply_chat_template(messages, add_generation_prompt,
                                            fmt=self.mcfg.chat_format)

    def add_request(self, prompt_ids: List[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[int] = None,
                    on_token: Optional[Callable[[Request, str], None]] = None,
                    mm: Optional[list] = None) -> Request:
        """Queue a request. ``mm``: [(position, features [n, hidden])] — the prompt rows
        [position, position + n) take these embeddings instead of their token ids' (image
        placeholders of a vision-language prompt)."""
        params = params or SamplingParams()
        V = self.mcfg.vocab_size
        if prompt_ids and (max(prompt_ids) >= V or min(prompt_ids) < 0):
            if not getattr(self.tok, "synthetic", False) or min(prompt_ids) < 0:
                raise ValueError(f"prompt token ids outside the model's vocabulary [0, {V}): "
                                 "tokenizer / model mismatch")
            # the synthetic tokenizer's id space (32768) exceeds a few real vocabularies
            # (32000): fold, as detokenisation folds sampled ids the other way
            prompt_ids = [t % V for t in prompt_ids]
        if mm:
            if self.p.mp_size > 1:
                raise ValueError("multimodal requests run on single-rank engines")
            for off, f in mm:
                if off < 0 or off + f.shape[0] > len(prompt_ids) or f.shape[1] != self.mcfg.hidden:
                    raise ValueError("multimodal features must cover prompt rows of the model's hidden size")
        if not prompt_ids:
            raise ValueError("empty prompt")
        rid = request_id if request_id is not None else next(self._ids)
        # what the scheduler would refuse at admission is refused here, before the request
        # can wait in the inbox (a step admits the inbox: a failure there is not the caller's)
        if rid in self._live_ids:
            raise ValueError(f"duplicate request id {rid}")
        max_new = max(1, min(params.max_tokens, self.cfg.max_model_len - len(prompt_ids)))
        if len(prompt_ids) >= self.cfg.max_model_len:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens exceeds max_model_len "
                             f"{self.cfg.max_model_len}")
        req = Request(rid, list(prompt_ids), params, arrival=time.perf_counter(),
                      seed=params.seed if params.seed is not None else self._rng.getrandbits(62),
                      on_token=on_token,
                      mm=[(int(o), f.to(self.device, self.model.dtype)) for o, f in mm] if mm else None)
        req.params = SamplingParams(**{**params.__dict__, "max_tokens": max_new})
        if self.cfg.detokenize:
            req.detok = IncrementalDetokenizer(self.tok)
        if mm:
            self._has_mm = True
        if params.response_format == "json_object":
            self._grammar()
            req.json_state = rt.JsonState(True)
        elif params.response_format not in (None, "text"):
            raise ValueError(f"unsupported response_format {params.response_format!r}")
        # A step holds the engine lock for its whole duration (GPU wait included). A producer
        # thread must not queue behind it: when the lock is busy the request goes to the
        # inbox, which the next step admits first (same order, no lost wake-ups).
        self._live_ids.add(rid)
        if self.lock.acquire(blocking=False):
            try:
                self._rejected += self._admit_inbox()   # earlier arrivals first
                try:
                    self._admit_one(req, max_new)
                except Exception:
                    self._live_ids.discard(rid)
                    raise
            finally:
                self.lock.release()
        else:
            self._inbox.append((req, max_new))
        return req

    def _admit_one(self, req: Request, max_new: int):
        rid, params = req.id, req.params
        self.sched.add(rid, req.prompt_ids, max_new)
        if params.beam_width > 1:
            g = BeamGroup(req, int(params.beam_width), float(params.length_penalty))
            g.beams[rid] = 0.0
            self._beam_of[rid] = g
        else:
            self.requests[rid] = req

    def _admit_inbox(self) -> List[Request]:
        """Admit the queued requests in arrival order; one that the scheduler refuses finishes
        alone with finish_reason "error" (its stream ends with the message), the others and the
        step go on. Returns the refused ones."""
        bad = []
        while self._inbox:
            req, max_new = self._inbox.popleft()
            try:
                self._admit_one(req, max_new)
            except Exception as e:  # noqa: BLE001 - this request's failure, not the step's
                self._live_ids.discard(req.id)
                req.finished, req.finish_reason, req.error = True, "error", str(e)
                req.finish_time = time.perf_counter()
                if req.on_token is not None:
                    try:
                        req.on_token(req, "")
                    except Exception:  # noqa: BLE001
                        log.exception("on_token callback failed")
                bad.append(req)
        return bad

    def abort(self, rid: int):
        with self.lock:
            self._rejected += self._admit_inbox()
            req = self.requests.pop(rid, None)
            self.sched.finish(rid)
            self._live_ids.discard(rid)
            g = next((g for g in set(self._beam_of.values()) if g.req.id == rid), None)
            if g is not None:
                req = g.req
                for sid in g.beams:
                    self.sched.finish(sid)
                    self._beam_of.pop(sid, None)
                g.beams = {}
            if req is not None and not req.finished:
                req.finished, req.finish_reason = True, "abort"
                req.finish_time = time.perf_counter()

    def has_work(self) -> bool:
        return bool(self._inbox) or self.sched.has_work()

    # ------------------------------------------------------------------ step
    def _fill_params(self, reqs, pending_ids=()):
        """Per-row sampling parameters. A row whose request finished while its step was being
        settled (None) samples greedily and is ignored."""
        if any(r is None for r in reqs):
            reqs = [r if r is not None else _INERT for r in reqs]
        n = len(reqs)
        self.n_temp[:n] = [r.params.temperature for r in reqs]
        self.n_topk[:n] = [r.params.top_k for r in reqs]
        self.n_topp[:n] = [r.params.top_p for r in reqs]
        self.n_seed[:n] = [r.seed for r in reqs]
        self.n_step[:n] = [len(r.output_ids) + (r.id in pending_ids) for r in reqs]
        self.n_pen[:n] = [r.params.repetition_penalty for r in reqs]
        self._step_reqs = reqs
        self._step_host = (n, any(r.host_sampling for r in reqs))

    def step(self, between: Optional[Callable[[], None]] = None) -> List[Request]:
        """Run one scheduler step; returns requests that finished in it.

        ``between`` (optional) runs after the next step has been launched and before the
        host blocks on the previous step's tokens — the window where the GPU is busy and the
        host would otherwise wait. A serving loop puts its own host work there (building
        prompts for finished retrievals, launching the next retrieval batch), so that work
        never delays the launch of the following step.

        Steps are pipelined when possible: step k+1 is scheduled and launched before step k's
        tokens are read back (input ids that step k is still producing are gathered on the
        GPU from its output), so host work — reading tokens, detokenising, stop checks,
        scheduling — overlaps the GPU instead of serialising with it. With mixed batching
        (``mixed_prefill_tokens``) a step carries the decode rows of every running sequence
        plus a prefill chunk, so decode rows ride on the prefill GEMMs."""
        with self.lock:
            done = self._admit_inbox()
            if self._rejected:
                done, self._rejected = self._rejected + done, []
            self._nstep += 1
            if self._faults:
                self._faults.check(self._nstep, "driver")
            done += self._step(between)
        return done

    def _step(self, between) -> List[Request]:
        t_enter = time.perf_counter()
        pend = self._pending
        done: List[Request] = []
        if pend is not None:
            cont = [r.id for r, s in zip(pend["reqs"], pend["smp"]) if s and r is not None
                    and len(r.output_ids) + 1 < r.params.max_tokens and r.id in self.requests]
            self.sched.append_placeholders(cont)
        ids, pos, sl, cu, ctx, bt, sid, smp = self._np
        if self._up_ev is not None:
            # the in-flight step's upload may still be queued behind the GPU's previous
            # step: the pinned buffers must not be rewritten before the DMA has read them
            self._up_ev.synchronize()
        t_sched = time.perf_counter()
        kind, n, ntok = self.sched.schedule(ids, pos, sl, cu, ctx, bt, sid, smp)
        nd = n if kind == 2 else (self.sched.last_num_decode() if kind == 3 else 0)
        if _KV_SHARE_STATS and nd:   # diagnostics: KV pages the decode rows share (prefix cache)
            nb = (ctx[:nd] + 63) // 64
            refs = np.concatenate([bt[i, :nb[i]] for i in range(nd)])
            self.stats["kv_page_refs"] = self.stats.get("kv_page_refs", 0) + int(refs.size)
            self.stats["kv_pages_unique"] = self.stats.get("kv_pages_unique", 0) + int(np.unique(refs).size)
        src = None
        sids = sid[:n].tolist()
        # rows that need the host between steps (penalty history, beam candidates) run the
        # step synchronously
        sync_rows = (self._needs_penalty_reqs([self.requests.get(int(s)) for s in sids])
                     or (bool(self._beam_of) and any(int(s) in self._beam_of for s in sids)))
        if pend is not None:
            ph = np.flatnonzero(ids[:ntok] < 0) if kind else np.empty(0, dtype=np.int64)
            rows = pend["rows"]
            ok = (kind != 0 and self.cfg.async_decode and not self._needs_penalty_reqs(pend["reqs"])
                  and not sync_rows
                  and all(i < nd and int(sid[i]) in rows for i in ph.tolist()))
            if ok:
                src = (ph, [rows[int(sid[i])] for i in ph.tolist()])
            else:
                # cannot pipeline: settle the in-flight step, then run this one normally (with
                # nothing left to schedule, kind 0, this is just the end-of-work drain)
                if kind != 0:
                    self.stats["unpipelined_steps"] += 1
                done += self._finalize(pend)
                pend = self._pending = None
                for i in ph.tolist():
                    r = int(np.searchsorted(cu[1:n + 1], i, side="right"))
                    try:
                        ids[i] = self.sched.tokens(int(sid[r]))[pos[i]]
                    except (IndexError, KeyError):  # finished meanwhile: row is inert
                        ids[i] = 0
        if kind == 0:
            if between is not None:
                between()
            return done
        t0 = time.perf_counter()
        reqs = [self.requests.get(int(s)) for s in sid[:n].tolist()]
        pending_ids = pend["sampled"] if pend is not None else ()
        self._fill_params(reqs, pending_ids=pending_ids)
        key = "decode_time" if kind == 2 else "prefill_time"
        self._count(kind, n, ntok, nd)
        self._beam_rows = ([(i, int(s)) for i, s in enumerate(sids) if int(s) in self._beam_of]
                           if self._beam_of else [])
        if self.cfg.async_decode and not sync_rows and not self._needs_penalty(n):
            h0 = time.perf_counter()
            nxt = self._launch(kind, n, ntok, nd, src)
            h1 = time.perf_counter()
            if between is not None:
                between()
            h2 = h3 = time.perf_counter()
            if pend is not None:
                if pend["ev"] is not None:
                    pend["ev"].synchronize()
                h3 = time.perf_counter()
                done += self._finalize(pend)
                self.stats["host_wait_s"] += h3 - h2
                self.stats["host_finalize_s"] += time.perf_counter() - h3
            self.stats["host_launch_s"] += h1 - h0
            self.stats["host_between_s"] += h2 - h1
            self.stats["host_sched_s"] += h0 - t_sched
            self._host_steps.append((t_enter, t_sched, h0, h1, h2, h3, time.perf_counter()))
            self._pending = nxt
            self.stats[key] += time.perf_counter() - t0
            return done
        if kind == 2:
            toks, lps = self._decode(n)
        else:
            toks, lps = self._prefill(n, ntok, nd)
        toks = toks.tolist()
        lps = lps.tolist()
        if self.step_hook is not None:
            toks = self.step_hook(self, n, toks) or toks
        self.stats[key] += time.perf_counter() - t0
        now = time.perf_counter()
        for i, (r, s) in enumerate(zip(reqs, smp[:n].tolist())):
            if s and r is not None and not r.finished and self._emit(r, toks[i], lps[i], now):
                done.append(r)
        if self._beam_rows:
            done += self._beam_step(smp[:n].tolist(), now)
        if between is not None:
            between()
        return done

    def gpu_step_timing(self) -> dict:
        """From the step events (``step_timing = True``): total ms the GPU spent inside
        steps (first upload to last token copy), total ms of gaps between consecutive steps
        (the GPU had finished a step before the next one's first command ran), and the
        largest gap."""
        evs = list(self._step_events)
        if not evs:
            return {}
        torch.cuda.synchronize()
        inside = sum(a.elapsed_time(b) for a, b in evs)
        gaps = [max(0.0, evs[i - 1][1].elapsed_time(evs[i][0])) for i in range(1, len(evs))]
        span = evs[0][0].elapsed_time(evs[-1][1])
        return {"steps": len(evs), "span_ms": round(span, 1), "in_step_ms": round(inside, 1),
                "between_steps_ms": round(sum(gaps), 1), "max_gap_ms": round(max(gaps, default=0.0), 2),
                "gaps_over_1ms": sum(1 for g in gaps if g > 1.0)}

    def timeline(self, last: int = 256) -> List[dict]:
        """Recent scheduler steps: wall time at launch, kind, rows, tokens, decode rows and
        the host time spent in ``step()`` (the engine step-timeline of SURVEY.md §5.1)."""
        return list(self._timeline)[-last:]

    def _count(self, kind, n, ntok, nd):
        self._timeline.append({"t": time.time(), "kind": "decode" if kind == 2 else ("mixed" if nd else "prefill"),
                               "rows": n, "tokens": ntok, "decode_rows": nd,
                               "waiting": self.sched.num_waiting(), "running": self.sched.num_running()})
        if kind == 2:
            self.stats["decode_steps"] += 1
            self.stats["decode_tokens"] += n
        else:
            self.stats["prefill_steps"] += 1
            self.stats["prefill_tokens"] += ntok - nd
            if nd:
                self.stats["mixed_steps"] += 1
                self.stats["decode_tokens"] += nd

    def _needs_penalty_reqs(self, reqs) -> bool:
        """Rows whose sampling needs host state (penalty history, JSON grammar)."""
        return any(r is not None and r.host_sampling for r in reqs)

    def _launch(self, kind: int, n: int, ntok: int, nd: int, src) -> dict:
        """Launch a step without waiting for it. ``src = (token_idx, prev_rows)`` gathers the
        input ids the previous in-flight step is still producing from its device output.
        Tokens are copied to pinned host memory right after sampling, so the next step may
        overwrite the device buffers."""
        t_ev = None
        if self.gpu and self.step_timing:
            t_ev = torch.cuda.Event(enable_timing=True)
            t_ev.record()
        if kind == 2:
            with gpu_range(f"decode n={n}"):
                self._decode_launch(n, src)
        else:
            cu = self._np[3][: n + 1]
            max_q = int((cu[1:] - cu[:-1]).max())
            max_ctx = int(self._np[4][:n].max())
            key = self._graph_key(n, ntok, nd)
            with gpu_range(f"{'mixed' if nd else 'prefill'} n={n} tok={ntok} dec={nd}"
                           + (" graph" if key is not None else "")):
                if key is not None:
                    self._graph_step(key, kind, n, ntok, max_q, max_ctx, nd, src)
                else:
                    self._sync_step(kind, n, ntok, max_q, max_ctx, 0, nd, src=src)
                    self._upload(n, ntok, src=src)
                    self._gather_ids(src)
                    logits = self._prefill_forward(n, ntok, max_q, max_ctx, nd)
                    self._sample(logits, n)
        buf = self._tok_host[self._tok_flip]
        self._tok_flip ^= 1
        buf[0][:n].copy_(self.d_tok[:n], non_blocking=self.gpu)
        buf[1][:n].copy_(self.d_lp[:n], non_blocking=self.gpu)
        ev = None
        if self.gpu:
            ev = torch.cuda.Event(enable_timing=t_ev is not None)
            ev.record()
            if t_ev is not None:
                self._step_events.append((t_ev, ev))
        reqs = [self.requests.get(int(s)) for s in self._np[6][:n].tolist()]
        smp = self._np[7][:n].tolist()
        return {"reqs": reqs, "smp": smp, "rows": {int(s): i for i, s in enumerate(self._np[6][:n].tolist())},
                "sampled": {r.id for r, m in zip(reqs, smp) if m and r is not None},
                "n": n, "buf": buf, "ev": ev}

    def _stage_gather(self, src):
        """Device copies of the gather's (token index, previous row) lists, uploaded from the
        pinned staging buffers; the upload event then covers them too. Lists that the step's
        packed upload already carried (``_upload(..., src=src)``) are not copied again."""
        k = len(src[0])
        if src is self._staged_src:
            return (self.d_gidx[:k], self.d_gprev[:k]) if self.gpu else (self.h_gidx[:k], self.h_gprev[:k])
        self.h_gidx.numpy()[:k] = src[0]
        self.h_gprev.numpy()[:k] = src[1]
        if not self.gpu:
            return self.h_gidx[:k], self.h_gprev[:k]
        self.d_gidx[:k].copy_(self.h_gidx[:k], non_blocking=True)
        self.d_gprev[:k].copy_(self.h_gprev[:k], non_blocking=True)
        self._up_ev = torch.cuda.Event()
        self._up_ev.record()
        return self.d_gidx[:k], self.d_gprev[:k]

    def _gather_ids(self, src) -> None:
        if src is None or len(src[0]) == 0:
            return
        idx, prev = self._stage_gather(src)
        self.d_ids.index_copy_(0, idx, self.d_tok.index_select(0, prev))

    def _decode_launch(self, n: int, src) -> None:
        """Replay the decode graph for n rows (padded to the captured bucket)."""
        bs = next((b for b in sorted(self.graphs) if b >= n), None)
        if bs is not None:
            self._pad_rows(n, bs)
        self._sync_step(2, n, n, 1, self.cfg.max_model_len, bs or 0, src=src)
        self._upload(bs or n, bs or n, src=src)
        self._apply_decode_src(n, src)
        if bs is not None:
            self.graphs[bs].replay()
        else:
            meta = self._meta("decode", n, n, 1, self.cfg.max_model_len)
            logits = self.model.logits(self.model.forward(self.d_ids[:n], self.d_pos[:n], meta))
            self._sample(logits, n)

    def _pad_rows(self, n: int, bs: int) -> None:
        """Padding rows of a graph bucket: no cache write, empty context, greedy."""
        self.h_slots[n:bs] = -1
        self.h_ctx[n:bs] = 0
        self.h_ids[n:bs] = 0
        self.h_pos[n:bs] = 0
        self.h_temp[n:bs] = 0.0
        self.h_topk[n:bs] = 0
        self.h_topp[n:bs] = 1.0
        self.h_step[n:bs] = 0
        self.h_seed[n:bs] = 0

    def _finalize(self, pend: dict) -> List[Request]:
        if pend["ev"] is not None:
            pend["ev"].synchronize()
        n = pend["n"]
        toks = pend["buf"][0][:n].tolist()
        lps = pend["buf"][1][:n].tolist()
        now = time.perf_counter()
        done = []
        for r, s, t, lp in zip(pend["reqs"], pend["smp"], toks, lps):
            if not s or r is None or r.finished:
                continue
            had = self.sched.has_placeholder(r.id)
            if had:
                self.sched.set_last_token(r.id, t)
            if self._emit(r, t, lp, now, appended=had):
                done.append(r)
        return done

    def drain_and_run(self, fn):
        """Run ``fn()`` with no step in flight (the pipelined step is settled first; requests
        it finishes still get their callbacks)."""
        with self.lock:
            if self._pending is not None:
                pend, self._pending = self._pending, None
                self._finalize(pend)
            return fn()

    def drain(self) -> List[Request]:
        """Settle the in-flight pipelined step (if any)."""
        with self.lock:
            if self._pending is None:
                return []
            pend, self._pending = self._pending, None
            return self._finalize(pend)

    # ------------------------------------------------------------------ beam search
    def _beam_step(self, smp: List[int], now: float) -> List[Request]:
        """Record this step's top-2·width candidates of every beam row; advance each group
        whose live beams have all reported (engine/beam.py)."""
        vals, idxs = self._beam_out
        self._beam_out = None
        touched = []
        for k, (row, sid) in enumerate(self._beam_rows):
            g = self._beam_of.get(sid)
            if g is None or not smp[row]:
                continue
            w2 = 2 * g.width
            g.reported[sid] = (vals[k][:w2], idxs[k][:w2])
            if g not in touched:
                touched.append(g)
        self._beam_rows = []
        done, copies = [], []
        for g in touched:
            if set(g.reported) != set(g.beams):
                continue
            r = g.req
            if r.first_token_time is None:
                r.first_token_time = now
            old = list(g.beams)
            finished, cp, forked = advance(
                g, self.sched, len(r.prompt_ids),
                lambda t, r=r: (t in self.stop_ids and not r.params.ignore_eos) or t in r.params.stop_token_ids,
                r.params.min_tokens, r.params.max_tokens)
            copies += cp
            for sid in old:
                if sid not in g.beams:
                    self._beam_of.pop(sid, None)
            for sid in forked:
                self._beam_of[sid] = g
            if finished:
                self._beam_finish(g, now)
                done.append(r)
        if copies:
            src = torch.tensor([c[0] for c in copies], dtype=torch.int32)
            dst = torch.tensor([c[1] for c in copies], dtype=torch.int32)
            if self.p.mp_size > 1:
                self._sync_step(-2, len(copies), 0, 0, 0, 0, 0, pairs=torch.stack([src, dst]).numpy())
            self.model.copy_kv_blocks(src, dst)
        return done

    def _beam_finish(self, g: BeamGroup, now: float) -> None:
        r = g.req
        self._live_ids.discard(r.id)
        for score, toks, eos in g.hyps:
            text = self.tok.decode([t for t in toks if t not in self.stop_ids]) if self.cfg.detokenize else ""
            for s in r.params.stop:
                if s and s in text:
                    text = text[: text.index(s)]
            r.beams.append((score, toks, text))
        score, toks, eos = g.hyps[0] if g.hyps else (0.0, [], False)
        r.output_ids = list(toks)
        r.text = r.beams[0][2] if r.beams else ""
        r.finished, r.finish_reason, r.finish_time = True, ("stop" if eos else "length"), now
        if r.on_token is not None:
            try:
                if r.text:
                    r.on_token(r, r.text)
                r.on_token(r, "")
            except Exception:  # noqa: BLE001
                log.exception("on_token callback failed")

    def _emit(self, r: Request, tok: int, lp: float, now: float, appended: bool = False) -> bool:
        if r.first_token_time is None:
            r.first_token_time = now
            r.cached_prefix = self.sched.cached_prefix(r.id)
        r.output_ids.append(tok)
        if r.json_state is not None:
            self._json_grammar.advance(r.json_state, tok)
        if r.params.logprobs:
            r.logprobs.append(lp)
        if not appended:
            self.sched.append_token(r.id, tok)
        delta = ""
        n = len(r.output_ids)
        reason = None
        is_stop_tok = (tok in self.stop_ids and not r.params.ignore_eos) or tok in r.params.stop_token_ids
        if is_stop_tok and n > r.params.min_tokens:
            reason = "stop"
        elif r.detok is not None:
            delta = r.detok.push(tok)
            r.text += delta
            if r.params.stop:
                for s in r.params.stop:
                    idx = r.text.find(s, max(0, len(r.text) - len(delta) - len(s)))
                    if s and idx >= 0:
                        delta = delta[: max(0, len(delta) - (len(r.text) - idx))]
                        r.text = r.text[:idx]
                        reason = "stop"
                        break
        if reason is None and n >= r.params.max_tokens:
            reason = "length"
        if r.on_token is not None and (delta or reason):
            try:
                r.on_token(r, delta)
            except Exception:  # noqa: BLE001 - a consumer error must not kill the engine
                log.exception("on_token callback failed")
        if reason is not None:
            r.finished, r.finish_reason, r.finish_time = True, reason, now
            self.sched.finish(r.id)
            self.requests.pop(r.id, None)
            self._live_ids.discard(r.id)
            if r.on_token is not None:
                try:
                    r.on_token(r, "")
                except Exception:  # noqa: BLE001
                    log.exception("on_token callback failed")
            return True
        return False

    def _meta(self, kind, n, ntok, max_q, max_ctx, nd: int = 0) -> AttnMeta:
        m = AttnMeta(kind=kind, slots=self.d_slots[:ntok], cu_q=self.d_cu[: n + 1],
                     ctx_lens=self.d_ctx[:n], block_tables=self.d_bt[:n], max_q_len=max_q,
                     max_ctx=max_ctx, decode_ws=self.decode_ws)
        if nd:
            # mixed step: rows [0, nd) decode, the rest prefill with its own cu_seqlens
            m.kind, m.n_decode, m.max_ctx = "mixed", nd, self.cfg.max_model_len
            m.cu_q_prefill = self.d_cu[nd: n + 1] - nd
        return m

    def _upload(self, n, ntok, nparam: Optional[int] = None, extra=(), src=None):
        """Step buffers host -> device: ``ntok`` token rows, ``n`` sequence rows, ``nparam``
        (default n) sampling-parameter rows, ``extra`` (host, device, rows) triples and, with
        ``src``, the pipelined id gather's lists (then :meth:`_stage_gather` reuses them). On the
        GPU one packed copy + one scatter kernel (ops/staging.py); the host buffers may be
        rewritten as soon as this returns."""
        npr = n if nparam is None else nparam
        segs = [(self.h_ids, self.d_ids, ntok), (self.h_pos, self.d_pos, ntok), (self.h_slots, self.d_slots, ntok),
                (self.h_cu, self.d_cu, n + 1), (self.h_ctx, self.d_ctx, n), (self.h_bt, self.d_bt, n),
                (self.h_temp, self.d_temp, npr), (self.h_topk, self.d_topk, npr), (self.h_topp, self.d_topp, npr),
                (self.h_seed, self.d_seed, npr), (self.h_step, self.d_step, npr), (self.h_pen, self.d_pen, npr)]
        segs += list(extra)
        self._staged_src = None
        if src is not None and len(src[0]):
            k = len(src[0])
            self.h_gidx.numpy()[:k] = src[0]
            self.h_gprev.numpy()[:k] = src[1]
            if self.gpu:
                segs += [(self.h_gidx, self.d_gidx, k), (self.h_gprev, self.d_gprev, k)]
            self._staged_src = src
        if self._stager is not None:
            self._stager.upload(segs)
            return
        for h, d, rows in segs:
            d[:rows].copy_(h[:rows], non_blocking=self.gpu)

    def _tap(self, logits, rows: int) -> None:
        if self.d_tap is not None and logits is not None:
            self.d_tap[:rows].copy_(logits[:rows])

    def _sample(self, logits, n):
        self._tap(logits, n)
        if self._beam_rows and logits is not None:
            rows = torch.tensor([i for i, _ in self._beam_rows], device=logits.device)
            k = max(2 * self._beam_of[s].width for _, s in self._beam_rows)
            lp = torch.log_softmax(logits.index_select(0, rows).float(), dim=-1)
            v, ix = lp.topk(min(k, lp.shape[-1]), dim=-1)
            self._beam_out = (v.cpu().tolist(), ix.cpu().tolist())
        self._apply_count_penalties(logits, n)
        self._apply_json_masks(logits, n)
        rep = self.d_pen[:n] if self._needs_penalty(n) else None
        hist = self._history(n) if rep is not None else None
        tok, lp = ops.sample(logits, self.d_temp[:n], self.d_topk[:n], self.d_topp[:n],
                             self.d_seed[:n], self.d_step[:n], rep, hist,
                             out_tok=self.d_tok[:n], out_lp=self.d_lp[:n])
        if tok.data_ptr() != self.d_tok.data_ptr():   # reference path returns fresh tensors
            self.d_tok[:n].copy_(tok[:n])
            self.d_lp[:n].copy_(lp[:n])
        return self.d_tok[:n], self.d_lp[:n]

    def _needs_penalty(self, n) -> bool:
        """This step's rows need host-side sampling state; computed once per step by
        ``_fill_params`` (the rows' repetition penalties are in ``h_pen``)."""
        if n == self._step_host[0]:
            return self._step_host[1]
        return any(r.host_sampling for r in self._step_reqs[:n])

    def _grammar(self):
        g = getattr(self, "_json_grammar", None)
        if g is None:
            from ..utils.tokenizer import token_bytes_table

            g = self._json_grammar = rt.JsonGrammar(token_bytes_table(self.tok), sorted(self.stop_ids))
        return g

    def _apply_json_masks(self, logits, n) -> None:
        """response_format=json_object rows: logits of tokens the JSON grammar rejects from
        the row's state become -inf before the sampling kernel (json_grammar.cpp)."""
        if logits is None:
            return
        rows = [i for i, r in enumerate(self._step_reqs[:n]) if r.json_state is not None]
        if not rows:
            return
        V = logits.shape[1]
        m = np.zeros((len(rows), V), dtype=np.uint8)
        for k, i in enumerate(rows):
            self._json_grammar.fill_mask(self._step_reqs[i].json_state, m[k])
        idx = torch.tensor(rows, device=logits.device)
        bad = torch.from_numpy(m).to(logits.device) == 0
        logits.index_copy_(0, idx, logits.index_select(0, idx).masked_fill(bad, float("-inf")))

    def _apply_count_penalties(self, logits, n) -> None:
        """frequency/presence penalties (OpenAI /v1/completions semantics) on the rows that
        ask for them: a bincount of the row's generated tokens, subtracted in place."""
        if logits is None:
            return
        for i, r in enumerate(self._step_reqs[:n]):
            if not (r.params.frequency_penalty or r.params.presence_penalty) or not r.output_ids:
                continue
            cnt = torch.bincount(torch.tensor(r.output_ids, dtype=torch.int64),
                                 minlength=logits.shape[1])[: logits.shape[1]].to(logits.device)
            logits[i] -= (r.params.frequency_penalty * cnt
                          + r.params.presence_penalty * (cnt > 0)).to(logits.dtype)

    def _history(self, n):
        rows = [self.sched.tokens(int(self.h_sid[i])) for i in range(n)]
        L = max(len(r) for r in rows)
        h = torch.full((n, L), -1, dtype=torch.int32)
        for i, r in enumerate(rows):
            h[i, : len(r)] = torch.tensor(r, dtype=torch.int32)
        return h.to(self.device)

    def _prefill(self, n, ntok, nd: int = 0):
        """Synchronous prefill (nd = 0) or mixed step (rows [0, nd) decode)."""
        cu = self._np[3][: n + 1]
        max_q = int((cu[nd + 1:] - cu[nd:-1]).max())
        max_ctx = int(self._np[4][:n].max())
        key = None if (self._beam_rows or self._needs_penalty(n)) else self._graph_key(n, ntok, nd)
        if key is not None:
            self._graph_step(key, 3 if nd else 1, n, ntok, max_q, max_ctx, nd, None)
            return self.d_tok[:n].cpu(), self.d_lp[:n].cpu()
        self._sync_step(3 if nd else 1, n, ntok, max_q, max_ctx, 0, nd)
        self._upload(n, ntok)
        logits = self._prefill_forward(n, ntok, max_q, max_ctx, nd)
        tok, lp = self._sample(logits, n)
        return tok[:n].cpu(), lp[:n].cpu()

    def _mm_override(self, n: int, nd: int):
        """(token rows, features) of this step's prompt rows that carry image features."""
        rows, feats = [], []
        pos, cu, sid = self._np[1], self._np[3], self._np[6]
        for r in range(nd, n):
            req = self.requests.get(int(sid[r]))
            if req is None or not req.mm:
                continue
            t0, t1 = int(cu[r]), int(cu[r + 1])
            if t1 <= t0:
                continue
            p0 = int(pos[t0])
            p1 = p0 + (t1 - t0)
            for off, f in req.mm:
                lo, hi = max(off, p0), min(off + f.shape[0], p1)
                if lo < hi:
                    rows.append(torch.arange(t0 + lo - p0, t0 + hi - p0))
                    feats.append(f[lo - off:hi - off])
        if not rows:
            return None
        return torch.cat(rows).to(self.device, non_blocking=True), torch.cat(feats)

    def _prefill_forward(self, n, ntok, max_q, max_ctx, nd: int = 0):
        meta = self._meta("prefill", n, ntok, max_q, max_ctx, nd)
        sample_idx = (self.d_cu[1: n + 1] - 1).long()
        ov = self._mm_override(n, nd) if self._has_mm else None
        h = self.model.forward(self.d_ids[:ntok], self.d_pos[:ntok], meta, sample_idx,
                               embed_override=ov)
        return None if h is None else self.model.logits(h)   # None: a later pipeline stage

    def _decode(self, n):
        if self.graphs and not self._needs_penalty(n) and not self._beam_rows:
            bs = next((b for b in sorted(self.graphs) if b >= n), None)
            if bs is not None:
                self._pad_rows(n, bs)
                self._sync_step(2, n, n, 1, self.cfg.max_model_len, bs)
                self._upload(bs, bs)
                self.graphs[bs].replay()
                return self.d_tok[:n].cpu(), self.d_lp[:n].cpu()
        self._sync_step(2, n, n, 1, self.cfg.max_model_len, 0)
        logits = self._decode_eager(n)
        tok, lp = self._sample(logits, n)
        return tok[:n].cpu(), lp[:n].cpu()

    def _decode_eager(self, n):
        self._upload(n, n)
        meta = self._meta("decode", n, n, 1, self.cfg.max_model_len)
        h = self.model.forward(self.d_ids[:n], self.d_pos[:n], meta)
        return None if h is None else self.model.logits(h)

    def _decode_body(self, bs):
        meta = self._meta("decode", bs, bs, 1, self.cfg.max_model_len)
        h = self.model.forward(self.d_ids[:bs], self.d_pos[:bs], meta)
        logits = self.model.logits(h)
        self._tap(logits, bs)
        ops.sample(logits, self.d_temp[:bs], self.d_topk[:bs], self.d_topp[:bs],
                   self.d_seed[:bs], self.d_step[:bs], None, None,
                   out_tok=self.d_tok[:bs], out_lp=self.d_lp[:bs])

    # ------------------------------------------------------------------ convenience
    def run_until_done(self, reqs: Optional[List[Request]] = None) -> None:
        while self.has_work():
            self.step()
            if reqs is not None and all(r.finished for r in reqs):
                break

    def generate(self, prompts: List[List[int]], params: Optional[SamplingParams] = None) -> List[Request]:
        reqs = [self.add_request(p, params) for p in prompts]
        self.run_until_done(reqs)
        return reqs

    def kv_usage(self) -> float:
        return self.sched.used_blocks() / max(1, self.sched.total_blocks())
