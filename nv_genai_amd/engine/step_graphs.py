"""Prefill / mixed-step hipGraphs of :class:`~.llm_engine.LLMEngine`: every prefill or mixed
step replays a graph keyed by (token bucket, decode-row bucket), with the step layout in device
buffers (work-list prefill attention, decode attention on the bucket's first rows), captured
lazily on first use under ``utils.runtime.capture_guard`` and sharing the decode graphs' pool.
"""
from __future__ import annotations

import os
import sys
import time

import torch

from .. import ops
from ..models.llama import AttnMeta
from ..utils.runtime import capture_guard

_TRACE_CAPTURE = os.environ.get("NGA_TRACE_CAPTURE", "0") == "1"   # per-rank timings of lazy captures


class StepGraphMixin:
    # ------------------------------------------------------------------ prefill / mixed step graphs
    def _mixed_graphs_eligible(self) -> bool:
        """Graph-captured prefill / mixed steps need a work-list prefill kernel (the 32x32
        one for bf16 head_dim-128 pages with <= 1024 pages per sequence, else the 16x16 one
        for head_dim 64 / 128 / 256 and fp8 pages), one pipeline stage and the plain stacked
        forward (no sequence-parallel prefill, no split mixed steps, no MoE)."""
        c, m = self.cfg, self.model
        if not c.mixed_graphs or not (self.gpu and c.use_graphs or c.graph_eager):
            return False
        self._pf_impl = 2 if (m.D == 128 and m.kv_dtype == "auto" and self.max_blocks <= 1024) else 1
        self._pf_seq_min = int(os.environ.get("NGA_PF_SEQ_MIN", "384"))   # _graph_pf_seq; 0 = off
        return (self.p.pp_size == 1 and not c.sequence_parallel and not m.split_mixed and m.D in (64, 128, 256)
                and not self.mcfg.is_moe)

    def _graph_key(self, n: int, ntok: int, nd: int):
        """(token bucket, decode-row bucket) of a prefill / mixed step, or None (eager)."""
        if not self._mg_ok or self._has_mm or n > self.cfg.max_num_seqs:
            return None
        step = self.cfg.graph_token_step
        tb = -(-ntok // step) * step
        if tb > self._mg_max_tokens:
            return None
        ndb = 0 if nd == 0 else next(b for b in self._nd_buckets if b >= nd)
        # the decode launch covers the first ndb rows of the bucket (fine token steps: a
        # mostly-decode step can round to fewer tokens than its decode-row bucket)
        tb = max(tb, -(-ndb // step) * step)
        if tb > self._mg_max_tokens:
            return None
        return (tb, ndb)

    def _graph_kernel(self, key):
        """(impl, ks) of the work-list prefill kernel in the step graph of ``key``, by the
        eager size rule: the 32x32 kernel from ~1,024 row-block workgroups up (two per CU),
        else the 16x16 one — whose small LDS footprint also lets the decode attention of a
        mixed step share the CUs (the 32x32 kernel's 64-128 KiB per workgroup crowds it out).
        The 8-wave split-key form only for a lone prompt with no decode rows beside it."""
        tb, ndb = key
        if self._pf_impl != 2:
            return 1, 1
        if self._graph_pf_seq(key):
            return 2, 1
        G = self.model.hq // self.model.hkv
        hpw = 4 if G % 4 == 0 else 2 if G % 2 == 0 else 1
        items = (tb - ndb) // ops.prefill_rows_per_block(self.model.hq, self.model.hkv) * self.model.hkv * (G // hpw)
        if items >= 1024:
            return 2, 1
        if ndb == 0:   # no decode attention beside it: the standalone size rule (impl 4)
            return (2, 2) if items <= 320 else (2, 1)
        return 1, 1

    def _graph_pf_seq(self, key) -> bool:
        """Mixed steps with a large prefill (NGA_PF_SEQ_MIN <= work items < 1,024, decode rows
        beside it): the 32x32 prefill kernel after the decode attention instead of the 16x16
        one concurrently. Beside a 60-150 us prefill the decode kernel stretches from 229 to
        331 us (profiles/r3_prof_bins/attn_overlap.json)."""
        tb, ndb = key
        if self._pf_impl != 2 or ndb == 0 or self._pf_seq_min <= 0:
            return False
        G = self.model.hq // self.model.hkv
        hpw = 4 if G % 4 == 0 else 2 if G % 2 == 0 else 1
        items = (tb - ndb) // ops.prefill_rows_per_block(self.model.hq, self.model.hkv) * self.model.hkv * (G // hpw)
        return self._pf_seq_min <= items < 1024

    def _graph_meta(self, key) -> AttnMeta:
        tb, ndb = key
        impl, ks = self._graph_kernel(key)
        S = self.cfg.max_num_seqs
        return AttnMeta(kind="graph", slots=self.d_slots[:tb], cu_q=self.d_cu[: S + 1], ctx_lens=self.d_ctx[:S],
                        block_tables=self.d_bt[:S], max_q_len=0, max_ctx=self.cfg.max_model_len,
                        decode_ws=self.decode_ws, n_decode=ndb, decode_ctx=self.d_ctxd[:max(ndb, 1)],
                        items=self.d_items, n_items=self.d_nitems, pf_grid=256 if ks == 2 else 512, pf_ks=ks,
                        pf_impl=impl, pf_seq=self._graph_pf_seq(key))

    def _graph_body(self, key) -> None:
        """One prefill / mixed step over the bucket: forward of tb token rows, logits of the
        S = max_num_seqs sampling rows (d_sidx), sampling into d_tok / d_lp."""
        tb, _ = key
        S = self.cfg.max_num_seqs
        h = self.model.forward(self.d_ids[:tb], self.d_pos[:tb], self._graph_meta(key), self.d_sidx[:S])
        logits = self.model.logits(h)
        self._tap(logits, S)
        tok, lp = ops.sample(logits, self.d_temp[:S], self.d_topk[:S], self.d_topp[:S], self.d_seed[:S],
                             self.d_step[:S], None, None, out_tok=self.d_tok[:S], out_lp=self.d_lp[:S])
        if tok.data_ptr() != self.d_tok.data_ptr():   # reference path returns fresh tensors
            self.d_tok[:S].copy_(tok[:S])
            self.d_lp[:S].copy_(lp[:S])

    def _capture_step_graph(self, key) -> "torch.cuda.CUDAGraph":
        """Capture the step graph of ``key`` (first use). The device is drained first; the
        warm-up and capture run on inert inputs (no KV writes or reads: slots -1, no decode
        rows, an empty work list) and the sampled tokens of the step in flight are kept."""
        tb, ndb = key
        dev = self.device
        t0 = time.perf_counter()
        trace = _TRACE_CAPTURE and (lambda m: print(f"[capture rank{self.p.rank} {key}] {m} "
                                                    f"+{time.perf_counter() - t0:.3f}s", file=sys.stderr, flush=True))
        torch.cuda.synchronize(dev)
        if trace:
            trace("drained")
        keep = (self.d_tok.clone(), self.d_lp.clone())
        self.d_ids[:tb].zero_()
        self.d_pos[:tb].zero_()
        self.d_slots[:tb].fill_(-1)
        self.d_ctxd.zero_()
        self.d_nitems.zero_()
        self.d_sidx.zero_()
        if self._cap_stream is None:
            self._cap_stream = torch.cuda.Stream(dev)
        stream = self._cap_stream
        stream.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(stream):
            self._graph_body(key)
            if trace:
                stream.synchronize()
                trace("warm-up done")
            g = torch.cuda.CUDAGraph()
            with capture_guard(), torch.cuda.graph(g, pool=self._graph_pool, stream=stream,
                                                   capture_error_mode="thread_local"):
                self._graph_body(key)
        torch.cuda.current_stream(dev).wait_stream(stream)
        torch.cuda.synchronize(dev)
        if trace:
            trace("captured")
        self._graph_pool = g.pool()
        self.d_tok.copy_(keep[0])
        self.d_lp.copy_(keep[1])
        self.mgraphs[key] = g
        self.stats["graph_captures"] += 1
        self.stats["graph_capture_s"] += time.perf_counter() - t0
        return g

    def _graph_step(self, key, kind, n, ntok, max_q, max_ctx, nd, src, follower: bool = False) -> None:
        """Launch a prefill / mixed step through its graph: pad the token rows to the bucket,
        fill the step's device layout (decode-row contexts, prefill work list, sampling rows
        and parameters), upload, gather pipelined ids, replay."""
        tb, ndb = key
        S = self.cfg.max_num_seqs
        if not follower:
            self.h_ids[ntok:tb] = 0
            self.h_pos[ntok:tb] = 0
            self.h_slots[ntok:tb] = -1
        cu, ctx = self._np[3], self._np[4]
        self.h_ctxd[:nd] = self.h_ctx[:nd]
        self.h_ctxd[nd:max(ndb, nd)] = 0
        items = ops.plan_prefill_items(cu, ctx, nd, n, self.model.hq, self.model.hkv, self.model.window,
                                       out=self.h_items.numpy(),
                                       rw=ops.worklist_rows(self._graph_kernel(key)[0], self.model.hq,
                                                            self.model.hkv))
        self.h_nitems[0] = len(items)
        sidx = self.h_sidx.numpy()
        sidx[:n] = cu[1:n + 1] - 1
        sidx[n:S] = 0
        self._pad_params(n, S)
        if not follower:
            self._sync_step(kind, n, ntok, max_q, max_ctx, 0, nd, gb=tb, src=src)
        # lazy capture only after the step header and payload went out: under TP the warm-up
        # and captured forwards issue all-reduces, which the followers (blocked in _recv_step
        # until the broadcast) must meet in the same order. The capture leaves the host-side
        # step layout alone and the upload below refills every device input it zeroed.
        g = self.mgraphs.get(key)
        if g is None and self.gpu and not self.cfg.graph_eager:
            g = self._capture_step_graph(key)
        self._upload(n, tb, nparam=S, extra=((self.h_ctxd, self.d_ctxd, max(ndb, 1)),
                                             (self.h_items, self.d_items, max(len(items), 1)),
                                             (self.h_nitems, self.d_nitems, 1), (self.h_sidx, self.d_sidx, S)),
                     src=src)
        self._gather_ids(src)
        self.stats["graph_steps"] += 1
        self.bucket_hist[tb] += 1
        self.ntok_hist[ntok // 128 * 128] += 1
        if g is not None:
            g.replay()
        else:
            self._graph_body(key)

    def _pad_params(self, n: int, rows: int) -> None:
        """Sampling-parameter rows [n, rows) of a padded launch: greedy, no penalty."""
        self.h_temp[n:rows] = 0.0
        self.h_topk[n:rows] = 0
        self.h_topp[n:rows] = 1.0
        self.h_seed[n:rows] = 0
        self.h_step[n:rows] = 0
        self.h_pen[n:rows] = 1.0

    def _capture_graphs(self):
        sizes = [b for b in self.cfg.graph_batch_sizes if b <= self.cfg.max_num_seqs]
        # inert inputs for capture: no cache writes, empty contexts
        self.d_slots.fill_(-1)
        self.d_ctx.zero_()
        self.d_temp.zero_()
        self.d_topp.fill_(1.0)
        pool = None
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream):
            for bs in sorted(sizes, reverse=True):
                for _ in range(2):
                    self._decode_body(bs)
                g = torch.cuda.CUDAGraph()
                # thread_local: other threads of a serving process (retrieval, embeddings, other
                # engines) keep launching on their own streams while this one captures
                with capture_guard(), torch.cuda.graph(g, pool=pool, stream=stream,
                                                       capture_error_mode="thread_local"):
                    self._decode_body(bs)
                pool = g.pool()
                self.graphs[bs] = g
        self._graph_pool = pool     # step graphs captured later share the pool
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
