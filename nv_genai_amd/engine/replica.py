"""Model-parallel replica plumbing of :class:`~.llm_engine.LLMEngine` (SURVEY.md §2.D CC5,
§2.E TP / PP): the driver publishes every step's layout to the replica's followers over the
step channel (``parallel/step_channel.py``: shared memory on one node, a process-group
broadcast otherwise), followers rebuild and replay the same step, and non-step commands
(sharded searches, barriers, copy-on-fork pages) travel in the same ordered stream so the
collectives inside them line up on every rank.

The reference's TP engine hides this inside TensorRT-LLM's in-flight batching with
``tensor_para_size`` (experimental/fm-asr-streaming-rag/nim/configs/mistral-7b.yaml:26-39).
"""
from __future__ import annotations

import time
from typing import Callable, Dict, Optional

import numpy as np
import torch

from .. import ops


class ReplicaMixin:
    # ------------------------------------------------------------------ model parallel
    # The replica's driver (pipeline stage 0, TP rank 0) schedules, then broadcasts the step
    # layout (one int32 payload over RCCL) to every rank of the replica (tp x pp) so they
    # all run the same forward; the collectives inside the model (row-parallel all-reduces,
    # vocab all-gather, stage-to-stage sends) then line up. Followers loop in
    # run_follower() until the driver broadcasts a stop header.
    @property
    def is_driver(self) -> bool:
        return self.p.mp_size == 1 or (self.p.tp_rank == 0 and self.p.pp_rank == 0)

    _HDR = 12   # int64 header: kind, n, ntok, max_q, max_ctx, bs, nd, gb, nsrc, prow, npairs, 0

    def _step_msg_bytes(self, T: int, S: int) -> int:
        """Largest step message: header, token rows (ids / positions / slots), sequence rows
        (cu_seqlens, contexts, block tables), S rows of sampling parameters and a pipelined
        id gather over every token row."""
        return (8 * self._HDR + 4 * (3 * T + (S + 1) + S + S * self.max_blocks) + 8
                + S * (4 + 4 + 4 + 8 + 8) + 16 * T + 64)

    def _sync_step(self, kind: int, n: int, ntok: int, max_q: int, max_ctx: int, bs: int, nd: int = 0,
                   gb: int = 0, src=None, pairs=None, payload=None) -> None:
        """Driver: publish a step (or a command, kind < 0) to the replica's ranks. ``gb``: token
        bucket of a graph-captured prefill / mixed step (its padded token rows travel too, so
        followers replay the same graph on the same inputs); ``src``: the pipelined id gather
        (token rows, rows of the in-flight step) — every follower applies it to its own sampled
        tokens; the sampling parameters travel so followers sample exactly what the driver
        samples. ``pairs``: [2, k] copy-on-fork pages (kind -2); ``payload``: a command's bytes
        (kind <= -3; their count travels in the pairs field)."""
        if self.p.mp_size == 1:
            return
        rows, toks = max(n, bs), max(ntok, bs, gb)
        prow = max(rows, self.cfg.max_num_seqs if gb else 0) if kind >= 0 else 0
        nsrc = 0 if src is None else len(src[0])
        npairs = int(payload.size) if payload is not None else (0 if pairs is None else int(pairs.shape[1]))
        m = self._msg
        m[:8 * self._HDR].view(np.int64)[:] = (kind, n, ntok, max_q, max_ctx, bs, nd, gb, nsrc, prow, npairs, 0)
        o = 8 * self._HDR

        def put(a):
            nonlocal o
            b = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
            m[o:o + b.size] = b
            o += b.size

        if kind >= 0:
            ids, pos, sl, cu, ctx, bt = self._np[:6]
            for a in (ids[:toks], pos[:toks], sl[:toks], cu[:rows + 1], ctx[:rows], bt[:rows]):
                put(a)
            o = (o + 7) & ~7
            for a in (self.n_temp, self.n_topk, self.n_topp, self.n_seed, self.n_step):
                put(a[:prow])
            if nsrc:
                put(np.asarray(src[0], dtype=np.int64))
                put(np.asarray(src[1], dtype=np.int64))
        elif payload is not None:
            put(payload)
        elif npairs:
            put(np.asarray(pairs, dtype=np.int32))
        self._chan.send(m[:o])

    def _recv_step(self):
        """Follower: the next message into the host step buffers. Returns (kind, n, ntok, max_q,
        max_ctx, bs, nd, gb, src, pairs)."""
        msg = self._chan.recv()
        hdr = msg[:8 * self._HDR].view(np.int64).tolist()
        kind, n, ntok, max_q, max_ctx, bs, nd, gb, nsrc, prow, npairs, _ = hdr
        o = 8 * self._HDR

        def take(dtype, count):
            nonlocal o
            nb = np.dtype(dtype).itemsize * count
            a = msg[o:o + nb].view(dtype)
            o += nb
            return a

        if kind < 0:
            if kind <= -3:   # a command: its payload bytes (or None)
                pairs = take(np.uint8, npairs).copy() if npairs else None
            else:
                pairs = take(np.int32, 2 * npairs).reshape(2, npairs).copy() if npairs else None
            return kind, n, 0, 0, 0, 0, 0, 0, None, pairs
        rows, toks = max(n, bs), max(ntok, bs, gb)
        if self._up_ev is not None:
            # the previous step's upload may still be reading the pinned buffers
            self._up_ev.synchronize()
        ids, pos, sl, cu, ctx, bt = self._np[:6]
        ids[:toks] = take(np.int32, toks)
        pos[:toks] = take(np.int32, toks)
        sl[:toks] = take(np.int32, toks)
        cu[:rows + 1] = take(np.int32, rows + 1)
        ctx[:rows] = take(np.int32, rows)
        bt[:rows] = take(np.int32, rows * self.max_blocks).reshape(rows, self.max_blocks)
        o = (o + 7) & ~7
        self.n_temp[:prow] = take(np.float32, prow)
        self.n_topk[:prow] = take(np.int32, prow)
        self.n_topp[:prow] = take(np.float32, prow)
        self.n_seed[:prow] = take(np.int64, prow)
        self.n_step[:prow] = take(np.int64, prow)
        self.n_pen[:prow] = 1.0
        src = None
        if nsrc:
            src = (take(np.int64, nsrc).copy(), take(np.int64, nsrc).copy())
        return kind, n, ntok, max_q, max_ctx, bs, nd, gb, src, None

    def _apply_decode_src(self, n: int, src) -> None:
        """Pipelined decode: input ids of rows still being produced by the in-flight step."""
        if src is not None and len(src[0]) == n:
            _, prev = self._stage_gather(src)
            self.d_ids[:n] = self.d_tok.index_select(0, prev)
        else:
            self._gather_ids(src)

    def _follower_sample(self, logits, n: int) -> None:
        """Sample the step's rows exactly as the driver does (same logits after the vocab
        all-gather, same per-row temperature / top-k / top-p / seed / step), so the next
        pipelined step's id gather reads the same tokens on every rank."""
        if logits is None:   # a pipeline stage without the LM head
            return
        tok, lp = ops.sample(logits, self.d_temp[:n], self.d_topk[:n], self.d_topp[:n],
                             self.d_seed[:n], self.d_step[:n], None, None,
                             out_tok=self.d_tok[:n], out_lp=self.d_lp[:n])
        if tok.data_ptr() != self.d_tok.data_ptr():   # reference path returns fresh tensors
            self.d_tok[:n].copy_(tok[:n])
            self.d_lp[:n].copy_(lp[:n])

    def run_follower(self, hooks: Optional[Dict[int, Callable[[int], None]]] = None) -> None:
        """Non-driver TP ranks: execute every step the driver publishes, and the hook for
        each command kind (<= -3) it broadcasts (``broadcast_command``)."""
        while True:
            if self._launch_t0 is not None:
                self._follower_launch.append(time.perf_counter() - self._launch_t0)
                self._launch_t0 = None
            kind, n, ntok, max_q, max_ctx, bs, nd, gb, src, pairs = self._recv_step()
            self._launch_t0 = time.perf_counter() if kind >= 0 else None
            self._nstep += 1
            if self._faults:
                self._faults.check(self._nstep, "follower")
            if kind <= -3:
                if not hooks or kind not in hooks:
                    raise RuntimeError(f"follower has no hook for command {kind}")
                if pairs is None:
                    hooks[kind](n)
                else:          # the command's payload bytes
                    hooks[kind](n, pairs)
                continue
            if kind == -2:   # copy-on-fork pages (beam search)
                self.model.copy_kv_blocks(torch.from_numpy(pairs[0]), torch.from_numpy(pairs[1]))
                continue
            if kind < 0:
                return
            if src is not None:
                self._tp_gathers += 1
            prow = max(n, bs, self.cfg.max_num_seqs if gb else 0)
            if kind in (1, 3) and gb:
                key = self._graph_key(n, ntok, nd)
                if key is None or key[0] != gb:
                    raise RuntimeError(f"follower cannot replay the driver's step graph {gb}")
                self._graph_step(key, kind, n, ntok, max_q, max_ctx, nd, src, follower=True)
            elif kind in (1, 3):
                self._upload(n, ntok, src=src)
                self._gather_ids(src)
                self._follower_sample(self._prefill_forward(n, ntok, max_q, max_ctx, nd), n)
            elif bs:
                self._upload(bs, bs, nparam=prow, src=src)
                self._apply_decode_src(n, src)
                self.graphs[bs].replay()
            else:
                self._upload(n, n, src=src)
                self._apply_decode_src(n, src)
                meta = self._meta("decode", n, n, 1, self.cfg.max_model_len)
                h = self.model.forward(self.d_ids[:n], self.d_pos[:n], meta)
                self._follower_sample(None if h is None else self.model.logits(h), n)

    def follower_stats(self) -> dict:
        """Follower of a model-parallel replica: the step channel's publish -> receipt latency
        (µs percentiles, and how many waits ended spinning / yielding / after a futex sleep)
        and the host time from a step's receipt to the end of its launch (µs percentiles)."""
        v = sorted(self._follower_launch)
        out = {"channel": self._chan.stats() if self._chan is not None else {}}
        if v:
            out["receipt_to_launched_us"] = {q: round(1e6 * v[min(len(v) - 1, int(f * (len(v) - 1)))], 1)
                                             for q, f in (("p50", 0.5), ("p99", 0.99), ("max", 1.0))}
            out["steps"] = len(v)
        return out

    def stop_followers(self) -> None:
        if self.p.mp_size > 1 and self.is_driver:
            self._sync_step(-1, 0, 0, 0, 0, 0, 0)


    def broadcast_command(self, kind: int, n: int = 0, payload: Optional[np.ndarray] = None) -> None:
        """Driver of a model-parallel replica: announce a non-step command (kind <= -3) to
        the followers, which run the hook registered for it in :meth:`run_follower` —
        the same ordered channel as the step layouts, so collectives line up. ``payload``: host
        bytes that travel inside the message (e.g. a sharded search's query block, so the
        search needs no broadcast collective); the hook receives them as a uint8 array."""
        if kind > -3:
            raise ValueError("command kinds are <= -3 (-1 stop, -2 copy-on-fork are reserved)")
        if self.p.mp_size > 1:
            pl = None
            if payload is not None:
                pl = np.ascontiguousarray(payload).view(np.uint8).reshape(-1)
                if 8 * self._HDR + pl.size > self._msg.size:
                    raise ValueError(f"command payload of {pl.size} B exceeds the step message slot")
            self._sync_step(kind, n, 0, 0, 0, 0, 0, payload=pl)

    def command_payload_capacity(self) -> int:
        """Largest ``broadcast_command`` payload in bytes (0 on a single-rank engine)."""
        return 0 if self._msg is None else int(self._msg.size - 8 * self._HDR)
