"""Beam search over the paged KV cache (the ``beam_width`` / ``length_penalty`` knobs of the
TRT-LLM ensemble the reference drives: experimental/AzureML/trt_llm_azureml.py:282-320,
SURVEY.md §2.B N1, K9 copy-on-fork).

Each live beam is a scheduler sequence, so beams ride in the same continuous batch as
sampled requests. A group advances one token once every live beam has reported the top
``2·width`` log-probs of its last position:

* candidates ``score(beam) + logp(token)`` are ranked over all beams;
* a stop token among the top ``width`` candidates closes a hypothesis, scored
  ``sum_logprobs / generated_len ** length_penalty``;
* the best ``width`` non-stop candidates become the next beams. A beam with several children
  keeps its sequence for the first and forks for the rest: the native scheduler shares the
  full KV pages (reference counts) and the engine copies only the partially filled last
  page (``LlamaModel.copy_kv_blocks``); beams with no children are freed.

The group finishes when ``width`` hypotheses exist and no live beam can still beat the
worst of them, or at ``max_tokens`` (live beams then join the hypotheses).
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field
from typing import Dict, List, Tuple

_internal_ids = itertools.count(1 << 40)   # forked beams never collide with request ids


@dataclass(eq=False)
class BeamGroup:
    req: object                      # the user-visible Request (its id is the root beam)
    width: int
    length_penalty: float
    beams: Dict[int, float] = field(default_factory=dict)   # live seq id -> sum logprob
    reported: Dict[int, Tuple[List[float], List[int]]] = field(default_factory=dict)
    hyps: List[Tuple[float, List[int], bool]] = field(default_factory=list)  # (score, toks, eos)
    gen_len: int = 0

    def norm(self, score: float, length: int) -> float:
        return score / (max(1, length) ** self.length_penalty)

    def add_hyp(self, score: float, toks: List[int], eos: bool) -> None:
        self.hyps.append((self.norm(score, len(toks)), toks, eos))
        self.hyps.sort(key=lambda h: -h[0])
        del self.hyps[self.width:]

    def is_done(self, best_live: float, cur_len: int) -> bool:
        if len(self.hyps) < self.width:
            return False
        return self.norm(best_live, cur_len) <= self.hyps[-1][0]


def advance(group: BeamGroup, sched, prompt_len: int, is_stop, min_tokens: int,
            max_tokens: int) -> Tuple[bool, List[Tuple[int, int]], List[int]]:
    """One beam-search step for a group whose live beams all reported.

    Returns ``(finished, kv_copies, new_seq_ids)``: ``kv_copies`` are (src, dst) page pairs
    the caller must copy before the next forward, ``new_seq_ids`` the forked sequences."""
    cur_len = group.gen_len + 1
    cands = []
    for sid, (vals, idxs) in group.reported.items():
        base = group.beams[sid]
        cands.extend((base + v, sid, t) for v, t in zip(vals, idxs))
    cands.sort(key=lambda c: -c[0])
    nxt: List[Tuple[float, int, int]] = []
    for rank, (score, sid, t) in enumerate(cands):
        if is_stop(t) and cur_len > min_tokens:
            if rank < group.width:
                gen = sched.tokens(sid)[prompt_len:]
                group.add_hyp(score, gen + [t], True)
            continue
        nxt.append((score, sid, t))
        if len(nxt) == group.width:
            break
    group.reported = {}
    live_done = not nxt or cur_len >= max_tokens or group.is_done(nxt[0][0], cur_len)
    if live_done:
        if cur_len >= max_tokens or len(group.hyps) < group.width:
            for score, sid, t in nxt:
                group.add_hyp(score, sched.tokens(sid)[prompt_len:] + [t], False)
        for sid in group.beams:
            sched.finish(sid)
        group.beams = {}
        return True, [], []
    children: Dict[int, List[Tuple[float, int]]] = {}
    for score, sid, t in nxt:
        children.setdefault(sid, []).append((score, t))
    for sid in list(group.beams):
        if sid not in children:
            sched.finish(sid)
    copies, forked, assign = [], [], []
    for sid, lst in children.items():
        for k, (score, t) in enumerate(lst):
            target = sid
            if k:
                target = next(_internal_ids)
                src, dst = sched.fork(sid, target)
                if src >= 0:
                    copies.append((src, dst))
                forked.append(target)
            assign.append((target, score, t))
    for target, _, t in assign:       # after every fork: children copy the parent's tokens
        sched.append_token(target, t)
    group.beams = {target: score for target, score, _ in assign}
    group.gen_len = cur_len
    return False, copies, forked
