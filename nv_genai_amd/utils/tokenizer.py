"""Tokenizers for the random-init models.

No model hub is reachable, so the framework trains its own tokenizers once, from the
deterministic synthetic corpus, with HF ``tokenizers`` and caches them under
``nv_genai_amd/assets/``:

* ``llm_tokenizer.json`` — byte-level BPE (32768 ids) with the Llama-3 chat special tokens
  (<|begin_of_text|>, <|start_header_id|>, <|end_header_id|>, <|eot_id|>, <|end_of_text|>);
* ``embed_tokenizer.json`` — BERT WordPiece (30522 ids, [CLS]/[SEP]/[PAD]/[UNK]/[MASK]).

The LLM's embedding / LM-head keep the real Llama-3 vocabulary (128256 rows): ids the
tokenizer never emits are valid model inputs, and sampled ids >= the tokenizer size are
folded into range for detokenisation (weights are random, text is synthetic either way).
"""
from __future__ import annotations

import os
import threading
from functools import lru_cache
from pathlib import Path
from typing import Iterable, List, Optional

from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

from .synthetic import corpus

ASSETS = Path(__file__).resolve().parent.parent / "assets"
LLM_SPECIALS = ["<|begin_of_text|>", "<|end_of_text|>", "<|start_header_id|>",
                "<|end_header_id|>", "<|eot_id|>"]
BERT_SPECIALS = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
_LOCK = threading.Lock()


def _train_corpus() -> Iterable[str]:
    return corpus(3000, seed=7)


def _build_llm(path: Path, vocab: int = 32768) -> Tokenizer:
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab, special_tokens=LLM_SPECIALS,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet(),
                             show_progress=False)
    tok.train_from_iterator(_train_corpus(), tr)
    path.parent.mkdir(parents=True, exist_ok=True)
    tok.save(str(path))
    return tok


def _build_bert(path: Path, vocab: int = 30522) -> Tokenizer:
    tok = Tokenizer(models.WordPiece(unk_token="[UNK]"))
    tok.normalizer = normalizers.BertNormalizer(lowercase=True)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.decoder = decoders.WordPiece()
    tr = trainers.WordPieceTrainer(vocab_size=vocab, special_tokens=BERT_SPECIALS,
                                   show_progress=False)
    tok.train_from_iterator(_train_corpus(), tr)
    cls, sep = tok.token_to_id("[CLS]"), tok.token_to_id("[SEP]")
    tok.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
        special_tokens=[("[CLS]", cls), ("[SEP]", sep)])
    path.parent.mkdir(parents=True, exist_ok=True)
    tok.save(str(path))
    return tok


class LLMTokenizer:
    """Text <-> ids plus the Llama-3 chat template."""

    def __init__(self, tok: Optional[Tokenizer] = None):
        # the bundled synthetic vocabulary (random-init benchmarks): its id space may exceed
        # a small model's vocabulary, and the engine folds such ids instead of refusing them
        self.synthetic = tok is None
        if tok is None:
            p = ASSETS / "llm_tokenizer.json"
            with _LOCK:
                tok = Tokenizer.from_file(str(p)) if p.exists() else _build_llm(p)
        self.tok = tok
        self.n = tok.get_vocab_size()
        self.bos_id = tok.token_to_id("<|begin_of_text|>")
        self.eot_id = tok.token_to_id("<|eot_id|>")
        self.eos_id = tok.token_to_id("<|end_of_text|>")
        self.header_start = tok.token_to_id("<|start_header_id|>")
        self.header_end = tok.token_to_id("<|end_header_id|>")

    @property
    def stop_ids(self):
        return (self.eot_id, self.eos_id)

    def encode(self, text: str) -> List[int]:
        if len(text) > 512:
            # the Rust tokenizer's batch entry point runs without the GIL (the single-text one
            # holds it): a serving process's event loop and engine thread keep running while a
            # prompt of a few thousand characters is encoded on a worker thread
            return self.tok.encode_batch([text], add_special_tokens=False)[0].ids
        return self.tok.encode(text, add_special_tokens=False).ids

    def encode_batch(self, texts: List[str]) -> List[List[int]]:
        return [e.ids for e in self.tok.encode_batch(texts, add_special_tokens=False)]

    def decode(self, ids: List[int], skip_special: bool = True) -> str:
        ids = [i % self.n for i in ids]
        return self.tok.decode(ids, skip_special_tokens=skip_special)

    def apply_chat_template(self, messages: List[dict], add_generation_prompt: bool = True,
                            fmt: str = "llama3") -> List[int]:
        """Render a chat in the model family's prompt format:

        * ``llama3``: <|begin_of_text|><|start_header_id|>role<|end_header_id|>\n\ncontent<|eot_id|>...
        * ``mistral``: <s>[INST] (system\n\n)user [/INST] assistant</s>[INST] ... — the
          template of the reference's Mistral NIM config (experimental/fm-asr-streaming-rag/
          nim/configs/mistral-7b.yaml:15-17: system folded into the first user turn);
        * ``gemma``: <bos><start_of_turn>user\ncontent<end_of_turn>\n<start_of_turn>model\n
          (no system role: it is folded into the first user turn, as Gemma's template does);
        * ``plain``: ``role: content`` lines (base / code models such as StarCoder2).

        BOS/EOS are this tokenizer's <|begin_of_text|> / <|eot_id|> (synthetic vocabulary)."""
        if fmt == "llama3":
            ids = [self.bos_id]
            for m in messages:
                ids.append(self.header_start)
                ids += self.encode(m.get("role", "user"))
                ids.append(self.header_end)
                ids += self.encode("\n\n" + str(m.get("content", "")))
                ids.append(self.eot_id)
            if add_generation_prompt:
                ids.append(self.header_start)
                ids += self.encode("assistant")
                ids.append(self.header_end)
                ids += self.encode("\n\n")
            return ids
        msgs = [dict(m) for m in messages]
        system = ""
        if msgs and msgs[0].get("role") == "system":
            system = str(msgs.pop(0).get("content", "")).strip() + "\n\n"
        if fmt == "mistral":
            ids = [self.bos_id]
            first = True
            for m in msgs:
                c = str(m.get("content", "")).strip()
                if m.get("role") == "user":
                    ids += self.encode("[INST] " + (system + c if first else c) + " [/INST]")
                    first = False
                elif m.get("role") == "assistant":
                    ids += self.encode(" " + c + " ")
                    ids.append(self.eot_id)
            return ids
        if fmt == "gemma":
            ids = [self.bos_id]
            first = True
            for m in msgs:
                role = "model" if m.get("role") == "assistant" else "user"
                c = str(m.get("content", "")).strip()
                if role == "user" and first:
                    c, first = system + c, False
                ids += self.encode(f"<start_of_turn>{role}\n{c}<end_of_turn>\n")
            if add_generation_prompt:
                ids += self.encode("<start_of_turn>model\n")
            return ids
        if fmt == "plain":
            text = system + "".join(f"{m.get('role', 'user')}: {m.get('content', '')}\n" for m in msgs)
            if add_generation_prompt:
                text += "assistant: "
            return [self.bos_id] + self.encode(text)
        raise ValueError(f"unknown chat format {fmt!r}")


def _byte_decoder() -> dict:
    """Inverse of the GPT-2 byte-level alphabet (printable stand-ins for the 256 bytes)."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return {chr(c): b for b, c in zip(bs, cs)}


class IncrementalDetokenizer:
    """Streams text for a growing id list at O(1) per token: every id maps to its raw bytes
    (precomputed once per tokenizer from the byte-level vocabulary) and an incremental UTF-8
    decoder emits only complete characters — no re-decoding of a window per token."""

    def __init__(self, tok: LLMTokenizer, prompt_tail: Optional[List[int]] = None):
        import codecs

        self.tok = tok
        self.table = token_bytes_table(tok)
        self.dec = codecs.getincrementaldecoder("utf-8")(errors="replace")

    def push(self, tid: int) -> str:
        b = self.table[tid % len(self.table)]
        return self.dec.decode(b) if b else ""


_TABLES: dict = {}


def token_bytes_table(tok: LLMTokenizer) -> List[bytes]:
    t = _TABLES.get(id(tok))
    if t is None:
        inv = _byte_decoder()
        specials = {tok.bos_id, tok.eot_id, tok.eos_id, tok.header_start, tok.header_end}
        t = []
        for i in range(tok.n):
            s = tok.tok.id_to_token(i)
            if s is None or i in specials:
                t.append(b"")
            else:
                t.append(bytes(inv.get(ch, 32) for ch in s))
        _TABLES[id(tok)] = t
    return t


class EmbedTokenizer:
    def __init__(self, tok: Optional[Tokenizer] = None, max_len: int = 512):
        if tok is None:
            p = ASSETS / "embed_tokenizer.json"
            with _LOCK:
                tok = Tokenizer.from_file(str(p)) if p.exists() else _build_bert(p)
        self.tok = tok
        self.max_len = max_len
        self.cls_id = tok.token_to_id("[CLS]")
        self.sep_id = tok.token_to_id("[SEP]")

    def encode(self, text: str, truncate: str = "END") -> List[int]:
        ids = self.tok.encode(text).ids
        return self._trunc(ids, truncate)

    def encode_batch(self, texts: List[str], truncate: str = "END") -> List[List[int]]:
        return [self._trunc(e.ids, truncate) for e in self.tok.encode_batch(texts)]

    def encode_pair(self, a: str, b: str, truncate: str = "END") -> List[int]:
        return self._trunc(self.tok.encode(a, b).ids, truncate)

    def _trunc(self, ids: List[int], truncate: str) -> List[int]:
        if len(ids) <= self.max_len:
            return ids
        t = (truncate or "NONE").upper()
        if t == "END":
            return ids[: self.max_len - 1] + [self.sep_id]
        if t == "START":
            return [self.cls_id] + ids[-(self.max_len - 1):]
        raise ValueError(f"input of {len(ids)} tokens exceeds {self.max_len} and truncate=NONE")

    def count(self, text: str) -> int:
        return len(self.tok.encode(text).ids)


@lru_cache(maxsize=1)
def llm_tokenizer() -> LLMTokenizer:
    return LLMTokenizer()


@lru_cache(maxsize=1)
def embed_tokenizer() -> EmbedTokenizer:
    return EmbedTokenizer()
