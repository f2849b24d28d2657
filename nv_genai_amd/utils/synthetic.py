"""Deterministic synthetic corpora (no datasets are reachable from this environment).

Documents are pseudo-English prose over a fixed generated lexicon, with Zipf-distributed
word frequencies and occasional "facts" (entity / attribute / value sentences) so retrieval
and QA plumbing has something to match on. Everything is a pure function of the seed.
"""
from __future__ import annotations

import random
from typing import List, Tuple

_ONSETS = ["b", "c", "d", "f", "g", "h", "j", "k", "l", "m", "n", "p", "r", "s", "t", "v",
           "w", "z", "br", "ch", "cl", "dr", "fl", "gr", "pl", "pr", "sh", "st", "th", "tr"]
_VOWELS = ["a", "e", "i", "o", "u", "ai", "ea", "io", "ou", "y"]
_CODAS = ["", "", "n", "r", "s", "t", "l", "m", "nd", "st", "ck", "ng"]
_FUNCTION = ["the", "of", "and", "to", "in", "is", "that", "for", "it", "as", "was", "with",
             "on", "by", "this", "are", "from", "at", "which", "be", "or", "an", "can", "has"]


def lexicon(n: int = 6000, seed: int = 1234) -> List[str]:
    rng = random.Random(seed)
    words, seen = [], set(_FUNCTION)
    words.extend(_FUNCTION)
    while len(words) < n:
        k = rng.choice((1, 2, 2, 3, 3, 4))
        w = "".join(rng.choice(_ONSETS) + rng.choice(_VOWELS) + rng.choice(_CODAS) for _ in range(k))
        if w not in seen:
            seen.add(w)
            words.append(w)
    return words


class TextGen:
    def __init__(self, seed: int = 0, vocab: int = 6000):
        self.rng = random.Random(seed)
        self.words = lexicon(vocab)
        # Zipf weights
        self.cum = []
        s = 0.0
        for i in range(len(self.words)):
            s += 1.0 / (i + 1) ** 1.07
            self.cum.append(s)
        self.total = s

    def word(self) -> str:
        import bisect

        return self.words[bisect.bisect_left(self.cum, self.rng.random() * self.total)]

    def sentence(self, n_min=6, n_max=22) -> str:
        n = self.rng.randint(n_min, n_max)
        ws = [self.word() for _ in range(n)]
        return (" ".join(ws)).capitalize() + "."

    def fact(self) -> Tuple[str, str, str]:
        ent = self.rng.choice(self.words[200:]).capitalize()
        attr = self.rng.choice(self.words[100:1500])
        val = str(self.rng.randint(1, 9999))
        return ent, attr, val

    def paragraph(self, n_sent=(3, 8)) -> str:
        return " ".join(self.sentence() for _ in range(self.rng.randint(*n_sent)))

    def document(self, n_par=(2, 6), facts: int = 2) -> Tuple[str, List[Tuple[str, str, str]]]:
        pars = [self.paragraph() for _ in range(self.rng.randint(*n_par))]
        fs = [self.fact() for _ in range(facts)]
        for ent, attr, val in fs:
            i = self.rng.randrange(len(pars))
            pars[i] += f" The {attr} of {ent} is {val}."
        return "\n\n".join(pars), fs

    def question(self) -> str:
        return (" ".join(self.word() for _ in range(self.rng.randint(6, 14)))).capitalize() + "?"


def corpus(n_docs: int, seed: int = 0) -> List[str]:
    g = TextGen(seed)
    return [g.document()[0] for _ in range(n_docs)]
