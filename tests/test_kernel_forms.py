"""The kernel-form registry (csrc/kernels/kernels.h KernelForm, csrc/bindings.cpp kForms) against
its documentation: every A/B form has its ``NGA_*`` row in docs/environment.md, and the
documented default is the registry's default. Runs on CPU (no kernel is launched)."""
import os
import re

import pytest

from nv_genai_amd import ops

DOC = os.path.join(os.path.dirname(__file__), "..", "docs", "environment.md")


def _doc_defaults():
    rows = {}
    for line in open(DOC, encoding="utf-8"):
        m = re.match(r"\|\s*`(NGA_[A-Z0-9_]+)`\s*\|\s*([^|]+)\|", line)
        if m:
            rows[m.group(1)] = m.group(2).strip().strip("`")
    return rows


@pytest.mark.skipif(not ops.have_kernels(), reason="needs the built _C extension")
def test_every_form_documented_with_its_default(monkeypatch):
    rows = _doc_defaults()
    for name in ops.KERNEL_FORMS:
        env = "NGA_" + name.upper()
        assert env in rows, f"{env} (form {name}) missing from docs/environment.md"
        if os.environ.get(env):
            continue   # the registry was seeded from the environment, not its default
        doc = rows[env]
        if re.fullmatch(r"-?\d+", doc):
            assert ops.kernel_form(name) == int(doc), (name, doc)


@pytest.mark.skipif(not ops.have_kernels(), reason="needs the built _C extension")
def test_form_set_and_restore(kernel_form):
    before = ops.kernel_form("decode_dma_aux")
    kernel_form("decode_dma_aux", 0)
    assert ops.kernel_form("decode_dma_aux") == 0
    kernel_form("decode_dma_aux", before)
    assert ops.kernel_form("decode_dma_aux") == before
