"""Event-driven CVE exploitability analysis (reference:
experimental/event-driven-rag-cve-analysis/cyber_dev_day/{pipeline.py, pipeline_utils.py,
checklist_node.py, tools.py, embeddings.py}).

For every CVE description: (1) an LLM writes an exploitability checklist (few-shot prompt,
python-list output, repaired and re-parsed through a second "parse this list" prompt when
needed); (2) a ReAct agent walks the checklist item by item with two tools — an SBOM package
checker (CSV ``package,version``) and a code QA tool (retrieval over the container's source
code, chunked by a Python-aware splitter) — and (3) the rows come back with ``checklist`` and
``response`` columns. Version tools compare PEP 440 versions, then Debian versions, then
strings, like the reference.
"""
from __future__ import annotations

import ast
import csv
import json
import logging
import pathlib
import re
from textwrap import dedent
from typing import Dict, List, Optional, Sequence

from packaging.version import InvalidVersion
from packaging.version import parse as parse_version

from .llm_graph import AgentNode, ExtracterNode, LambdaNode, LLMGenerateNode, LLMGraph, PromptTemplateNode
from .react import ReActAgent, Tool

log = logging.getLogger(__name__)

CHECKLIST_PROMPT = dedent("""\
    You are an expert security analyst. Produce an exploitability assessment checklist for the CVE below: concrete
    steps an analyst runs against a containerised environment to decide whether the CVE is exploitable there. Start
    every item with an action verb; cover the affected packages and versions, vulnerable functions or
    configurations, and any mitigating conditions named in the CVE details.

    Example CVE details: aiohttp before 3.9.2 follows symlinks outside the static root when follow_symlinks=True.
    Example checklist:
    ["Check for aiohttp: verify whether the project depends on aiohttp.",
     "Review affected versions: versions before 3.9.2 are affected.",
     "Review configuration: check whether static routes set follow_symlinks=True."]

    **CVE Details:**
    {{cve_details}}

    **Checklist**:
    Please only provide the comma separated, python formatted list, no other text.""")
PARSELIST_PROMPT = dedent("""\
    Parse the following numbered checklist's contents into a python list in the format ['x', 'y', 'z'], a comma
    separated list surrounded by square braces.

    Checklist:
    {{template}}

    Please only provide the comma separated, python formatted, list.""")
AGENT_PREAMBLE = ("You are a very powerful assistant who helps investigate Docker containers given a checklist of "
                  "investigation items. Your role is to walk through a provided checklist and answer each item in "
                  "the checklist. Do not investigate additional information per checklist item, just answer the "
                  "checklist. Information about the Docker container under investigation is stored in vector "
                  "databases available to you via tools.")

_QUOTED = re.compile(r"""(['"])((?:\\.|[^\\])*?)\1(?=\s*,|\s*\])""")


def fix_list_string(s: str) -> str:
    """Bracket a list literal and escape stray quotes inside its string items."""
    s = s.strip()
    if not s.startswith("["):
        s = "[" + s
    if not s.endswith("]"):
        s = s + "]"

    def esc(m):
        q, body = m.group(1), m.group(2)
        return q + re.sub(r"(?<!\\)" + re.escape(q), "\\\\" + q, body) + q

    return _QUOTED.sub(esc, s)


def parse_list(text: str) -> Optional[List[str]]:
    m = re.search(r"\[.*\]", text, re.DOTALL)
    for cand in ([m.group(0)] if m else []) + [text]:
        for fixed in (cand, fix_list_string(cand)):
            try:
                v = ast.literal_eval(fixed)
                if isinstance(v, (list, tuple)) and all(isinstance(x, str) for x in v):
                    return [x.strip() for x in v]
            except (ValueError, SyntaxError):
                continue
    return None


def numbered_to_list(text: str) -> List[str]:
    items = re.findall(r"^\s*(?:\d+[.)]|[-*])\s+(.*\S)", text, re.MULTILINE)
    return items or [ln.strip() for ln in text.splitlines() if ln.strip()]


# ---------------------------------------------------------------------------- versions
def _deb_order(c: str) -> int:
    if c == "~":
        return -1
    if c.isdigit():
        return 0
    if c.isalpha():
        return ord(c)
    return ord(c) + 256


def _deb_part(a: str, b: str) -> int:
    """dpkg's verrevcmp on one version part."""
    i = j = 0
    while i < len(a) or j < len(b):
        first = 0
        while (i < len(a) and not a[i].isdigit()) or (j < len(b) and not b[j].isdigit()):
            ac = _deb_order(a[i]) if i < len(a) and not a[i].isdigit() else 0
            bc = _deb_order(b[j]) if j < len(b) and not b[j].isdigit() else 0
            if ac != bc:
                return -1 if ac < bc else 1
            i += 1
            j += 1
        while i < len(a) and a[i] == "0":
            i += 1
        while j < len(b) and b[j] == "0":
            j += 1
        while i < len(a) and a[i].isdigit() and j < len(b) and b[j].isdigit():
            if not first:
                first = ord(a[i]) - ord(b[j])
            i += 1
            j += 1
        if i < len(a) and a[i].isdigit():
            return 1
        if j < len(b) and b[j].isdigit():
            return -1
        if first:
            return -1 if first < 0 else 1
    return 0


def debian_compare(a: str, b: str) -> int:
    """-1/0/1 under Debian version ordering ([epoch:]upstream[-revision])."""
    def split(v):
        e, _, rest = v.partition(":") if ":" in v else ("0", "", v)
        up, _, rev = rest.rpartition("-") if "-" in rest else (rest, "", "0")
        if not e.isdigit():
            raise ValueError(f"bad epoch in {v!r}")
        return int(e), up, rev

    ea, ua, ra = split(a)
    eb, ub, rb = split(b)
    if ea != eb:
        return -1 if ea < eb else 1
    return _deb_part(ua, ub) or _deb_part(ra, rb)


def _cmp(a: str, b: str) -> int:
    try:
        x, y = parse_version(a), parse_version(b)
        return (x > y) - (x < y)
    except InvalidVersion:
        pass
    try:
        return debian_compare(a, b)
    except ValueError:
        return (a > b) - (a < b)


def version_comparator(spec: str):
    """"software,vulnerable" → software <= vulnerable; "software,lower,upper" → in range;
    more values → equality with any of them (tools.py:120-150)."""
    v = [x.strip() for x in spec.split(",")]
    if len(v) == 2:
        return _cmp(v[0], v[1]) <= 0
    if len(v) == 3:
        return _cmp(v[0], v[1]) >= 0 and _cmp(v[0], v[2]) <= 0
    if len(v) > 3:
        return any(v[0] == x for x in v[1:])
    return "Couldn't able compare the software version, not enough input"


class SBOMChecker:
    def __init__(self, sbom: Dict[str, str]):
        self.sbom = {k.lower().strip(): v for k, v in sbom.items()}

    @classmethod
    def from_csv(cls, path: str) -> "SBOMChecker":
        with open(path, newline="") as f:
            return cls({r["package"]: r["version"] for r in csv.DictReader(f)})

    def __call__(self, package: str) -> str:
        parts = package.split()
        if len(parts) > 1:
            return (f"Could not comple action, try again. Action input must be only the package name. Input should "
                    f"not contain {parts[1:]} or any text after {parts[0]}")
        p = package.lower().strip()
        return self.sbom.get(p, f"The package '{p}' was not found in the SBOM")


# ---------------------------------------------------------------------------- code QA
PY_SEPARATORS = ["\nclass ", "\ndef ", "\n\tdef ", "\n    def ", "\n\n", "\n", " ", ""]


def notebook_code(path: str) -> str:
    with open(path) as f:
        nb = json.load(f)
    return "\n\n".join("".join(c.get("source", [])) for c in nb.get("cells", []) if c.get("cell_type") == "code")


def code_documents(code_dir: str, include: str = "**/*.py", exclude: Sequence[str] = (),
                   include_notebooks: bool = False, chunk_size: int = 1000, chunk_overlap: int = 200):
    from ..index.vectorstore import Document
    from ..rag.splitters import RecursiveCharacterTextSplitter

    root = pathlib.Path(code_dir)
    files = set(root.glob(include))
    for ex in exclude:
        files -= set(root.glob(ex))
    sp = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap, PY_SEPARATORS)
    docs = []
    for p in sorted(files):
        text = p.read_text(encoding="utf-8", errors="replace")
        docs += [Document(c, {"source": str(p), "language": "python"}) for c in sp.split_text(text)]
    if include_notebooks:
        for nb in sorted(root.glob("**/[!.]*.ipynb")):
            docs += [Document(c, {"source": str(nb), "language": "python"}) for c in sp.split_text(notebook_code(str(nb)))]
    return docs


class CodeQA:
    """RetrievalQA "stuff" chain over the code store."""

    def __init__(self, llm, store, k: int = 4):
        self.llm, self.store, self.k = llm, store, k

    def __call__(self, question: str) -> str:
        docs = self.store.similarity_search(question, self.k)
        ctx = "\n\n".join(d.page_content for d in docs)
        return self.llm.invoke([("system", "Use the following pieces of context to answer the question at the end. "
                                           "If you don't know the answer, just say that you don't know.\n\n" + ctx),
                                ("user", question)])


# ---------------------------------------------------------------------------- pipeline
def build_cve_graph(checklist_llm, agent_llm, sbom: Optional[SBOMChecker] = None, code_store=None,
                    max_iterations: int = 15) -> LLMGraph:
    def to_list(raw: str) -> List[str]:
        got = parse_list(raw)
        if got is not None:
            return got
        again = checklist_llm.invoke([("user", PARSELIST_PROMPT.replace("{{template}}", raw))])
        return parse_list(again) or numbered_to_list(raw)

    tools = []
    if sbom is not None:
        tools.append(Tool("SBOM Package Checker", sbom,
                          "useful for when you need to check the Docker container's software bill of materials "
                          "(SBOM) to get whether or not a given library is in the container. Input should be the "
                          "name of the library or software, and no text following it until a response is returned."))
    if code_store is not None:
        tools.append(Tool("Docker Container Code QA System", CodeQA(agent_llm, code_store),
                          "useful for when you need to review code to check for an import or function usage in the "
                          "Docker container. Input should be a question or the actual code."))
    tools.append(Tool("Version Comparator", version_comparator,
                      "compare a software version against a vulnerable version or range. Input: 'version,vulnerable'"
                      " or 'version,lower,upper'."))

    g = LLMGraph()
    g.add_node("extracter", ExtracterNode(["cve_info"]))
    g.add_node("checklist_prompt", PromptTemplateNode(CHECKLIST_PROMPT, "cve_details"), ["/extracter"])
    g.add_node("checklist_raw", LLMGenerateNode(checklist_llm, temperature=0.0, max_tokens=300), ["/checklist_prompt"])
    g.add_node("checklist", LambdaNode(to_list), ["/checklist_raw"])
    g.add_node("agent", AgentNode(lambda: ReActAgent(agent_llm, tools, AGENT_PREAMBLE, max_iterations)), ["/checklist"])
    g.add_task_handler([("/checklist", "checklist"), ("/agent", "response")])
    return g


def run_cve_pipeline(cves: Sequence[str], checklist_llm, agent_llm=None, sbom_csv: Optional[str] = None,
                     code_store=None, repeat: int = 1) -> List[dict]:
    g = build_cve_graph(checklist_llm, agent_llm or checklist_llm,
                        SBOMChecker.from_csv(sbom_csv) if sbom_csv else None, code_store)
    rows = [{"cve_info": c} for c in cves] * repeat
    return g.run(rows)
