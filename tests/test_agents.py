"""CVE exploitability pipeline (checklist → ReAct agent with SBOM / code-QA / version
tools), the LLM graph, list repair, Debian/PEP 440 version ordering, the response cache
proxy and TTS segmentation — on CPU with scripted LLMs."""
import json

import httpx
import pytest

from nv_genai_amd.connectors.fake import HashEmbeddings
from nv_genai_amd.index.vectorstore import VectorStore


def test_list_repair_and_parsing():
    from nv_genai_amd.agents.cve import fix_list_string, numbered_to_list, parse_list

    assert parse_list('Sure: ["Check for lxml", "Review versions"] done') == ["Check for lxml", "Review versions"]
    assert parse_list("'a', 'b'") == ["a", "b"]
    assert parse_list('["Check the \'iterwalk\' use", "x"]') == ["Check the 'iterwalk' use", "x"]
    assert fix_list_string('"it"s broken", "ok"').startswith("[")
    assert numbered_to_list("1. first\n2) second\n- third") == ["first", "second", "third"]


def test_version_tools():
    from nv_genai_amd.agents.cve import SBOMChecker, debian_compare, version_comparator

    assert version_comparator("4.9.0,4.9.1") is True
    assert version_comparator("4.9.2,4.9.1") is False
    assert version_comparator("2.9.12,2.9.10,2.9.14") is True
    assert version_comparator("1.0,0.9,1.0,1.1") is True
    assert "not enough" in version_comparator("1.0")
    assert debian_compare("1:2.30-1ubuntu1", "1:2.30-1ubuntu2") == -1
    assert debian_compare("2.30~rc1-1", "2.30-1") == -1
    assert debian_compare("1:1.0", "2.0") == 1
    assert version_comparator("2.36-0ubuntu1~rc2,2.36-0ubuntu1") is True     # Debian path (not PEP 440)
    sb = SBOMChecker({"LXML": "4.9.0", "libxml2": "2.9.12"})
    assert sb("lxml") == "4.9.0" and "not found" in sb("requests")
    assert "Action input must be only the package name" in sb("lxml version")


def test_react_agent_tools_and_parse_errors():
    from nv_genai_amd.agents.react import PARSE_ERROR, ReActAgent, Tool

    script = iter([
        "I should check the SBOM.\nAction: SBOM Package Checker\nAction Input: lxml",
        "gibberish without the format",
        "Thought: I now know the final answer\nFinal Answer: lxml 4.9.0 is present and vulnerable",
    ])

    class LLM:
        prompts = []

        def invoke(self, messages, **kw):
            assert kw.get("stop") == ["\nObservation:"]
            self.prompts.append(messages[-1][1])
            return next(script)

    llm = LLM()
    agent = ReActAgent(llm, [Tool("SBOM Package Checker", lambda p: {"lxml": "4.9.0"}.get(p, "absent"), "sbom")],
                       preamble="You investigate containers.")
    out = agent.run("Check for lxml")
    assert out["output"] == "lxml 4.9.0 is present and vulnerable"
    assert out["intermediate_steps"][0] == ("SBOM Package Checker", "lxml", "4.9.0")
    assert out["intermediate_steps"][1][2] == PARSE_ERROR
    assert "Observation: 4.9.0" in llm.prompts[1] and "You investigate containers." in llm.prompts[0]


class CVEScript:
    """Checklist LLM answers with a numbered list (forcing the re-parse prompt); the agent LLM
    calls the SBOM tool, then the code QA tool, then answers."""

    def __init__(self):
        self.n = {}

    def invoke(self, messages, **kw):
        text = messages[-1][1]
        if "exploitability assessment checklist" in text:
            return "1. Check for lxml usage\n2. Check for iterwalk calls"
        if "Parse the following numbered checklist" in text:
            return "['Check for lxml usage', 'Check for iterwalk calls']"
        if messages[0][0] == "system" and "pieces of context" in messages[0][1]:
            return "iterwalk is called in parser.py" if "iterwalk" in messages[0][1] else "no usage found"
        q = text.split("Question: ")[-1].split("\n")[0]
        seen = self.n.setdefault(q, 0)
        self.n[q] += 1
        if seen == 0:
            return "Action: SBOM Package Checker\nAction Input: lxml"
        if seen == 1:
            return "Action: Docker Container Code QA System\nAction Input: where is iterwalk used?"
        return f"Final Answer: done: {q}"


def test_cve_pipeline_end_to_end(tmp_path):
    from nv_genai_amd.agents.cve import code_documents, run_cve_pipeline

    (tmp_path / "sbom.csv").write_text("package,version\nlxml,4.9.0\nrequests,2.31.0\n")
    code = tmp_path / "src"
    code.mkdir()
    (code / "parser.py").write_text("import lxml.etree as et\n\ndef walk(doc):\n    return et.iterwalk(doc)\n")
    (code / "other.py").write_text("def unrelated():\n    return 42\n")
    store = VectorStore(HashEmbeddings(dim=64), 64, device="cpu")
    store.add_documents(code_documents(str(code)))
    rows = run_cve_pipeline(["lxml up to 4.9.1 with libxml2 2.9.10-2.9.14: NULL deref via iterwalk"], CVEScript(),
                            sbom_csv=str(tmp_path / "sbom.csv"), code_store=store, repeat=2)
    assert len(rows) == 2
    assert rows[0]["checklist"] == ["Check for lxml usage", "Check for iterwalk calls"]
    assert rows[0]["response"] == ["done: Check for lxml usage", "done: Check for iterwalk calls"]


def test_llm_graph_rejects_cycles():
    from nv_genai_amd.agents.llm_graph import LambdaNode, LLMGraph

    g = LLMGraph().add_node("a", LambdaNode(lambda x: x), ["/b"]).add_node("b", LambdaNode(lambda x: x), ["/a"])
    with pytest.raises(ValueError):
        g.run([{}])


def test_response_cache_proxy_hit_miss_stale():
    from fastapi.testclient import TestClient

    from nv_genai_amd.serving.cache_proxy import ResponseCache, create_cache_proxy

    calls = {"n": 0, "down": False}

    def handler(req: httpx.Request):
        if calls["down"]:
            raise httpx.ConnectError("down")
        calls["n"] += 1
        body = json.loads(req.content)
        return httpx.Response(200, json={"echo": body["input"], "n": calls["n"]})

    cache = ResponseCache(ttl=3600)
    app = create_cache_proxy("http://upstream", cache, transport=httpx.MockTransport(handler))
    with TestClient(app) as c:
        r1 = c.post("/v1/embeddings", json={"input": "a"})
        r2 = c.post("/v1/embeddings", json={"input": "a"})
        r3 = c.post("/v1/embeddings", json={"input": "b"})
        assert r1.headers["x-cache-status"] == "MISS" and r2.headers["x-cache-status"] == "HIT"
        assert r1.json() == r2.json() and r3.json()["n"] == 2 and calls["n"] == 2
        cache.ttl = -1                      # everything expired
        calls["down"] = True
        r4 = c.post("/v1/embeddings", json={"input": "a"})
        assert r4.headers["x-cache-status"] == "STALE" and r4.json()["echo"] == "a"
        assert c.post("/v1/embeddings", json={"input": "zzz"}).status_code == 502


def test_tts_segmentation_matches_reference_rule():
    from nv_genai_amd.dsp.tts import segment_for_tts

    text = " ".join(["word"] * 150)                  # 749 chars
    out = segment_for_tts(text)
    assert out.count(" . ") == len(text) // 300 + 1
    assert out.replace(" . ", "") == text
