"""Tutorial 01 — the REST data loader (reference notebooks/01_dataloader.ipynb): upload
documents to the chain server's ``/documents`` endpoint with timing, then ask the same
question without and with the knowledge base through ``/generate`` (SSE), counting the
streamed chunks and the time to the last one.

    python notebooks/01_dataloader.py --tiny          # in-process chain server, CPU
    python notebooks/01_dataloader.py --url http://chain-server:8081 --docs ./dataset
"""
import argparse
import json
import os
import tempfile
import time

from _stack import local_stack  # noqa: F401  (path setup)


def upload_documents(client, folder, limit=100):
    n = 0
    for name in sorted(os.listdir(folder))[:limit]:
        with open(os.path.join(folder, name), "rb") as f:
            r = client.post("/documents", files={"file": (name, f, "application/octet-stream")})
            r.raise_for_status()
            n += 1
    return n


def ask(client, question, use_kb, max_tokens=64):
    body = {"messages": [{"role": "user", "content": question}], "use_knowledge_base": use_kb,
            "max_tokens": max_tokens}
    t0 = time.time()
    chunks, text = 0, ""
    with client.stream("POST", "/generate", json=body) as r:
        for line in r.iter_lines():
            if line.startswith("data: "):
                d = json.loads(line[6:])
                if d["choices"][0].get("finish_reason") == "[DONE]":
                    break
                text += d["choices"][0]["message"]["content"]
                chunks += 1
    return text, chunks, time.time() - t0


def main(tiny=True, url=None, docs=None):
    if url:
        import httpx

        client = httpx.Client(base_url=url, timeout=600)
    else:
        # in-process chain server: deterministic fake LLM + hash embedder (tiny), or the
        # in-process GPU engines
        os.environ.setdefault("APP_LLM_MODELENGINE", "fake" if tiny else "local")
        os.environ.setdefault("APP_EMBEDDINGS_MODELENGINE", "hash" if tiny else "local")
        os.environ.setdefault("APP_EMBEDDINGS_DIMENSIONS", "256" if tiny else "1024")
        from fastapi.testclient import TestClient

        from nv_genai_amd.chain_server import server
        server.UPLOAD_DIR = tempfile.mkdtemp()
        client = TestClient(server.app)
        client.__enter__()
    folder = docs
    if folder is None:
        folder = tempfile.mkdtemp()
        for i in range(3):
            with open(os.path.join(folder, f"press_{i}.txt"), "w") as f:
                f.write(f"Press release {i}: the Grace superchip has 144 Arm cores. " * 20)
    t0 = time.time()
    n = upload_documents(client, folder)
    print(f"uploaded {n} documents in {time.time() - t0:.2f}s")
    for kb in (False, True):
        text, chunks, dt = ask(client, "how many cores are on the grace superchip?", kb)
        print(f"use_knowledge_base={kb}: {chunks} chunks in {dt:.2f}s: {text[:80]!r}")
    return n


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--url")
    ap.add_argument("--docs")
    a = ap.parse_args()
    main(a.tiny, a.url, a.docs)
