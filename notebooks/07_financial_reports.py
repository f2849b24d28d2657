"""Tutorial 07 — chat with financial reports (reference notebook 07: fetch quarterly-results
HTML pages, pull out title/time/text and the tables, have the LLM summarise each table, split
text + table summaries with a 200/50 token splitter, store in the vector DB, answer with a
[INST] prompt over the retrieved content list).

    python notebooks/07_financial_reports.py --tiny
"""
import argparse
import re

from _stack import local_stack

from nv_genai_amd.index.vectorstore import Document, VectorStore
from nv_genai_amd.rag.loaders import html_to_text
from nv_genai_amd.rag.splitters import TokenTextSplitter

REPORT = ("<html><head><title>NVIDIA Announces Financial Results for Fourth Quarter and Fiscal 2024</title></head>"
          "<body><p>Record quarterly revenue of $22.1 billion, up 22% from Q3.</p><table><tr><th>Quarter</th>"
          "<th>Revenue</th></tr><tr><td>Q4 FY24</td><td>$22,103M</td></tr><tr><td>Q3 FY24</td><td>$18,120M</td></tr>"
          "</table><p>Data Center revenue was a record $18.4 billion.</p></body></html>")
PROMPT = ("[INST]You are a friendly virtual assistant. Your task is to understand the QUESTION, read the Content "
          "list from the DOCUMENT delimited by ```, generate an answer based on the Content, and provide "
          "references used in answering the question.\nDOCUMENT: ```{context}```\nQUESTION: ```{question}```[/INST]")


def extract(html: str):
    title = re.search(r"<title>(.*?)</title>", html, re.S)
    tables = re.findall(r"<table.*?</table>", html, re.S)
    text = html_to_text(re.sub(r"<table.*?</table>", " ", html, flags=re.S))
    return (title.group(1).strip() if title else ""), text, tables


def table_to_markdown(t: str) -> str:
    rows = re.findall(r"<tr>(.*?)</tr>", t, re.S)
    cells = [[html_to_text(c) for c in re.findall(r"<t[hd]>(.*?)</t[hd]>", r, re.S)] for r in rows]
    return "\n".join("| " + " | ".join(c) + " |" for c in cells)


def main(tiny=True):
    llm, emb, _, svc, engine = local_stack(tiny, max_tokens=48)
    try:
        title, text, tables = extract(REPORT)
        summaries = [llm.invoke([("user", "[INST] Summarise the following TABLE in the markdown format, keep every "
                                          f"number.\nTITLE: {title}\nTABLE:\n{table_to_markdown(t)} [/INST]")])
                     for t in tables]
        sp = TokenTextSplitter(tokens_per_chunk=200, chunk_overlap=50)
        docs = [Document(c, {"title": title, "kind": "text"}) for c in sp.split_text(text)]
        docs += [Document(table_to_markdown(t) + "\n" + s, {"title": title, "kind": "table"})
                 for t, s in zip(tables, summaries)]
        store = VectorStore(emb, engine.dim, device=str(engine.device), name="NVIDIA_Finance")
        store.add_documents(docs)
        q = "What was the revenue in Q4 FY24?"
        ctx = "\n".join(d.page_content for d in store.similarity_search(q, 4))
        answer = "".join(llm.stream([("user", PROMPT.format(context=ctx, question=q))]))
        print(f"{len(docs)} chunks ({len(tables)} tables); answer: {answer[:60]!r}")
        return docs
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    main(ap.parse_args().tiny)
