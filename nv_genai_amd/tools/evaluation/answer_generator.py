"""Answer generation against a running chain server (tools/evaluation/rag_evaluator/
llm_answer_generator.py): upload the PDFs of a folder (``POST /documents``), then for every
synthetic question call ``POST /generate`` (knowledge base on, temperature 0.2, top_p 0.7,
max_tokens 256) and ``POST /search`` (top_k 1), and save question / generated answer /
retrieved context / ground truth to the evaluation file."""
from __future__ import annotations

import json
import logging
import os
from typing import List

from ...frontend.chat_client import ChatClient

log = logging.getLogger(__name__)


def upload_pdf_files(client: ChatClient, folder: str) -> int:
    n = 0
    for f in sorted(os.listdir(folder)):
        if f.lower().endswith(".pdf"):
            client.upload_documents([os.path.join(folder, f)])
            n += 1
        else:
            log.info("Please ingest PDF file. %s not uploaded", f)
    return n


def generate_answers(base_url: str, dataset_folder: str, qa_path: str, eval_path: str,
                     temperature: float = 0.2, top_p: float = 0.7, max_tokens: int = 256, top_k: int = 1,
                     upload: bool = True) -> List[dict]:
    client = ChatClient(base_url)
    if upload and dataset_folder:
        upload_pdf_files(client, dataset_folder)
    with open(qa_path, encoding="utf-8") as fh:
        data = json.load(fh)
    out = []
    for i, e in enumerate(data, 1):
        log.info("%d/%d", i, len(data))
        e = dict(e)
        e["generated_answer"] = "".join(c for c in client.predict(e["question"], True, max_tokens, temperature, top_p) if c)
        hits = client.search(e["question"], top_k)
        e["retrieved_context"] = [h.get("content", "") for h in hits]
        out.append(e)
    with open(eval_path, "w", encoding="utf-8") as fh:
        json.dump(out, fh, indent=2)
    return out
