"""Synthetic QA generation (SURVEY.md §2.A C18;
tools/evaluation/synthetic_data_generator/data_generator.py): every file in a folder is loaded,
split into 3000-character chunks (overlap 100), and the LLM is asked for two question/answer
pairs per chunk as JSON; pairs are extracted with a tolerant regex and saved with their
ground-truth context."""
from __future__ import annotations

import json
import logging
import os
import re
from typing import List, Optional

from ...rag.loaders import load_file
from ...rag.splitters import RecursiveCharacterTextSplitter

log = logging.getLogger(__name__)
SYS_PROMPT = ("Given the context paragraph, create two very good question answer pairs. Your output should be "
              "strictly in a json format of individual question answer pairs with keys from "
              "[\"question\",\"answer\"]. Restrict the question to the context information provided.")
_Q = re.compile(r'"question":\s*"([^"]*)"')
_A = re.compile(r'"answer":\s*"([^"]*)"')


def generate_synthetic_data(folder: str, out_path: str, llm, chunk_size: int = 3000, chunk_overlap: int = 100,
                            max_files: Optional[int] = None) -> List[dict]:
    split = RecursiveCharacterTextSplitter(chunk_size, chunk_overlap)
    files = sorted(f for f in os.listdir(folder) if os.path.isfile(os.path.join(folder, f)))[:max_files]
    rows: List[dict] = []
    for i, f in enumerate(files, 1):
        log.info("%d/%d %s", i, len(files), f)
        try:
            docs = load_file(os.path.join(folder, f))
        except ValueError:
            continue
        for chunk in split.split_documents(docs):
            out = llm.invoke([("system", SYS_PROMPT), ("user", f"[The Start of the Reference Context]{chunk.page_content}"
                                                                f"[The End of Reference Context]")])
            for q, a in zip(_Q.findall(out), _A.findall(out)):
                rows.append({"question": q, "ground_truth_answer": a, "ground_truth_context": chunk.page_content,
                             "document": f})
    with open(out_path, "w", encoding="utf-8") as fh:
        json.dump(rows, fh, indent=2)
    return rows
