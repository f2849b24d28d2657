"""Multimodal RAG over PDF / PPTX (SURVEY.md §2.A C10;
RetrievalAugmentedGeneration/examples/multimodal_rag/chains.py,
vectorstore/custom_pdf_parser.py, custom_powerpoint_parser.py, vectorstore_updater.py).

ingest (.pdf/.pptx only): page / slide text, plus every embedded image sent to the vision
client — first "is it a graph/plot/chart?", and for charts a chart-to-table pass whose
linearised table the LLM then explains in plain English (the Neva -> DePlot -> LLM path);
all texts are split with a 1000/100 character splitter and stored with
``{"filename", "page"|"slide", "type"}`` metadata.
rag: "Relevant documents:" + retrieved chunks + "\\n\\n[[QUESTION]]\\n\\n" + query with
``rag_template`` as the system prompt. The reference builds that string from a list, which
raises and always lands in its fallback branch (plain top-k, no score threshold — SURVEY.md
§7.4 item 7); that effective behaviour is what is implemented.
"""
from __future__ import annotations

import logging
import os
import re
import zipfile
import zlib
from typing import Any, Dict, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ...connectors.vision import get_vision_client
from ...index.vectorstore import Document
from ...rag.loaders import load_file
from ...rag.splitters import RecursiveCharacterTextSplitter
from ..common import NO_CONTEXT, NO_DOCS, TracedExample

logger = logging.getLogger(__name__)
CHART_SYSTEM = ("Your responsibility is to explain charts. You are an expert in describing the responses of "
                "linearized tables into plain English text for LLMs to use.")


def pdf_images(data: bytes) -> List[bytes]:
    out = []
    for m in re.finditer(rb"obj(.*?)stream\r?\n(.*?)\r?\nendstream", data, re.S):
        head, body = m.group(1), m.group(2)
        if b"/Subtype /Image" not in head and b"/Subtype/Image" not in head:
            continue
        if b"/DCTDecode" in head:
            out.append(body)  # JPEG bytes as stored
        elif b"/FlateDecode" in head:
            try:
                zlib.decompress(body)
                out.append(body)
            except zlib.error:
                pass
    return out


def pptx_images(path: str) -> List[bytes]:
    with zipfile.ZipFile(path) as z:
        return [z.read(n) for n in sorted(z.namelist()) if n.startswith("ppt/media/")]


class MultimodalRAG(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)
        self.splitter = RecursiveCharacterTextSplitter(1000, 100)

    def _image_texts(self, images: List[bytes], filename: str) -> List[Document]:
        neva = get_vision_client("ai-neva-22b")
        deplot = get_vision_client("ai-google-deplot")
        docs = []
        for i, img in enumerate(images):
            desc = neva.describe(img, "Describe this image in detail", creativity=0, quality=9,
                                 complexity=0, verbosity=9)
            if any(w in desc.lower() for w in ("graph", "plot", "chart")):
                table = deplot.describe(img, "Generate underlying data table of the figure below:")
                desc = self.invoke_llm([("system", CHART_SYSTEM),
                                        ("user", "Explain the following linearized table. " + table)])
            docs.append(Document(desc, {"filename": filename, "type": "image", "image": i}))
        return docs

    def ingest_docs(self, filepath: str, filename: str):
        if not filename.endswith((".pdf", ".pptx")):
            raise ValueError(f"{filename} is not a valid PDF/PPTX file. Only PDF/PPTX files are supported for "
                             "multimodal rag. The PDF/PPTX files can contain multimodal data.")
        try:
            docs = load_file(filepath, filename)
            for d in docs:
                d.metadata.update({"filename": filename, "type": "text"})
            if filename.endswith(".pdf"):
                with open(filepath, "rb") as f:
                    images = pdf_images(f.read())
            else:
                images = pptx_images(filepath)
            docs += self._image_texts(images, filename)
            utils.get_vectorstore().add_documents(self.splitter.split_documents(docs))
        except Exception as e:
            logger.error("Failed to ingest document due to exception %s", e)
            raise ValueError("Failed to upload document. Please upload an unstructured text document.")

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        return self.stream_llm([("system", utils.get_config().prompts.chat_template), ("user", query)], **kwargs)

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        cfg = utils.get_config()
        try:
            docs = [d for d, _ in self.retrieve(utils.get_vectorstore(), query, cfg.retriever.top_k)]
            if not docs:
                return iter([NO_CONTEXT])
            prompt = "Relevant documents:" + " ".join(d.page_content for d in docs) + "\n\n[[QUESTION]]\n\n" + query
            return self.stream_llm([("system", cfg.prompts.rag_template), ("user", prompt)], **kwargs)
        except Exception as e:  # noqa: BLE001
            logger.warning("Failed to generate response due to exception %s", e)
        return iter([NO_DOCS])

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        hits = self.retrieve(utils.get_vectorstore(), content, utils.get_config().retriever.top_k)
        return [{"source": d.metadata.get("filename", ""), "content": d.page_content, "score": s} for d, s in hits]

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)
