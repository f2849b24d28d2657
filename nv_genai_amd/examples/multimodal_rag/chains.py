"""Multimodal RAG over PDF / PPTX (SURVEY.md §2.A C10;
RetrievalAugmentedGeneration/examples/multimodal_rag/chains.py,
vectorstore/custom_pdf_parser.py, custom_powerpoint_parser.py, vectorstore_updater.py).

ingest (.pdf/.pptx only): :mod:`.parsers` turns every page / slide into text, table and image
documents — header/footer crop, ruled tables through DePlot + the LLM, captioned images that
NeVA calls a graph/plot/chart explained the same way, PPTX speaker notes (the Neva -> DePlot ->
LLM path); all documents are split with a 1000/100 character splitter and stored with the
parser's metadata plus ``filename``.
rag: "Relevant documents:" + retrieved chunks + "\\n\\n[[QUESTION]]\\n\\n" + query with
``rag_template`` as the system prompt. The reference builds that string from a list, which
raises and always lands in its fallback branch (plain top-k, no score threshold — SURVEY.md
§7.4 item 7); that effective behaviour is what is implemented.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, Generator, List

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ...connectors.vision import get_vision_client
from ...rag.splitters import RecursiveCharacterTextSplitter
from ..common import NO_CONTEXT, NO_DOCS, TracedExample
from .parsers import CHART_WORDS, get_pdf_documents, process_ppt_file

logger = logging.getLogger(__name__)
CHART_SYSTEM = ("Your responsibility is to explain charts. You are an expert in describing the responses of "
                "linearized tables into plain English text for LLMs to use.")


class MultimodalRAG(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)
        self.splitter = RecursiveCharacterTextSplitter(1000, 100)

    # the reference's is_graph / process_graph (custom_pdf_parser.py:40-70) on JPEG q=20 bytes
    def is_graph(self, jpeg: bytes) -> bool:
        res = get_vision_client("ai-neva-22b").describe(jpeg, "Describe this image in detail", creativity=0,
                                                        quality=9, complexity=0, verbosity=9)
        return any(w in res for w in CHART_WORDS)

    def process_graph(self, jpeg: bytes) -> str:
        table = get_vision_client("ai-google-deplot").describe(jpeg, "Generate underlying data table of the figure below:")
        return self.invoke_llm([("system", CHART_SYSTEM), ("user", "Explain the following linearized table. " + table)])

    def ocr(self, jpeg: bytes) -> str:
        """Page transcription for PDF pages without a text layer (the reference runs tesseract,
        custom_pdf_parser.py:142-165, not installed here: the vision model reads the page)."""
        return get_vision_client("ai-neva-22b").describe(jpeg, "Transcribe all the text in this image", creativity=0,
                                                         quality=9, complexity=0, verbosity=9)

    def ingest_docs(self, filepath: str, filename: str):
        if not filename.endswith((".pdf", ".pptx")):
            raise ValueError(f"{filename} is not a valid PDF/PPTX file. Only PDF/PPTX files are supported for "
                             "multimodal rag. The PDF/PPTX files can contain multimodal data.")
        try:
            if filename.endswith(".pdf"):
                docs = [d for page in get_pdf_documents(filepath, self.is_graph, self.process_graph, ocr=self.ocr)
                        for d in page]
            else:
                docs = process_ppt_file(filepath, self.is_graph, self.process_graph)
            docs = self.splitter.split_documents(docs)
            for d in docs:
                d.metadata["filename"] = filename
            utils.get_vectorstore().add_documents(docs)
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
