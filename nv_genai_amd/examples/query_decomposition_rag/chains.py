"""Query-decomposition agent (SURVEY.md §2.A C9, §3.4;
RetrievalAugmentedGeneration/examples/query_decomposition_rag/chains.py).

A recursive agent with two tools, no LangChain:
* the LLM (stop sequence "\\n\\n") is shown the question + the ledger of sub-questions and
  answers so far and must emit ``{"Tool_Request": "Search"|"Math"|"Nil",
  "Generated Sub Questions": [...]}``;
* **Search** retrieves chunks for each sub-question and asks the LLM to extract the answer;
* **Math** asks the LLM for ``{IsPossible, variable1, variable2, operation}`` and evaluates it
  with a safe arithmetic evaluator (the reference calls Python ``eval`` on model output —
  replaced here, no code from the model is ever executed); on failure it falls back to a
  direct "solve this" LLM call;
* the loop stops when the model says Nil, repeats a sub-question, or after the 4th Search
  round (``trace > 3``); the final answer streams from a prompt built from the ledger.
Malformed JSON is repaired (single -> double quotes, first {...} object) before giving up
with "I can't find an answer for that."
"""
from __future__ import annotations

import json
import logging
import operator
import re
from typing import Any, Dict, Generator, List, Optional

import jinja2

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ...rag.splitters import CharacterTextSplitter
from ..common import NO_CONTEXT, TracedExample, ingest_file

logger = logging.getLogger(__name__)

TEMPLATE = """Your task is to answer questions. If you cannot answer the question, you can request use for a tool and break the question into specific sub questions. Fill with Nil where no action is required. You should only return a JSON containing the tool and the generated sub questions. Consider the contextual information and only ask for information that you do not already have. Do not return any other explanations or text. The output should be a simple JSON structure! You are given two tools:
- Search
- Math
Search tool quickly finds and retrieves relevant answers from a given context, providing accurate and precise information to meet search needs.
Math tool performs essential operations, including multiplication, addition, subtraction, division, and greater than or less than comparisons, providing accurate results with ease. Utilize math tool when asked to find sum, difference of values.
Do not pass sub questions to any tool if they already have an answer in the Contextual Information.
If you have all the information needed to answer the question, mark the Tool_Request as Nil.

Contextual Information:
{{ context }}

Question:
{{ question }}

{"Tool_Request": "<Fill>", "Generated Sub Questions": [<Fill>]}
"""

MATH_TEMPLATE = """Your task is to identify 2 variables and an operation from given questions. If you cannot answer the question, you can simply return "Not Possible". You should only return a JSON containing the `IsPossible`, `variable1`, `variable2`, and `operation`. Do not return any other explanations or text. The output should be a simple JSON structure!
 You are given two options for `IsPossible`:
- Possible
- Not Possible
 `variable1` and `variable2` should be real floating point numbers.
 You are given four options for `operation symbols`:
- '+' (addition)
- '-' (subtraction)
- '*' (multiplication)
- '/' (division)
- '=' (equal to)
- '>' (greater than)
- '<' (less than)
- '>=' (greater than or equal to)
- '<=' (less than or equal to)
    Only return the symbols for the specified operations and nothing else.
Contextual Information:
{{ context }}

Question:
{{ question }}

{"IsPossible": "<Fill>", "variable1": [<Fill>], "variable2": [<Fill>], "operation": [<Fill>]}
"""

EXTRACT_PROMPT = ("Below is a Question and set of Passages that may or may not be relevant. Your task is to "
                  "Extract the answer for question using only the information available in the passages. Be as "
                  "concise as possible and only include the answer if present. Do not infer or process the passage "
                  "in any other way\n\n")

_OPS = {"+": operator.add, "-": operator.sub, "*": operator.mul, "/": operator.truediv,
        "=": operator.eq, "==": operator.eq, ">": operator.gt, "<": operator.lt,
        ">=": operator.ge, "<=": operator.le}


class Ledger:
    def __init__(self):
        self.question_trace: List[str] = []
        self.answer_trace: List[str] = []
        self.trace = 0
        self.done = False

    def context(self) -> str:
        return "".join(f"Sub-Question: {q}\nSub-Answer: {a}\n" for q, a in zip(self.question_trace, self.answer_trace))


def parse_json(text: str) -> Any:
    """json.loads with the repairs of the reference's structured-output helpers
    (experimental/fm-asr-streaming-rag/chain-server/utils.py:41-95)."""
    for cand in (text, text.replace("'", '"')):
        try:
            return json.loads(cand)
        except (json.JSONDecodeError, TypeError):
            pass
        for m in re.finditer(r"\{.*?\}|\[.*?\]", cand, re.S):
            try:
                return json.loads(m.group(0))
            except json.JSONDecodeError:
                continue
    raise ValueError(f"could not parse JSON from model output: {text[:200]!r}")


def _scalar(v) -> float:
    if isinstance(v, list):
        v = v[0] if v else 0
    return float(str(v).replace(",", ""))


def safe_math(var1, op, var2) -> str:
    op = op[0] if isinstance(op, list) else op
    if op not in _OPS:
        raise ValueError(f"unsupported operation {op!r}")
    a, b = _scalar(var1), _scalar(var2)
    return f"{a}{op}{b}={_OPS[op](a, b)}"


class QueryDecompositionChatbot(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)
        self.env = jinja2.Environment()
        self.max_search_rounds = 3

    def ingest_docs(self, filepath: str, filename: str):
        if not filename.endswith((".txt", ".pdf", ".md")):
            raise ValueError(f"{filename} is not a valid Text, PDF or Markdown file")
        try:
            ts = utils.get_config().text_splitter
            ingest_file(utils.get_vectorstore(), filepath, filename,
                        splitter=CharacterTextSplitter(ts.chunk_size, ts.chunk_overlap))
        except Exception as e:
            logger.error("Failed to ingest document due to exception %s", e)
            raise ValueError("Failed to upload document. Please upload an unstructured text document.")

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        cfg = utils.get_config()
        return self.stream_llm([("system", cfg.prompts.chat_template), ("user", "\n\nQuestion: " + query + "\n")], **kwargs)

    # ------------------------------------------------------------------ agent
    def _llm(self, prompt: str, stop=None) -> str:
        llm = utils.get_llm(**self.kwargs)
        kw = {"stop": stop} if stop else {}
        return "".join(llm.stream([("user", prompt)], **kw))

    def retriever(self, query: str) -> List[str]:
        return [d.page_content for d, _ in self.retrieve(utils.get_vectorstore(), query, 4)]

    def extract_answer(self, chunks: List[str], question: str) -> str:
        prompt = EXTRACT_PROMPT + "Question: " + question + "\n\n"
        for i, c in enumerate(chunks):
            prompt += f"Passage {i + 1}:\n{c}\n"
        return self._llm(prompt)

    def search(self, sub_questions: List[str]):
        for sq in sub_questions:
            ans = self.extract_answer(self.retriever(sq), sq)
            self.ledger.question_trace.append(sq)
            self.ledger.answer_trace.append(ans)

    def math(self, sub_questions: List[str]):
        ctx = self.ledger.context()
        try:
            prompt = self.env.from_string(MATH_TEMPLATE).render(context=ctx, question=sub_questions[0])
            out = parse_json(self._llm(prompt))
            answer = safe_math(out["variable1"], out["operation"], out["variable2"])
        except Exception:  # noqa: BLE001 - fall back to a direct answer
            prompt = ("Solve this mathematical question:\nQuestion: " + sub_questions[0]
                      + f"Context:\n{ctx}\nBe concise and only return the answer.")
            answer = self._llm(prompt)
        self.ledger.question_trace.append(sub_questions[0])
        self.ledger.answer_trace.append(answer)
        self.ledger.done = True

    def run_agent(self, question: str, **kwargs) -> str:
        self.ledger = Ledger()
        self.kwargs = kwargs
        tmpl = self.env.from_string(TEMPLATE)
        for _ in range(16):  # hard bound on agent iterations
            prompt = tmpl.render(context=self.ledger.context().strip("\n"), question=question)
            state = parse_json(self._llm(prompt, stop=["\n\n"]))
            subs = state.get("Generated Sub Questions") or ["Nil"]
            tool = state.get("Tool_Request", "Nil")
            if (subs[0] == "Nil" or tool == "Nil" or self.ledger.trace > self.max_search_rounds
                    or subs[0] in self.ledger.question_trace):
                break
            if tool == "Search":
                self.ledger.trace += 1
                self.search(subs)
            elif tool == "Math":
                self.math(subs)
            else:
                raise ValueError(f"Invalid Tool name: {tool}")
        prompt = "Question: " + question + "\n\nSub Questions and Answers\n"
        for q, a in zip(self.ledger.question_trace, self.ledger.answer_trace):
            prompt += f"Sub Question: {q}\nSub Answer: {a}\n"
        return prompt + "\nFinal Answer: "

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        try:
            final_context = self.run_agent(query, **kwargs)
            if not final_context:
                return iter([NO_CONTEXT])
            return self.stream_llm([("user", final_context)], **kwargs)
        except ValueError as e:
            logger.warning("Failed to get response because %s", e)
            return iter(["I can't find an answer for that."])

    def document_search(self, content: str, num_docs: int) -> List[Dict[str, Any]]:
        import os

        hits = self.retrieve(utils.get_vectorstore(), content, 4)
        return [{"source": os.path.basename(d.metadata.get("source", "")), "content": d.page_content, "score": s}
                for d, s in hits]

    def get_documents(self) -> List[str]:
        return utils.get_docs_vectorstore(utils.get_vectorstore())

    def delete_documents(self, filenames: List[str]) -> bool:
        return utils.del_docs_vectorstore(utils.get_vectorstore(), filenames)
