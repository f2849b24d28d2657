"""Zero-shot ReAct agent over plain-text tools (the LangChain ``ZERO_SHOT_REACT_DESCRIPTION``
agent the CVE pipeline builds in experimental/event-driven-rag-cve-analysis/cyber_dev_day/
pipeline_utils.py:38-107, including its prompt edits: a system preamble, "formulate the input
into a question first", the strict prefix format and ``handle_parsing_errors``).

Loop: prompt = preamble + tool list + format + question + scratchpad → LLM (stopped at
"Observation:") → parse either ``Final Answer:`` or ``Action:`` / ``Action Input:`` → run the
tool → append "Observation: <result>" → repeat, at most ``max_iterations`` times. A reply that
matches neither form gets the parsing-error observation and another turn (when enabled).
"""
from __future__ import annotations

import re
from dataclasses import dataclass
from typing import Callable, List, Optional, Tuple


@dataclass
class Tool:
    name: str
    func: Callable[[str], object]
    description: str


FORMAT = ("Use the following format (start each response with one of the following prefixes): "
          "[Question, Thought, Action, Action Input, Final Answer]). If you are making an action, wait for a "
          "response to the action input before making an observation. Every response must contain at least one "
          "action (and thoughts and observations if you have them), but you cannot have both a final answer and an "
          "action in a response. Action input must only contain the exact input, do not provide any text following "
          "that in your response. Always end your response with either an action, or a final answer.\n\n"
          "Question: the input question you must answer\nThought: you should always think about what to do\n"
          "Action: the action to take, should be one of [{names}]\nAction Input: the input to the action\n"
          "Observation: the result of the action\n... (this Thought/Action/Action Input/Observation can repeat N "
          "times)\nThought: I now know the final answer\nFinal Answer: the final answer to the original input "
          "question")
PARSE_ERROR = "Check your output. Make sure you're using the right Action/Action input syntax."

_ACTION = re.compile(r"Action\s*\d*\s*:[\s]*(.*?)[\s]*Action\s*\d*\s*Input\s*\d*\s*:[\s]*(.*)", re.DOTALL)


def parse_step(text: str) -> Tuple[str, str, str]:
    """→ ("final", answer, "") | ("action", tool, input) | ("error", text, "")."""
    m = _ACTION.search(text)
    if "Final Answer:" in text and not m:
        return "final", text.split("Final Answer:")[-1].strip(), ""
    if m:
        tool = m.group(1).strip().strip("`").strip()
        arg = m.group(2).strip().split("\n")[0].strip().strip('"').strip("`")
        return "action", tool, arg
    return "error", text, ""


class ReActAgent:
    def __init__(self, llm, tools: List[Tool], preamble: str = "", max_iterations: int = 15,
                 handle_parsing_errors: bool = True, include_thoughts: bool = True):
        self.llm, self.tools = llm, {t.name: t for t in tools}
        self.preamble, self.max_iterations = preamble, max_iterations
        self.handle_parsing_errors, self.include_thoughts = handle_parsing_errors, include_thoughts

    def prompt(self, question: str, scratch: str) -> str:
        tool_lines = "\n".join(f"{t.name}: {t.description}" for t in self.tools.values())
        head = (f"{self.preamble} If the input is not a question, formulate it into a question first. "
                f"Include intermediate thought in the final answer. You have access to the following tools:\n\n"
                f"{tool_lines}\n\n" + FORMAT.format(names=", ".join(self.tools)) + "\n\nBegin!\n\n")
        return f"{head}Question: {question}\nThought:{scratch}"

    def run(self, question: str) -> dict:
        scratch = ""
        steps = []
        for _ in range(self.max_iterations):
            out = self.llm.invoke([("user", self.prompt(question, scratch))], stop=["\nObservation:"])
            kind, a, b = parse_step(out)
            if kind == "final":
                return {"output": a, "intermediate_steps": steps}
            if kind == "error":
                if not self.handle_parsing_errors:
                    raise ValueError(f"Could not parse LLM output: {out!r}")
                obs = PARSE_ERROR
                steps.append(("_Exception", out, obs))
            else:
                tool = self.tools.get(a)
                if tool is None:
                    obs = f"{a} is not a valid tool, try one of [{', '.join(self.tools)}]."
                else:
                    try:
                        obs = str(tool.func(b))
                    except Exception as e:  # noqa: BLE001 - tool errors go back to the model
                        obs = f"Tool error: {e}"
                steps.append((a, b, obs))
            scratch += f" {out.strip()}\nObservation: {obs}\nThought:"
        return {"output": "Agent stopped due to iteration limit or time limit.", "intermediate_steps": steps}
