"""A small LLM-engine graph (the Morpheus ``LLMEngine`` role used by the CVE pipeline,
experimental/event-driven-rag-cve-analysis/cyber_dev_day/pipeline_utils.py:110-127 and
checklist_node.py:222-266): named nodes wired by input paths, run over a batch of rows.

* ``ExtracterNode`` pulls the task's input columns out of each row;
* ``PromptTemplateNode`` renders ``{{var}}`` / ``{var}`` templates;
* ``LLMGenerateNode`` sends every row's prompt concurrently, so with the in-process engine a
  batch of N CVEs becomes N sequences of one continuous batch on the GPU;
* ``LambdaNode`` applies any Python function (e.g. list parsing);
* ``AgentNode`` runs an agent per row (thread pool — agents call tools and the LLM);
* the task handler copies chosen node outputs into output columns.
"""
from __future__ import annotations

import re
from concurrent.futures import ThreadPoolExecutor
from typing import Callable, Dict, List, Optional, Sequence, Tuple, Union


class Node:
    def run(self, inputs: Dict[str, list], rows: List[dict]) -> list:
        raise NotImplementedError


class ExtracterNode(Node):
    def __init__(self, keys: Sequence[str]):
        self.keys = list(keys)

    def run(self, inputs, rows):
        if len(self.keys) == 1:
            return [r[self.keys[0]] for r in rows]
        return [{k: r[k] for k in self.keys} for r in rows]


class PromptTemplateNode(Node):
    def __init__(self, template: str, var: str = "input"):
        self.template, self.var = template, var

    def render(self, value) -> str:
        vals = value if isinstance(value, dict) else {self.var: value}
        out = self.template
        for k, v in vals.items():
            out = out.replace("{{" + k + "}}", str(v)).replace("{" + k + "}", str(v))
        return out

    def run(self, inputs, rows):
        (vals,) = inputs.values()
        return [self.render(v) for v in vals]


class LLMGenerateNode(Node):
    def __init__(self, llm, workers: int = 64, **gen_kwargs):
        self.llm, self.workers, self.kw = llm, workers, gen_kwargs

    def run(self, inputs, rows):
        (prompts,) = inputs.values()
        with ThreadPoolExecutor(max_workers=max(1, min(self.workers, len(prompts)))) as ex:
            return list(ex.map(lambda p: self.llm.invoke([("user", p)], **self.kw), prompts))


class LambdaNode(Node):
    def __init__(self, fn: Callable):
        self.fn = fn

    def run(self, inputs, rows):
        cols = list(inputs.values())
        return [self.fn(*vals) for vals in zip(*cols)]


class AgentNode(Node):
    def __init__(self, make_agent: Callable[[], object], workers: int = 16):
        self.make_agent, self.workers = make_agent, workers

    def run(self, inputs, rows):
        (items,) = inputs.values()

        def one(item):
            qs = item if isinstance(item, list) else [item]
            agent = self.make_agent()
            return [agent.run(q)["output"] for q in qs]

        with ThreadPoolExecutor(max_workers=max(1, min(self.workers, len(items)))) as ex:
            return list(ex.map(one, items))


class LLMGraph:
    def __init__(self):
        self.nodes: Dict[str, Tuple[Node, List[str]]] = {}
        self.outputs: List[Tuple[str, str]] = []

    def add_node(self, name: str, node: Node, inputs: Sequence[str] = ()):
        self.nodes[name] = (node, [i.lstrip("/") for i in inputs])
        return self

    def add_task_handler(self, outputs: Sequence[Tuple[str, str]]):
        self.outputs = [(n.lstrip("/"), col) for n, col in outputs]
        return self

    def run(self, rows: List[dict]) -> List[dict]:
        done: Dict[str, list] = {}
        pending = list(self.nodes)
        while pending:
            progressed = False
            for name in list(pending):
                node, ins = self.nodes[name]
                if all(i in done for i in ins):
                    done[name] = node.run({i: done[i] for i in ins}, rows)
                    pending.remove(name)
                    progressed = True
            if not progressed:
                raise ValueError(f"graph has a cycle or a missing input among {pending}")
        return [dict(r, **{col: done[n][i] for n, col in self.outputs}) for i, r in enumerate(rows)]
