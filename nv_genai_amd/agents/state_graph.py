"""A minimal state graph for agent loops (the LangGraph ``StateGraph`` role in
notebooks/06_LangGraph_HandlingAgent_IntermediateSteps.ipynb: an ``agent`` node that decides,
an ``action`` node that runs tools, a conditional edge ``continue``/``end``, and an
``intermediate_steps`` list that accumulates (operator.add) across iterations).

Nodes return partial state updates; keys registered with a reducer are combined
(``reducers={"intermediate_steps": operator.add}``), others overwrite.
"""
from __future__ import annotations

from typing import Callable, Dict, Optional

END = "__end__"


class StateGraph:
    def __init__(self, reducers: Optional[Dict[str, Callable]] = None):
        self.nodes: Dict[str, Callable[[dict], dict]] = {}
        self.edges: Dict[str, str] = {}
        self.cond: Dict[str, tuple] = {}
        self.entry: Optional[str] = None
        self.reducers = reducers or {}

    def add_node(self, name: str, fn: Callable[[dict], dict]):
        self.nodes[name] = fn
        return self

    def set_entry_point(self, name: str):
        self.entry = name
        return self

    def add_edge(self, a: str, b: str):
        self.edges[a] = b
        return self

    def add_conditional_edges(self, a: str, decide: Callable[[dict], str], mapping: Dict[str, str]):
        self.cond[a] = (decide, mapping)
        return self

    def invoke(self, state: dict, max_steps: int = 50, on_step: Optional[Callable[[str, dict], None]] = None) -> dict:
        state = dict(state)
        node = self.entry
        for _ in range(max_steps):
            if node == END or node is None:
                return state
            upd = self.nodes[node](state) or {}
            for k, v in upd.items():
                state[k] = self.reducers[k](state.get(k, type(v)()), v) if k in self.reducers else v
            if on_step:
                on_step(node, upd)
            if node in self.cond:
                decide, mapping = self.cond[node]
                node = mapping[decide(state)]
            else:
                node = self.edges.get(node, END)
        raise RuntimeError("state graph did not reach END within max_steps")
