"""Tutorial 06 — an agent loop as a state graph, keeping the intermediate steps (reference
notebook 06: LangGraph ``StateGraph`` with an ``agent`` node, an ``action`` node, a
conditional ``continue``/``end`` edge and ``intermediate_steps`` accumulated with
operator.add; tools: a retriever over a Sweden text and a Wikipedia lookup).

    python notebooks/06_graph_agent.py --tiny
"""
import argparse
import operator

from _stack import local_stack

from nv_genai_amd.agents.react import parse_step
from nv_genai_amd.agents.state_graph import END, StateGraph
from nv_genai_amd.index.vectorstore import VectorStore

SWEDEN = ["Sweden has a population of about 10.5 million.", "Stockholm is the capital of Sweden.",
          "Sweden joined the European Union in 1995."]


def build_app(llm, store):
    tools = {"AboutSweden": lambda q: store.similarity_search(q, 1)[0].page_content,
             "Wiki": lambda q: f"(offline encyclopedia) no article for {q!r}"}

    def run_agent(state):
        scratch = "".join(f"\nAction: {a}\nAction Input: {i}\nObservation: {o}" for a, i, o in state["intermediate_steps"])
        if len(state["intermediate_steps"]) >= 2:
            return {"agent_outcome": ("final", state["intermediate_steps"][-1][2], "")}
        out = llm.invoke([("system", "Use a tool: AboutSweden (questions about Sweden) or Wiki (anything else). "
                                     "Reply with 'Action: <tool>' and 'Action Input: <query>' or 'Final Answer: ...'."),
                          ("user", state["input"] + scratch)])
        kind, a, b = parse_step(out)
        if kind == "error":            # route a free-form reply to the retriever like a tool call
            kind, a, b = "action", "AboutSweden", state["input"]
        return {"agent_outcome": (kind, a, b)}

    def execute_tools(state):
        _, tool, arg = state["agent_outcome"]
        obs = tools.get(tool, tools["Wiki"])(arg)
        return {"intermediate_steps": [(tool, arg, obs)]}

    g = StateGraph(reducers={"intermediate_steps": operator.add})
    g.add_node("agent", run_agent).add_node("action", execute_tools).set_entry_point("agent")
    g.add_conditional_edges("agent", lambda s: "end" if s["agent_outcome"][0] == "final" else "continue",
                            {"continue": "action", "end": END})
    g.add_edge("action", "agent")
    return g


def main(tiny=True):
    llm, emb, _, svc, engine = local_stack(tiny, max_tokens=32)
    try:
        store = VectorStore(emb, engine.dim, device=str(engine.device))
        store.add_texts(SWEDEN)
        out = build_app(llm, store).invoke({"input": "What is Sweden's population?", "intermediate_steps": []})
        for step in out["intermediate_steps"]:
            print("step:", step)
        return out
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    main(ap.parse_args().tiny)
