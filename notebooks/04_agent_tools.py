"""Tutorial 04 — an agent that uses tools (reference notebook 04: a LangChain
conversational-react agent with an image-caption tool and a chart-to-table tool backed by
Fuyu / DePlot endpoints). Tools here: an image describer (the vision connector against any
OpenAI-compatible VLM endpoint, or a local stand-in that reports image statistics) and a
table tool; the ReAct loop decides which to call.

    python notebooks/04_agent_tools.py --tiny
"""
import argparse
import os
import tempfile

import numpy as np

from _stack import local_stack

from nv_genai_amd.agents.react import ReActAgent, Tool


def describe_image_locally(path: str) -> str:
    """Stand-in caption tool: size and dominant colour of a PPM/PGM/raw image file."""
    data = np.fromfile(path, dtype=np.uint8)
    return f"image of {data.size} bytes, mean intensity {data.mean():.1f}"


def main(tiny=True, vlm_url=None):
    llm, _, _, svc, _ = local_stack(tiny, max_tokens=48)
    try:
        img = os.path.join(tempfile.mkdtemp(), "sneakers.raw")
        (np.ones((32, 32, 3), dtype=np.uint8) * 230).tofile(img)
        if vlm_url:
            from nv_genai_amd.connectors.vision import VisionClient

            vc = VisionClient(vlm_url)
            caption = lambda p: vc.describe(open(p, "rb").read(), "Describe the image")  # noqa: E731
        else:
            caption = describe_image_locally
        tools = [Tool("ImageCaption", caption, "describe the image at the given file path"),
                 Tool("TabularPlot", lambda p: "| x | y |\n| 1 | 2 |", "convert a chart image at a path to a table")]
        agent = ReActAgent(llm, tools, max_iterations=3)
        out = agent.run(f"this is the image path: {img}")
        print(out["output"][:120], "| steps:", len(out["intermediate_steps"]))
        return out
    finally:
        svc.shutdown()


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--vlm-url")
    a = ap.parse_args()
    main(a.tiny, a.vlm_url)
