"""Tutorial 04 — an agent that uses tools (reference notebook 04: a LangChain
conversational-react agent with an image-caption tool and a chart-to-table tool backed by
Fuyu / DePlot endpoints). Tools here: an image describer and a chart-to-table tool, both
served by this framework's own vision-language model (models/vision.py, LLaVA / NeVA
architecture; ``--vlm-url`` points them at any OpenAI-compatible VLM endpoint instead); the
ReAct loop decides which to call.

    python notebooks/04_agent_tools.py --tiny
"""
import argparse
import os
import tempfile

import numpy as np

from _stack import local_stack

from nv_genai_amd.agents.react import ReActAgent, Tool


def _write_png(path: str) -> None:
    from PIL import Image

    arr = np.zeros((96, 128, 3), dtype=np.uint8)
    arr[:, :, 0] = 230
    arr[40:90, 20:40, 1] = 200          # a bar-chart-like blob
    arr[20:90, 60:80, 2] = 200
    Image.fromarray(arr).save(path)


def main(tiny=True, vlm_url=None):
    llm, _, _, svc, _ = local_stack(tiny, max_tokens=48)
    try:
        img = os.path.join(tempfile.mkdtemp(), "sneakers.png")
        _write_png(img)
        if vlm_url:
            from nv_genai_amd.connectors.vision import VisionClient

            vlm = VisionClient(vlm_url)
        else:
            from nv_genai_amd.engine.llm_engine import EngineConfig
            from nv_genai_amd.models.vision import VisionLanguageModel

            if tiny:
                vlm = VisionLanguageModel("vlm-tiny", device="cpu", engine_cfg=EngineConfig(
                    model="llama-tiny", max_num_seqs=4, max_batched_tokens=1024, max_model_len=1024,
                    kv_cache_blocks=64, use_graphs=False))
            else:
                vlm = VisionLanguageModel("llava-1.5-7b")

        def caption(p):
            return vlm.describe(open(p.strip(), "rb").read(), "Describe the image", max_tokens=24)

        def chart_table(p):
            return vlm.describe(open(p.strip(), "rb").read(),
                                "Generate underlying data table of the figure below:", max_tokens=24)

        tools = [Tool("ImageCaption", caption, "describe the image at the given file path"),
                 Tool("TabularPlot", chart_table, "convert a chart image at a path to a table")]
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
