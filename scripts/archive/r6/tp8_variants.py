"""Which engine setting makes the W = 8 one-GPU rehearsal's custom all-reduce time out:
run the rehearsal worker (tests/test_tp8_rehearsal_gpu.py) under several EngineConfig
overrides and print, per variant, the timeout codes, whether tokens match eager, and steps."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import test_tp8_rehearsal_gpu as t  # noqa: E402

VARIANTS = {
    "eager_sync": {"use_graphs": False, "mixed_graphs": False, "async_decode": False},
    "eager_pipelined": {"use_graphs": False, "mixed_graphs": False},
    "decode_graphs": {"mixed_graphs": False},
    "all_graphs_sync": {"async_decode": False},
    "all": {},
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    for name in names:
        res = t._run(True, VARIANTS[name], check=False)
        d = res[0]
        print(json.dumps({"variant": name, "errors": [(r.get("ar_error_init"), r.get("ar_error_mid"), r.get("ar_error")) for r in res],
                          "exc": [r["exc"][-300:] for r in res if "exc" in r][:1],
                          "eq_eager": d.get("out") == d.get("eager"), "out": d.get("out"), "eager": d.get("eager"),
                          "graph_steps": d.get("graph_steps"), "unpipelined": d.get("unpipelined"),
                          "algo": d.get("algo_counts")}), flush=True)
