#!/usr/bin/env python3
"""Regenerate the machine-derived reference docs: the APP_* configuration schema (the
chain server's --help-config output) and the OpenAPI documents of the chain server and the
model server (the reference ships docs/api_reference/openapi_schema.json for its chain
server). Run from the repo root: ``python scripts/gen_docs.py``."""
import json
import os
import sys
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
warnings.filterwarnings("ignore")


def main():
    from nv_genai_amd.chain_server.configuration import AppConfig
    from nv_genai_amd.chain_server.server import app as chain_app
    from nv_genai_amd.serving.model_server import create_app

    out = os.path.join(ROOT, "docs")
    lines = []
    AppConfig.print_help(lines.append)
    with open(os.path.join(out, "configuration_reference.yaml"), "w") as f:
        f.write("".join(lines))
    with open(os.path.join(out, "api_reference", "chain_server_openapi.json"), "w") as f:
        json.dump(chain_app.openapi(), f, indent=1)
    model_app = create_app(None, None, llm_name="meta/llama3-8b-instruct")
    with open(os.path.join(out, "api_reference", "model_server_openapi.json"), "w") as f:
        json.dump(model_app.openapi(), f, indent=1)
    print("wrote docs/configuration_reference.yaml and docs/api_reference/*.json")


if __name__ == "__main__":
    main()
