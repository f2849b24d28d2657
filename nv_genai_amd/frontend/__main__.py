"""``python -m nv_genai_amd.frontend`` — run the RAG playground
(frontend/frontend/__main__.py: --host/--port, -v/-q verbosity, --help-config).

Config (frontend/frontend/configuration.py): ``APP_SERVERURL``, ``APP_SERVERPORT``,
``APP_MODELNAME`` or a JSON/YAML file in ``APP_CONFIG_FILE``.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

from ..chain_server.config_wizard import ConfigWizard, configclass, configfield


@configclass
class FrontendConfig(ConfigWizard):
    server_url: str = configfield("serverUrl", default="http://localhost",
                                  help_txt="The location of the chain server.")
    server_port: str = configfield("serverPort", default="8081", help_txt="The port on which the chain server is listening.")
    model_name: str = configfield("modelName", default="meta/llama3-8b-instruct",
                                  help_txt="The name of the hosted LLM model.")


def main(argv=None):
    ap = argparse.ArgumentParser(prog="nv_genai_amd.frontend")
    ap.add_argument("--host", default=os.environ.get("APP_HOST", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("APP_PORT", "8090")))
    ap.add_argument("-v", "--verbose", action="count", default=int(os.environ.get("APP_VERBOSITY", "1")))
    ap.add_argument("-q", "--quiet", action="count", default=0)
    ap.add_argument("--help-config", action="store_true")
    args = ap.parse_args(argv)
    if args.help_config:
        FrontendConfig.print_help(sys.stdout.write)
        return
    level = max(logging.DEBUG, logging.WARNING - 10 * (args.verbose - args.quiet))
    logging.basicConfig(level=level)
    path = os.environ.get("APP_CONFIG_FILE")
    cfg = (FrontendConfig.from_file(path) if path else None) or FrontendConfig.from_dict({})
    import uvicorn

    from .api import create_frontend
    from .chat_client import ChatClient

    client = ChatClient(f"{cfg.server_url}:{cfg.server_port}", cfg.model_name)
    uvicorn.run(create_frontend(client), host=args.host, port=args.port, log_level=logging.getLevelName(level).lower())


if __name__ == "__main__":
    main()
