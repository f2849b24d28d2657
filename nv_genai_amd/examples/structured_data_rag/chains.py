"""Structured-data (CSV) chatbot (SURVEY.md §2.A C11/C12;
RetrievalAugmentedGeneration/examples/structured_data_rag/chains.py, csv_utils.py,
integrations/pandasai/llms/nv_aiplay.py).

ingest: only .csv; the path is appended to ``ingested_csv_files.txt`` and every later CSV must
have the same columns as the first. rag: all ingested CSVs are concatenated (NaN -> 0), the
LLM is shown the frame description + the ``csv_data_retrieval_template`` instructions and
writes ONE pandas expression over ``df``; the expression is executed in an AST-whitelisted
sandbox (no imports, no dunders, no builtins beyond a few math/type helpers — the reference
runs PandasAI-generated code with full Python); failures are fed back for up to 6 retries
(PandasAI ``max_retries: 6``); the result is phrased by the LLM with ``csv_response_template``.
"""
from __future__ import annotations

import ast
import logging
import os
from typing import Any, Generator, List

import yaml

from ...chain_server import utils
from ...chain_server.base import BaseExample
from ..common import TracedExample

logger = logging.getLogger(__name__)
INGESTED_CSV_FILES_LIST = os.environ.get("INGESTED_CSV_FILES_LIST", "ingested_csv_files.txt")
PROMPT_CONFIG = os.path.join(os.path.dirname(__file__), "csv_prompt_config.yaml")

_ALLOWED_ATTRS = {
    "head", "tail", "sum", "mean", "median", "max", "min", "count", "nunique", "unique", "std", "var",
    "groupby", "sort_values", "nlargest", "nsmallest", "describe", "value_counts", "loc", "iloc",
    "query", "filter", "agg", "size", "reset_index", "idxmax", "idxmin", "round", "abs", "astype",
    "str", "dt", "contains", "startswith", "endswith", "lower", "upper", "extract", "year", "month",
    "day", "hour", "date", "isin", "between", "shape", "columns", "values", "tolist", "to_dict",
    "drop_duplicates", "dropna", "fillna", "cumsum", "diff", "pct_change", "quantile", "mode", "first",
    "last", "apply_len", "len", "T", "index", "name", "prod", "any", "all", "eq", "ne", "gt", "lt", "ge", "le",
}
_ALLOWED_FUNCS = {"len", "round", "abs", "min", "max", "sum", "int", "float", "str", "list", "sorted", "to_datetime"}


def check_expression(expr: str) -> ast.Expression:
    tree = ast.parse(expr.strip(), mode="eval")
    for node in ast.walk(tree):
        if isinstance(node, ast.Attribute):
            if node.attr.startswith("_") or node.attr not in _ALLOWED_ATTRS:
                raise ValueError(f"attribute {node.attr!r} not allowed")
        elif isinstance(node, ast.Name):
            if node.id not in ("df", "pd") and node.id not in _ALLOWED_FUNCS:
                raise ValueError(f"name {node.id!r} not allowed")
        elif isinstance(node, (ast.Lambda, ast.GeneratorExp, ast.ListComp, ast.DictComp, ast.SetComp,
                               ast.NamedExpr, ast.Await, ast.Yield)):
            raise ValueError(f"{type(node).__name__} not allowed")
        elif isinstance(node, ast.Call):
            f = node.func
            if isinstance(f, ast.Name) and f.id not in _ALLOWED_FUNCS:
                raise ValueError(f"call to {f.id!r} not allowed")
            if isinstance(f, ast.Attribute) and isinstance(f.value, ast.Name) and f.value.id == "pd" and f.attr != "to_datetime":
                raise ValueError("only pd.to_datetime is allowed")
    return tree


def run_expression(expr: str, df):
    import pandas as pd

    class _PD:  # only to_datetime is reachable
        to_datetime = staticmethod(pd.to_datetime)

    tree = check_expression(expr)
    env = {"__builtins__": {}, "df": df, "pd": _PD, "len": len, "round": round, "abs": abs,
           "min": min, "max": max, "sum": sum, "int": int, "float": float, "str": str, "list": list,
           "sorted": sorted, "to_datetime": pd.to_datetime}
    return eval(compile(tree, "<csv-query>", "eval"), env, {})  # noqa: S307 - AST-whitelisted above


def extract_df_desc(df) -> str:
    return "\n".join(f"- {c} ({df[c].dtype}), e.g. {df[c].iloc[0]!r}" for c in df.columns) if len(df) else ""


def parse_prompt_config(path: str = PROMPT_CONFIG) -> dict:
    env_path = os.environ.get("CSV_PROMPTS")
    p = env_path if env_path and os.path.exists(env_path) else path
    with open(p) as f:
        return yaml.safe_load(f).get("prompts", {})


def get_prompt_params(csv_prompts: List[dict]) -> dict:
    name = os.environ.get("CSV_NAME", "")
    for p in csv_prompts or []:
        if p.get("name") == name:
            return p
    return {"description": "", "instructions": ""}


class CSVChatbot(BaseExample, TracedExample):
    def __init__(self):
        TracedExample.__init__(self)

    @staticmethod
    def _columns(path: str):
        import pandas as pd

        return list(pd.read_csv(path.strip(), nrows=0).columns)

    def read_and_concatenate_csv(self, file_paths_txt: str):
        import pandas as pd

        with open(file_paths_txt, encoding="UTF-8") as f:
            paths = [p for p in f.read().splitlines() if p]
        frames, ref = [], None
        for p in paths:
            df = pd.read_csv(p)
            if ref is None:
                ref = list(df.columns)
            elif list(df.columns) != ref:
                raise ValueError(f"Columns of the file {p} do not match the reference columns of {paths[0]} file.")
            frames.append(df)
        return pd.concat(frames, ignore_index=True) if frames else pd.DataFrame()

    def ingest_docs(self, filepath: str, filename: str):
        if not filename.endswith(".csv"):
            raise ValueError(f"{filename} is not a valid CSV file")
        with open(INGESTED_CSV_FILES_LIST, "a+", encoding="UTF-8") as f:
            f.seek(0)
            ref = f.readline().strip()
            if ref and self._columns(ref) != self._columns(filepath):
                raise ValueError(f"Columns of the file {filepath} do not match the reference columns of {ref} file.")
            f.write(filepath + "\n")
        logger.info("Document %s ingested successfully", filename)

    def llm_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        return self.stream_llm([("system", utils.get_config().prompts.chat_template), ("user", query)], **kwargs)

    def rag_chain(self, query: str, chat_history: List[Any], **kwargs) -> Generator[str, None, None]:
        if not os.path.exists(INGESTED_CSV_FILES_LIST):
            return iter(["No CSV file ingested"])
        df = self.read_and_concatenate_csv(INGESTED_CSV_FILES_LIST).fillna(0)
        cfg = parse_prompt_config()
        params = get_prompt_params(cfg.get("csv_prompts", []))
        system = cfg["csv_data_retrieval_template"].format(
            description=params.get("description", ""), instructions=params.get("instructions", ""))
        system += ("\nReturn ONLY one Python expression over the dataframe named df "
                   "(no imports, no assignments).\nColumns:\n" + extract_df_desc(df))
        err, result = "", None
        for _attempt in range(6):
            user = query if not err else f"{query}\nThe previous expression failed with: {err}. Fix it."
            expr = self.invoke_llm([("system", system), ("user", user)], **kwargs).strip().strip("`")
            if expr.startswith("python"):
                expr = expr[6:].strip()
            try:
                result = run_expression(expr, df)
                break
            except Exception as e:  # noqa: BLE001 - feed the error back
                err = str(e)
        if result is None:
            return iter(["Could not compute an answer from the ingested CSV data."])
        data = result.to_string() if hasattr(result, "to_string") else str(result)
        prompt = cfg["csv_response_template"].format(query=query, data=data)
        return self.stream_llm([("user", prompt)], **kwargs)

    def get_documents(self) -> List[str]:
        if not os.path.exists(INGESTED_CSV_FILES_LIST):
            return []
        with open(INGESTED_CSV_FILES_LIST) as f:
            return [os.path.basename(p) for p in f.read().splitlines() if p]

    def delete_documents(self, filenames: List[str]) -> bool:
        if not os.path.exists(INGESTED_CSV_FILES_LIST):
            return False
        with open(INGESTED_CSV_FILES_LIST) as f:
            paths = [p for p in f.read().splitlines() if p]
        keep = [p for p in paths if os.path.basename(p) not in filenames]
        with open(INGESTED_CSV_FILES_LIST, "w") as f:
            f.write("".join(p + "\n" for p in keep))
        return len(keep) != len(paths)
