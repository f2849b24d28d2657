"""Frozen-dataclass configuration with file + environment-variable loading.

Behavioural contract kept from the reference's ConfigWizard
(RetrievalAugmentedGeneration/common/configuration_wizard.py:44-411), re-implemented on plain
``dataclasses`` (dataclass-wizard is not a dependency here):

* a field's JSON/YAML key is the camelCase of its name (``vector_store`` -> ``vectorStore``);
  snake_case keys are accepted too;
* its environment variable is ``APP`` + ``_<PARENT>`` per nesting level + ``_<KEY>`` where each
  part is the upper-cased camelCase key: ``APP_VECTORSTORE_URL``, ``APP_LLM_MODELNAME``,
  ``APP_TEXTSPLITTER_CHUNKSIZE``, ``APP_RETRIEVER_SCORETHRESHOLD`` ...;
* env values are JSON-decoded when they parse as JSON, else kept as strings;
* precedence quirk: an env value is applied only when the file leaves that key unset or
  falsy (``update_dict(..., overwrite=False)``, configuration_wizard.py:375-411);
* ``from_file`` tries JSON, then YAML (``yaml.safe_load``); unreadable / invalid files log an
  error and return ``None``; an empty file yields the all-defaults config;
* ``print_help`` writes the documented config tree with defaults, types and env names.
"""
from __future__ import annotations

import dataclasses
import json
import logging
import os
import typing
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml

ENV_PREFIX = "APP"
log = logging.getLogger(__name__)


def configclass(cls):
    """Decorator: a frozen dataclass that is also a config section."""
    return dataclasses.dataclass(frozen=True)(cls)


def configfield(name: str, *, default: Any = dataclasses.MISSING, env: bool = True,
                help_txt: str = "", default_factory: Any = dataclasses.MISSING):
    meta = {"json": _camel(name), "env": env, "help": help_txt}
    if default_factory is not dataclasses.MISSING:
        return dataclasses.field(default_factory=default_factory, metadata=meta)
    if default is not dataclasses.MISSING and dataclasses.is_dataclass(default):
        d = default
        return dataclasses.field(default_factory=lambda: d, metadata=meta)
    return dataclasses.field(default=default, metadata=meta)


def _camel(name: str) -> str:
    parts = name.split("_")
    return parts[0] + "".join(p[:1].upper() + p[1:] for p in parts[1:])


def try_json_load(value: str) -> Any:
    try:
        return json.loads(value)
    except (json.JSONDecodeError, TypeError):
        return value


def update_dict(data: Dict[str, Any], path: Tuple[str, ...], value: Any,
                overwrite: bool = False) -> None:
    node = data
    for i, key in enumerate(path):
        last = i == len(path) - 1
        if last:
            if overwrite or not node.get(key):
                node[key] = value
            return
        if not node.get(key):
            node[key] = {}
        if not isinstance(node[key], dict):
            return
        node = node[key]


def read_json_or_yaml(text: str) -> Any:
    try:
        return json.loads(text)
    except ValueError as je:
        try:
            return yaml.safe_load(text)
        except yaml.YAMLError as ye:
            raise ValueError(f"JSON Parser Errors:\n{je}\n\nYAML Parser Errors:\n{ye}") from ye


def _field_json(f: dataclasses.Field) -> str:
    return f.metadata.get("json", _camel(f.name))


def _is_section(tp) -> bool:
    return isinstance(tp, type) and dataclasses.is_dataclass(tp)


def _coerce(tp, value):
    if value is None:
        return None
    origin = typing.get_origin(tp)
    if origin is typing.Union:
        args = [a for a in typing.get_args(tp) if a is not type(None)]
        return _coerce(args[0], value) if args else value
    if _is_section(tp):
        return tp.from_dict(value if isinstance(value, dict) else {}, _env=False)
    if tp is bool:
        if isinstance(value, str):
            return value.strip().lower() in ("1", "true", "yes", "on")
        return bool(value)
    if tp in (int, float, str):
        return tp(value)
    if origin in (list, List):
        return list(value) if isinstance(value, (list, tuple)) else [value]
    return value


class ConfigWizard:
    """Mixin for @configclass sections."""

    @classmethod
    def _hints(cls):
        return typing.get_type_hints(cls)

    @classmethod
    def envvars(cls, env_parent: str = "", json_parent: Tuple[str, ...] = ()) -> List[Tuple[str, Tuple[str, ...], type]]:
        out = []
        hints = cls._hints()
        for f in dataclasses.fields(cls):
            jn = _field_json(f)
            tp = hints.get(f.name, f.type)
            env_name = f"{ENV_PREFIX}{env_parent}_{jn.upper()}"
            if _is_section(tp):
                out += tp.envvars(f"{env_parent}_{jn.upper()}", json_parent + (jn,))
            elif f.metadata.get("env", True):
                out.append((env_name, json_parent + (jn,), tp))
        return out

    @classmethod
    def from_dict(cls, data: Optional[Dict[str, Any]] = None, _env: bool = True):
        if not data:
            data = {}
        if not isinstance(data, dict):
            raise RuntimeError("Configuration data is not a dictionary.")
        data = json.loads(json.dumps(data))  # deep copy, plain types
        if _env:
            for name, path, _tp in cls.envvars():
                raw = os.environ.get(name)
                if raw:
                    update_dict(data, path, try_json_load(raw))
        kwargs = {}
        hints = cls._hints()
        for f in dataclasses.fields(cls):
            jn = _field_json(f)
            tp = hints.get(f.name, f.type)
            if jn in data:
                v = data[jn]
            elif f.name in data:
                v = data[f.name]
            else:
                if _is_section(tp):
                    kwargs[f.name] = tp.from_dict({}, _env=False)
                continue
            try:
                kwargs[f.name] = _coerce(tp, v)
            except (TypeError, ValueError) as e:
                raise ValueError(f"invalid value for {cls.__name__}.{f.name}: {v!r} ({e})") from e
        return cls(**kwargs)

    @classmethod
    def from_file(cls, filepath: str):
        try:
            with open(filepath, encoding="utf-8") as fh:
                text = fh.read()
        except FileNotFoundError:
            log.error("The configuration file cannot be found.")
            return None
        except PermissionError:
            log.error("Permission denied when trying to read the configuration file.")
            return None
        try:
            data = read_json_or_yaml(text) if text.strip() else None
        except ValueError as e:
            log.error("Configuration file must be valid JSON or YAML. The following errors occured:\n%s", e)
            return None
        try:
            return cls.from_dict(data or {})
        except (ValueError, RuntimeError) as e:
            log.error("Invalid configuration value provided:\n%s", e)
            return None

    def to_dict(self) -> Dict[str, Any]:
        out = {}
        for f in dataclasses.fields(self):
            v = getattr(self, f.name)
            out[_field_json(f)] = v.to_dict() if isinstance(v, ConfigWizard) else v
        return out

    @classmethod
    def print_help(cls, write: Callable[[str], Any], env_parent: str = "", depth: int = 0) -> None:
        if depth == 0:
            write("---\n")
        hints = cls._hints()
        pad = "  " * depth
        for f in dataclasses.fields(cls):
            jn = _field_json(f)
            tp = hints.get(f.name, f.type)
            sec = _is_section(tp)
            if sec:
                default = ""
            elif f.default_factory is not dataclasses.MISSING:  # type: ignore[misc]
                default = f.default_factory()  # type: ignore[misc]
            elif f.default is dataclasses.MISSING:
                default = "NO-DEFAULT-VALUE"
            else:
                default = f.default
            write(f"{pad}{jn}: {default}\n")
            inner = pad + ("  " if sec else "")
            if f.metadata.get("help"):
                write(f"{inner}# {f.metadata['help']}\n")
            if not sec:
                write(f"{inner}# Type: {getattr(tp, '__name__', str(tp))}\n")
            if f.metadata.get("env", True):
                write(f"{inner}# ENV Variable: {ENV_PREFIX}{env_parent}_{jn.upper()}\n")
            write("\n")
            if sec:
                tp.print_help(write, f"{env_parent}_{jn.upper()}", depth + 1)
        if depth == 0:
            write("\n")
