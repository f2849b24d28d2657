"""Minimal ``multipart/form-data`` parser (python-multipart, which FastAPI's ``UploadFile``
needs, is not installed). Enough for the ``POST /documents`` upload contract: returns
``{field_name: (filename or None, bytes)}``."""
from __future__ import annotations

import re
from typing import Dict, Optional, Tuple

_DISP = re.compile(r'(\w+)="((?:[^"\\]|\\.)*)"')


def boundary_of(content_type: str) -> Optional[str]:
    for part in content_type.split(";"):
        part = part.strip()
        if part.lower().startswith("boundary="):
            return part[9:].strip('"')
    return None


def parse_multipart(body: bytes, content_type: str) -> Dict[str, Tuple[Optional[str], bytes]]:
    b = boundary_of(content_type)
    if not b or "multipart/form-data" not in content_type.lower():
        raise ValueError("expected multipart/form-data with a boundary")
    delim = b"--" + b.encode()
    out: Dict[str, Tuple[Optional[str], bytes]] = {}
    for chunk in body.split(delim)[1:]:
        if chunk.startswith(b"--"):
            break
        chunk = chunk[2:] if chunk.startswith(b"\r\n") else chunk
        head, sep, data = chunk.partition(b"\r\n\r\n")
        if not sep:
            continue
        if data.endswith(b"\r\n"):
            data = data[:-2]
        headers = {}
        for line in head.decode("utf-8", errors="replace").split("\r\n"):
            if ":" in line:
                k, v = line.split(":", 1)
                headers[k.strip().lower()] = v.strip()
        params = dict(_DISP.findall(headers.get("content-disposition", "")))
        name = params.get("name")
        if name is not None:
            out[name] = (params.get("filename"), data)
    return out
