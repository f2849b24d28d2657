"""Document loaders for ingestion (replacing UnstructuredFileLoader / PDFReader /
pdfplumber / python-pptx of the reference, none of which are installed here):

* ``.txt .md .rst .py .json .log`` — plain text;
* ``.html .htm`` — tag-stripped text (stdlib ``html.parser``);
* ``.csv`` — one document per file, rows rendered "col: value" (structured_data_rag reads
  CSVs with pandas directly);
* ``.pdf`` — a self-contained text-layer extractor: objects -> streams (FlateDecode via zlib)
  -> text-showing operators (Tj, TJ, ', ") with literal / hex string decoding, one document
  per page (page number in metadata);
* ``.pptx`` / ``.docx`` — OOXML zip parts, ``<a:t>`` / ``<w:t>`` runs, one document per slide.
Image / OCR extraction (multimodal_rag) goes through the pluggable VLM client instead.
"""
from __future__ import annotations

import csv
import io
import os
import re
import zipfile
import zlib
from html.parser import HTMLParser
from typing import List
from xml.etree import ElementTree

from ..index.vectorstore import Document

TEXT_EXT = {".txt", ".md", ".rst", ".py", ".json", ".log", ".yaml", ".yml"}


def load_file(path: str, filename: str = "") -> List[Document]:
    filename = filename or os.path.basename(path)
    ext = os.path.splitext(filename)[1].lower()
    meta = {"source": path, "filename": filename}
    if ext in TEXT_EXT or ext == "":
        with open(path, encoding="utf-8", errors="replace") as f:
            return [Document(f.read(), meta)]
    if ext in (".html", ".htm"):
        with open(path, encoding="utf-8", errors="replace") as f:
            return [Document(html_to_text(f.read()), meta)]
    if ext == ".csv":
        with open(path, encoding="utf-8", errors="replace", newline="") as f:
            rows = list(csv.DictReader(f))
        text = "\n".join("; ".join(f"{k}: {v}" for k, v in r.items()) for r in rows)
        return [Document(text, meta)]
    if ext == ".pdf":
        with open(path, "rb") as f:
            pages = pdf_pages_text(f.read())
        return [Document(t, {**meta, "page": i + 1}) for i, t in enumerate(pages) if t.strip()]
    if ext == ".pptx":
        return [Document(t, {**meta, "slide": i + 1}) for i, t in enumerate(ooxml_texts(path, "ppt/slides/slide", "a")) if t.strip()]
    if ext == ".docx":
        return [Document("\n".join(ooxml_texts(path, "word/document", "w")), meta)]
    raise ValueError(f"Unsupported file type {ext}")


class _Stripper(HTMLParser):
    def __init__(self):
        super().__init__()
        self.out: List[str] = []
        self._skip = 0

    def handle_starttag(self, tag, attrs):
        if tag in ("script", "style"):
            self._skip += 1
        if tag in ("p", "br", "div", "li", "h1", "h2", "h3", "h4", "tr"):
            self.out.append("\n")

    def handle_endtag(self, tag):
        if tag in ("script", "style") and self._skip:
            self._skip -= 1

    def handle_data(self, data):
        if not self._skip:
            self.out.append(data)


def html_to_text(html: str) -> str:
    p = _Stripper()
    p.feed(html)
    return re.sub(r"\n\s*\n+", "\n\n", "".join(p.out)).strip()


# ------------------------------------------------------------------------------- PDF
_OBJ = re.compile(rb"(\d+)\s+(\d+)\s+obj(.*?)endobj", re.S)
_STREAM = re.compile(rb"stream\r?\n(.*?)\r?\nendstream", re.S)


def _decode_stream(dict_part: bytes, data: bytes) -> bytes:
    if b"/FlateDecode" in dict_part:
        try:
            return zlib.decompress(data)
        except zlib.error:
            try:
                return zlib.decompressobj().decompress(data)
            except zlib.error:
                return b""
    return data


def _pdf_literal(s: bytes, i: int):
    """Parse a (literal) string starting at s[i] == '('; return (bytes, next index)."""
    out = bytearray()
    depth = 1
    i += 1
    while i < len(s) and depth:
        c = s[i]
        if c == 0x5C:  # backslash
            i += 1
            if i >= len(s):
                break
            e = s[i]
            m = {ord("n"): 10, ord("r"): 13, ord("t"): 9, ord("b"): 8, ord("f"): 12}
            if e in m:
                out.append(m[e])
            elif 0x30 <= e <= 0x37:
                j = i
                while j < min(i + 3, len(s)) and 0x30 <= s[j] <= 0x37:
                    j += 1
                out.append(int(s[i:j], 8) & 0xFF)
                i = j - 1
            elif e in (10, 13):
                pass
            else:
                out.append(e)
        elif c == 0x28:
            depth += 1
            out.append(c)
        elif c == 0x29:
            depth -= 1
            if depth:
                out.append(c)
        else:
            out.append(c)
        i += 1
    return bytes(out), i


def _bytes_to_text(b: bytes) -> str:
    if b.startswith(b"\xfe\xff"):
        return b[2:].decode("utf-16-be", errors="replace")
    return b.decode("latin-1")


def content_stream_text(cs: bytes) -> str:
    out: List[str] = []
    i, n = 0, len(cs)
    pending: List[str] = []
    while i < n:
        c = cs[i]
        if c == 0x28:  # (
            s, i = _pdf_literal(cs, i)
            pending.append(_bytes_to_text(s))
            continue
        if c == 0x3C and i + 1 < n and cs[i + 1] != 0x3C:  # <hex>
            j = cs.find(b">", i)
            hx = re.sub(rb"\s", b"", cs[i + 1:j])
            if len(hx) % 2:
                hx += b"0"
            try:
                raw = bytes.fromhex(hx.decode())
                pending.append(raw.decode("utf-16-be", errors="replace") if len(raw) % 2 == 0 and b"\x00" in raw else _bytes_to_text(raw))
            except ValueError:
                pass
            i = j + 1
            continue
        if c == 0x54 and i + 1 < n:  # T-operators
            nx = cs[i + 1]
            if nx in b"jJ":
                out.append("".join(pending))
                pending = []
            elif nx in b"dD*":
                if out and not out[-1].endswith((" ", "\n")):
                    out.append("\n" if nx == 0x2A else " ")
                pending = []
            i += 2
            continue
        if c in b"'\"":
            out.append("\n" + "".join(pending))
            pending = []
            i += 1
            continue
        if c == 0x45 and cs[i:i + 2] == b"ET":
            out.append("\n")
            pending = []
            i += 2
            continue
        i += 1
    return re.sub(r"[ \t]+", " ", "".join(out)).strip()


def pdf_pages_text(data: bytes) -> List[str]:
    objs = {}
    for m in _OBJ.finditer(data):
        objs[int(m.group(1))] = m.group(3)
    # pages in document order, each with its /Contents references
    pages = []
    for num, body in objs.items():
        if re.search(rb"/Type\s*/Page\b", body):
            refs = re.findall(rb"/Contents\s*\[?([\d\s R]+)\]?", body)
            ids = [int(x) for x in re.findall(rb"(\d+)\s+\d+\s+R", refs[0])] if refs else []
            pages.append((num, ids))
    texts = []
    for _, ids in sorted(pages):
        parts = []
        for cid in ids:
            body = objs.get(cid, b"")
            sm = _STREAM.search(body)
            if sm:
                parts.append(content_stream_text(_decode_stream(body[: sm.start()], sm.group(1))))
        texts.append("\n".join(parts))
    if not texts:  # no page tree found: scan every stream
        for body in objs.values():
            sm = _STREAM.search(body)
            if sm:
                t = content_stream_text(_decode_stream(body[: sm.start()], sm.group(1)))
                if t:
                    texts.append(t)
    return texts


def make_pdf(pages: List[str]) -> bytes:
    """Minimal single-font PDF writer (tests / synthetic corpora)."""
    objs = []
    kids = []
    n_pages = len(pages)
    # 1 catalog, 2 pages, 3 font, then per page: page obj + content obj
    font_id = 3
    for i, text in enumerate(pages):
        pid, cid = 4 + 2 * i, 5 + 2 * i
        kids.append(pid)
        lines = text.split("\n")
        ops = ["BT", "/F1 12 Tf", "72 720 Td"]
        for j, ln in enumerate(lines):
            esc = ln.replace("\\", "\\\\").replace("(", "\\(").replace(")", "\\)")
            if j:
                ops.append("0 -14 Td")
            ops.append(f"({esc}) Tj")
        ops.append("ET")
        stream = zlib.compress("\n".join(ops).encode("latin-1", errors="replace"))
        objs.append((pid, f"<< /Type /Page /Parent 2 0 R /Resources << /Font << /F1 {font_id} 0 R >> >> /Contents {cid} 0 R >>".encode()))
        objs.append((cid, b"<< /Length %d /Filter /FlateDecode >>\nstream\n" % len(stream) + stream + b"\nendstream"))
    head = [(1, b"<< /Type /Catalog /Pages 2 0 R >>"),
            (2, f"<< /Type /Pages /Kids [{' '.join(f'{k} 0 R' for k in kids)}] /Count {n_pages} >>".encode()),
            (3, b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica >>")]
    buf = io.BytesIO()
    buf.write(b"%PDF-1.4\n")
    offs = {}
    for oid, body in head + objs:
        offs[oid] = buf.tell()
        buf.write(f"{oid} 0 obj\n".encode() + body + b"\nendobj\n")
    xref = buf.tell()
    nobj = max(offs) + 1
    buf.write(f"xref\n0 {nobj}\n0000000000 65535 f \n".encode())
    for oid in range(1, nobj):
        buf.write(f"{offs.get(oid, 0):010d} 00000 n \n".encode())
    buf.write(f"trailer << /Size {nobj} /Root 1 0 R >>\nstartxref\n{xref}\n%%EOF\n".encode())
    return buf.getvalue()


# ------------------------------------------------------------------------------- OOXML
def ooxml_texts(path: str, part_prefix: str, ns_tag: str) -> List[str]:
    out = []
    with zipfile.ZipFile(path) as z:
        names = [n for n in z.namelist() if n.startswith(part_prefix) and n.endswith(".xml")]

        def key(n):
            m = re.search(r"(\d+)\.xml$", n)
            return int(m.group(1)) if m else 0

        for n in sorted(names, key=key):
            root = ElementTree.fromstring(z.read(n))
            runs = [el.text or "" for el in root.iter() if el.tag.endswith("}t") or el.tag == "t"]
            out.append(" ".join(r for r in runs if r))
    return out
