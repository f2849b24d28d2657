"""Layout-aware PDF reader for multimodal ingestion (the pdfplumber role in
RetrievalAugmentedGeneration/examples/multimodal_rag/vectorstore/custom_pdf_parser.py; neither
pdfplumber nor pdfminer is installed here, so this is a self-contained reader).

What it recovers per page, in pdfplumber's top-left coordinates (``top`` grows downwards):

* ``chars`` — every shown glyph with its box (x0, x1, top, bottom) and font size, from a
  content-stream interpreter that tracks the CTM (q / Q / cm), the text matrices (BT, Tm, Td,
  TD, T*, TL, Tf, Tc, Tw, Tz, Ts) and the string operators (Tj, TJ, ', "); glyph widths come
  from the font's /Widths when it has them, else 0.5 em;
* ``lines`` — stroked ruling segments (``l`` segments and ``re`` rectangle edges that are
  painted by S / s / B / b, axis-aligned), the input of ruled-table detection;
* ``images`` — every image XObject placed by ``Do`` with its placed box and its pixels decoded
  by the image dictionary: /DCTDecode (JPEG) or /FlateDecode with /Width /Height
  /BitsPerComponent /ColorSpace (DeviceGray / DeviceRGB / DeviceCMYK / Indexed / ICCBased by
  component count) and PNG predictors (/DecodeParms /Predictor >= 10).

Object streams (/Type /ObjStm) are read, so files written by current tools parse too.
Encrypted PDFs, Type3 glyph procedures and shading patterns are out of scope.
"""
from __future__ import annotations

import io
import re
import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

# ------------------------------------------------------------------------- object model


class Ref(tuple):
    """Indirect reference (num, gen)."""


class Name(str):
    pass


_WS = b" \t\r\n\x0c\x00"
_DELIM = b"()<>[]{}/%"


def _skip_ws(s: bytes, i: int) -> int:
    n = len(s)
    while i < n:
        c = s[i]
        if c in _WS:
            i += 1
        elif c == 0x25:  # % comment
            while i < n and s[i] not in b"\r\n":
                i += 1
        else:
            break
    return i


def _literal(s: bytes, i: int) -> Tuple[bytes, int]:
    """(string) starting at s[i] == '('."""
    out = bytearray()
    depth = 1
    i += 1
    esc = {ord("n"): 10, ord("r"): 13, ord("t"): 9, ord("b"): 8, ord("f"): 12}
    while i < len(s) and depth:
        c = s[i]
        if c == 0x5C:
            i += 1
            if i >= len(s):
                break
            e = s[i]
            if e in esc:
                out.append(esc[e])
            elif 0x30 <= e <= 0x37:
                j = i
                while j < min(i + 3, len(s)) and 0x30 <= s[j] <= 0x37:
                    j += 1
                out.append(int(s[i:j], 8) & 0xFF)
                i = j - 1
            elif e == 13:
                if i + 1 < len(s) and s[i + 1] == 10:
                    i += 1
            elif e != 10:
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


def _token(s: bytes, i: int):
    """Next raw token: returns (kind, value, next index); kind in num, name, str, hex, kw,
    '[', ']', '<<', '>>', or None at the end."""
    i = _skip_ws(s, i)
    n = len(s)
    if i >= n:
        return None, None, i
    c = s[i]
    if c == 0x2F:  # /name
        j = i + 1
        while j < n and s[j] not in _WS and s[j] not in _DELIM:
            j += 1
        raw = s[i + 1:j]
        nm = re.sub(rb"#([0-9a-fA-F]{2})", lambda m: bytes([int(m.group(1), 16)]), raw)
        return "name", Name(nm.decode("latin-1")), j
    if c == 0x28:
        v, j = _literal(s, i)
        return "str", v, j
    if c == 0x3C:
        if i + 1 < n and s[i + 1] == 0x3C:
            return "<<", None, i + 2
        j = s.find(b">", i)
        j = n if j < 0 else j
        hx = re.sub(rb"\s", b"", s[i + 1:j])
        if len(hx) % 2:
            hx += b"0"
        try:
            v = bytes.fromhex(hx.decode("latin-1"))
        except ValueError:
            v = b""
        return "hex", v, j + 1
    if c == 0x3E and i + 1 < n and s[i + 1] == 0x3E:
        return ">>", None, i + 2
    if c in b"[]{}":
        return chr(c), None, i + 1
    j = i
    while j < n and s[j] not in _WS and s[j] not in _DELIM:
        j += 1
    if j == i:   # stray delimiter
        return "kw", chr(c), i + 1
    w = s[i:j]
    if re.fullmatch(rb"[+-]?(\d+\.?\d*|\.\d+)", w):
        return "num", float(w) if b"." in w else int(w), j
    return "kw", w.decode("latin-1"), j


def parse_value(s: bytes, i: int = 0):
    """One PDF object at s[i]: returns (value, next index). Dicts -> dict, arrays -> list,
    ``n g R`` -> Ref, names -> Name, strings -> bytes, numbers, booleans, None."""
    kind, v, j = _token(s, i)
    if kind is None:
        return None, j
    if kind == "<<":
        d = {}
        while True:
            k2, key, j2 = _token(s, j)
            if k2 in (">>", None):
                return d, j2
            if k2 != "name":
                j = j2
                continue
            val, j = parse_value(s, j2)
            d[str(key)] = val
    if kind == "[":
        arr = []
        while True:
            k2, _, j2 = _token(s, j)
            if k2 in ("]", None):
                return arr, j2
            val, j = parse_value(s, j)
            arr.append(val)
    if kind == "num" and isinstance(v, int):
        # "n g R" reference?
        k2, v2, j2 = _token(s, j)
        if k2 == "num" and isinstance(v2, int):
            k3, v3, j3 = _token(s, j2)
            if k3 == "kw" and v3 == "R":
                return Ref((v, v2)), j3
        return v, j
    if kind == "kw":
        if v == "true":
            return True, j
        if v == "false":
            return False, j
        if v == "null":
            return None, j
        return v, j
    return v, j


_OBJ_RE = re.compile(rb"(\d+)\s+(\d+)\s+obj\b")


class PdfDocument:
    """Objects of a PDF file (classic ``n g obj`` bodies plus object streams), resolvable
    by reference, and the page list."""

    def __init__(self, data: bytes):
        self.data = data
        self.objs: Dict[int, object] = {}
        self.streams: Dict[int, bytes] = {}   # raw (still encoded) stream bytes of stream objects
        for m in _OBJ_RE.finditer(data):
            num = int(m.group(1))
            try:
                val, j = parse_value(data, m.end())
            except (RecursionError, ValueError, IndexError):
                continue
            self.objs[num] = val
            if isinstance(val, dict):
                k = _skip_ws(data, j)
                if data.startswith(b"stream", k):
                    k += 6
                    if data[k:k + 2] == b"\r\n":
                        k += 2
                    elif data[k:k + 1] in (b"\n", b"\r"):
                        k += 1
                    ln = self.resolve(val.get("Length"))
                    end = -1
                    if isinstance(ln, int) and data[k + ln:k + ln + 30].lstrip().startswith(b"endstream"):
                        end = k + ln
                    if end < 0:
                        end = data.find(b"endstream", k)
                        while end > k and data[end - 1] in b"\r\n":
                            end -= 1
                    self.streams[num] = data[k:end]
        for num, val in list(self.objs.items()):
            if isinstance(val, dict) and val.get("Type") == "ObjStm" and num in self.streams:
                self._read_objstm(num, val)

    def _read_objstm(self, num: int, d: dict) -> None:
        try:
            raw = self.stream_data(num)
        except Exception:  # noqa: BLE001
            return
        n, first = int(d.get("N", 0)), int(d.get("First", 0))
        head = raw[:first].split()
        for k in range(min(n, len(head) // 2)):
            onum, off = int(head[2 * k]), int(head[2 * k + 1])
            if onum not in self.objs:
                try:
                    self.objs[onum] = parse_value(raw, first + off)[0]
                except (RecursionError, ValueError, IndexError):
                    pass

    def resolve(self, v, depth: int = 0):
        while isinstance(v, Ref) and depth < 32:
            v = self.objs.get(v[0])
            depth += 1
        return v

    def stream_data(self, num: int, decode_images: bool = False) -> bytes:
        """Decoded bytes of stream object ``num`` (FlateDecode with predictors; image codecs
        such as DCTDecode are left encoded unless nothing else is in the chain)."""
        d = self.objs.get(num)
        raw = self.streams.get(num, b"")
        if not isinstance(d, dict):
            return raw
        filters = self.resolve(d.get("Filter"))
        parms = self.resolve(d.get("DecodeParms"))
        if not isinstance(filters, list):
            filters = [filters] if filters else []
        if not isinstance(parms, list):
            parms = [parms] * len(filters)
        data = raw
        for f, p in zip(filters, parms):
            p = self.resolve(p) or {}
            if f in ("FlateDecode", "Fl"):
                data = _inflate(data)
                pred = int(p.get("Predictor", 1)) if isinstance(p, dict) else 1
                if pred >= 10:
                    data = _png_unpredict(data, int(p.get("Colors", 1)), int(p.get("BitsPerComponent", 8)),
                                          int(p.get("Columns", 1)))
            elif f in ("ASCIIHexDecode", "AHx"):
                data = bytes.fromhex(re.sub(rb"[^0-9a-fA-F]", b"", data.split(b">")[0]).decode() + "")
            else:   # DCTDecode, JPXDecode, ...: image codecs, returned as stored
                break
        return data

    def pages(self) -> List[Tuple[int, dict, dict]]:
        """(object number, page dict, inherited attributes) in document order."""
        root = None
        for v in self.objs.values():
            if isinstance(v, dict) and v.get("Type") == "Catalog":
                root = v
                break
        out: List[Tuple[int, dict, dict]] = []
        seen = set()

        def walk(ref, inherit, depth=0):
            if depth > 64 or not isinstance(ref, Ref) or ref[0] in seen:
                return
            seen.add(ref[0])
            node = self.resolve(ref)
            if not isinstance(node, dict):
                return
            inh = dict(inherit)
            for k in ("Resources", "MediaBox", "CropBox", "Rotate"):
                if k in node:
                    inh[k] = node[k]
            if node.get("Type") == "Pages" or "Kids" in node:
                for kid in self.resolve(node.get("Kids")) or []:
                    walk(kid, inh, depth + 1)
            else:
                out.append((ref[0], node, inh))

        if root is not None:
            walk(root.get("Pages"), {})
        if not out:   # no usable page tree: every /Type /Page object in file order
            for num, v in sorted(self.objs.items()):
                if isinstance(v, dict) and v.get("Type") == "Page":
                    out.append((num, v, {}))
        return out


def _inflate(data: bytes) -> bytes:
    try:
        return zlib.decompress(data)
    except zlib.error:
        try:
            return zlib.decompressobj().decompress(data)
        except zlib.error:
            return b""


def _png_unpredict(data: bytes, colors: int, bpc: int, columns: int) -> bytes:
    """Undo PNG row filters (PDF /Predictor 10-15: a filter-type byte per row)."""
    bpp = max(1, colors * bpc // 8)
    row = (colors * bpc * columns + 7) // 8
    out = bytearray()
    prev = bytearray(row)
    i = 0
    while i + row + 1 <= len(data):
        ft = data[i]
        cur = bytearray(data[i + 1:i + 1 + row])
        for x in range(row):
            a = cur[x - bpp] if x >= bpp else 0
            b = prev[x]
            c = prev[x - bpp] if x >= bpp else 0
            if ft == 1:
                cur[x] = (cur[x] + a) & 0xFF
            elif ft == 2:
                cur[x] = (cur[x] + b) & 0xFF
            elif ft == 3:
                cur[x] = (cur[x] + ((a + b) >> 1)) & 0xFF
            elif ft == 4:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                cur[x] = (cur[x] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)) & 0xFF
        out += cur
        prev = cur
        i += row + 1
    return bytes(out)


# ------------------------------------------------------------------------- page content
@dataclass
class PdfChar:
    text: str
    x0: float
    x1: float
    top: float
    bottom: float
    size: float


@dataclass
class PdfLine:
    x0: float
    top: float
    x1: float
    bottom: float

    @property
    def horizontal(self) -> bool:
        return abs(self.bottom - self.top) <= 1.0


@dataclass
class PdfImage:
    name: str
    x0: float
    top: float
    x1: float
    bottom: float
    src_width: int
    src_height: int
    pil: Optional[object] = None      # decoded PIL image (None when the codec is unsupported)

    @property
    def width(self) -> float:
        return self.x1 - self.x0

    @property
    def height(self) -> float:
        return self.bottom - self.top


@dataclass
class PdfPage:
    number: int
    width: float
    height: float
    chars: List[PdfChar] = field(default_factory=list)
    lines: List[PdfLine] = field(default_factory=list)
    images: List[PdfImage] = field(default_factory=list)


def _mul(m, n):
    a, b, c, d, e, f = m
    A, B, C, D, E, F = n
    return (a * A + b * C, a * B + b * D, c * A + d * C, c * B + d * D, e * A + f * C + E, e * B + f * D + F)


def _apply(m, x, y):
    a, b, c, d, e, f = m
    return a * x + c * y + e, b * x + d * y + f


def decode_image(doc: PdfDocument, num: int, d: dict):
    """PIL image of image XObject ``num`` (dictionary ``d``), or None."""
    from PIL import Image

    filters = doc.resolve(d.get("Filter"))
    flist = filters if isinstance(filters, list) else ([filters] if filters else [])
    try:
        if "DCTDecode" in flist or "DCT" in flist:
            data = doc.stream_data(num)   # non-image filters before DCT are undone
            return Image.open(io.BytesIO(data)).convert("RGB")
        if any(f not in ("FlateDecode", "Fl", "ASCIIHexDecode", "AHx") for f in flist):
            return None   # JPX / JBIG2 / CCITT: not decoded here
        data = doc.stream_data(num)
        w, h = int(doc.resolve(d.get("Width"))), int(doc.resolve(d.get("Height")))
        bpc = int(doc.resolve(d.get("BitsPerComponent", 8)) or 8)
        cs = doc.resolve(d.get("ColorSpace", "DeviceGray"))
        palette = None
        if isinstance(cs, list) and cs and cs[0] == "Indexed":
            base = doc.resolve(cs[1])
            lookup = doc.resolve(cs[3])
            if isinstance(lookup, Ref):
                lookup = doc.stream_data(lookup[0])
            elif isinstance(cs[3], Ref) and cs[3][0] in doc.streams:
                lookup = doc.stream_data(cs[3][0])
            ncomp = _components(doc, base)
            palette = (bytes(lookup) if isinstance(lookup, (bytes, bytearray)) else b"", ncomp)
            comps = 1
        else:
            comps = _components(doc, cs)
        if bpc != 8 and not (palette and bpc in (1, 2, 4)) and not (comps == 1 and bpc == 1):
            return None
        if palette:
            raw = _unpack_bits(data, w, h, bpc) if bpc != 8 else data[: w * h]
            lut, nc = palette
            px = bytearray()
            for v in raw:
                entry = lut[v * nc: v * nc + nc]
                px += entry.ljust(nc, b"\x00")
            mode = {1: "L", 3: "RGB", 4: "CMYK"}.get(nc)
            if mode is None:
                return None
            return Image.frombytes(mode, (w, h), bytes(px)).convert("RGB")
        if comps == 1 and bpc == 1:
            return Image.frombytes("1", (w, h), data[: ((w + 7) // 8) * h]).convert("RGB")
        mode = {1: "L", 3: "RGB", 4: "CMYK"}.get(comps)
        if mode is None or len(data) < w * h * comps:
            return None
        img = Image.frombytes(mode, (w, h), data[: w * h * comps])
        if mode == "CMYK" and "Adobe" not in str(d.get("Decode", "")):
            pass
        return img.convert("RGB")
    except Exception:  # noqa: BLE001 - an undecodable image is skipped, not fatal
        return None


def _unpack_bits(data: bytes, w: int, h: int, bpc: int) -> bytes:
    out = bytearray()
    per = 8 // bpc
    rowb = (w * bpc + 7) // 8
    mask = (1 << bpc) - 1
    for y in range(h):
        row = data[y * rowb:(y + 1) * rowb]
        vals = []
        for byte in row:
            for k in range(per):
                vals.append((byte >> (8 - bpc * (k + 1))) & mask)
        out += bytes(vals[:w])
    return bytes(out)


def _components(doc: PdfDocument, cs) -> int:
    cs = doc.resolve(cs)
    if isinstance(cs, str):
        return {"DeviceGray": 1, "G": 1, "CalGray": 1, "DeviceRGB": 3, "RGB": 3, "CalRGB": 3,
                "DeviceCMYK": 4, "CMYK": 4, "Lab": 3}.get(cs, 3)
    if isinstance(cs, list) and cs:
        if cs[0] == "ICCBased":
            d = doc.resolve(cs[1])
            return int(d.get("N", 3)) if isinstance(d, dict) else 3
        if cs[0] in ("CalRGB", "Lab"):
            return 3
        if cs[0] == "CalGray":
            return 1
    return 3


class _Font:
    def __init__(self, doc: PdfDocument, d):
        d = doc.resolve(d) if d is not None else {}
        d = d if isinstance(d, dict) else {}
        self.first = int(doc.resolve(d.get("FirstChar", 0)) or 0)
        w = doc.resolve(d.get("Widths"))
        self.widths = [float(doc.resolve(x) or 0) for x in w] if isinstance(w, list) else None
        self.two_byte = d.get("Subtype") == "Type0"

    def width(self, code: int) -> float:
        if self.widths and 0 <= code - self.first < len(self.widths) and self.widths[code - self.first] > 0:
            return self.widths[code - self.first] / 1000.0
        return 0.5

    def decode(self, b: bytes) -> List[Tuple[str, int]]:
        if self.two_byte or b.startswith(b"\xfe\xff"):
            if b.startswith(b"\xfe\xff"):
                b = b[2:]
            return [(b[i:i + 2].decode("utf-16-be", errors="replace"), int.from_bytes(b[i:i + 2], "big"))
                    for i in range(0, len(b) - 1, 2)]
        return [(chr(c), c) for c in b]


def _ops(cs: bytes):
    """Content-stream tokens grouped as (operator, operands)."""
    operands = []
    i, n = 0, len(cs)
    while i < n:
        i = _skip_ws(cs, i)
        if i >= n:
            break
        c = cs[i]
        if c in b"/([<-+.0123456789" or (c == 0x3C):
            if c == 0x3C and i + 1 < n and cs[i + 1] == 0x3C:   # inline dict (BDC properties)
                val, i = parse_value(cs, i)
                operands.append(val)
                continue
            val, i = parse_value(cs, i)
            if isinstance(val, Ref):   # never in content streams: numbers then "R" operator
                operands.extend([val[0], val[1]])
                continue
            operands.append(val)
            continue
        kind, v, j = _token(cs, i)
        i = j
        if kind in ("]", ">>", "}", "{"):
            continue
        if v == "BI":   # inline image: skip its data up to EI
            k = cs.find(b"ID", i)
            e = re.compile(rb"[\s]EI[\s]").search(cs, k + 2 if k >= 0 else i)
            i = e.end() if e else n
            operands = []
            continue
        yield v, operands
        operands = []


def parse_pages(data: bytes, decode_images: bool = True) -> List[PdfPage]:
    doc = PdfDocument(data)
    pages = []
    for pno, (num, pd, inh) in enumerate(doc.pages()):
        box = doc.resolve(pd.get("MediaBox", inh.get("MediaBox"))) or [0, 0, 612, 792]
        box = [float(doc.resolve(v) or 0) for v in box]
        x_off, y_off = box[0], box[1]
        W, H = box[2] - box[0], box[3] - box[1]
        page = PdfPage(pno, W, H)
        res = doc.resolve(pd.get("Resources", inh.get("Resources"))) or {}
        contents = doc.resolve(pd.get("Contents"))
        refs = contents if isinstance(contents, list) else [pd.get("Contents")]
        cs = b"\n".join(doc.stream_data(r[0]) for r in refs if isinstance(r, Ref))
        _interpret(doc, cs, res, page, (1, 0, 0, 1, -x_off, -y_off), decode_images, 0)
        pages.append(page)
    return pages


def _interpret(doc, cs, res, page: PdfPage, ctm0, decode_images: bool, depth: int) -> None:
    if depth > 8:
        return
    H = page.height
    fonts = doc.resolve(res.get("Font")) if isinstance(res, dict) else None
    xobjs = doc.resolve(res.get("XObject")) if isinstance(res, dict) else None
    fonts = fonts if isinstance(fonts, dict) else {}
    xobjs = xobjs if isinstance(xobjs, dict) else {}
    font_cache: Dict[str, _Font] = {}
    ctm = ctm0
    stack = []
    tm = tlm = (1, 0, 0, 1, 0, 0)
    fs, font, tl, tc, tw, th, rise = 12.0, _Font(doc, None), 0.0, 0.0, 0.0, 1.0, 0.0
    path: List[Tuple[float, float, float, float]] = []   # user-space segments of the current path
    cur = start = None

    def show(s: bytes):
        nonlocal tm
        for ch, code in font.decode(s):
            trm = _mul((fs * th, 0, 0, fs, 0, rise), _mul(tm, ctm))
            w = font.width(code)
            x, y = trm[4], trm[5]
            sx = (trm[0] ** 2 + trm[1] ** 2) ** 0.5 / max(th, 1e-6)
            sy = (trm[2] ** 2 + trm[3] ** 2) ** 0.5
            size = sy if sy > 0 else fs
            if ch.strip() or ch == " ":
                page.chars.append(PdfChar(ch, x, x + w * sx * th, H - (y + 0.8 * size), H - (y - 0.2 * size), size))
            adv = (w * fs + tc + (tw if code == 32 else 0.0)) * th
            tm = _mul((1, 0, 0, 1, adv, 0), tm)

    for op, a in _ops(cs):
        try:
            if op == "q":
                stack.append(ctm)
            elif op == "Q":
                if stack:
                    ctm = stack.pop()
            elif op == "cm" and len(a) == 6:
                ctm = _mul(tuple(float(v) for v in a), ctm)
            elif op == "BT":
                tm = tlm = (1, 0, 0, 1, 0, 0)
            elif op == "Tf" and len(a) == 2:
                fs = float(a[1])
                key = str(a[0])
                if key not in font_cache:
                    font_cache[key] = _Font(doc, fonts.get(key))
                font = font_cache[key]
            elif op == "Tm" and len(a) == 6:
                tm = tlm = tuple(float(v) for v in a)
            elif op in ("Td", "TD") and len(a) == 2:
                if op == "TD":
                    tl = -float(a[1])
                tm = tlm = _mul((1, 0, 0, 1, float(a[0]), float(a[1])), tlm)
            elif op == "T*":
                tm = tlm = _mul((1, 0, 0, 1, 0, -tl), tlm)
            elif op == "TL" and a:
                tl = float(a[0])
            elif op == "Tc" and a:
                tc = float(a[0])
            elif op == "Tw" and a:
                tw = float(a[0])
            elif op == "Tz" and a:
                th = float(a[0]) / 100.0
            elif op == "Ts" and a:
                rise = float(a[0])
            elif op == "Tj" and a and isinstance(a[-1], bytes):
                show(a[-1])
            elif op in ("'", '"') and a and isinstance(a[-1], bytes):
                if op == '"' and len(a) == 3:
                    tw, tc = float(a[0]), float(a[1])
                tm = tlm = _mul((1, 0, 0, 1, 0, -tl), tlm)
                show(a[-1])
            elif op == "TJ" and a and isinstance(a[-1], list):
                for el in a[-1]:
                    if isinstance(el, bytes):
                        show(el)
                    elif isinstance(el, (int, float)):
                        tm = _mul((1, 0, 0, 1, -float(el) / 1000.0 * fs * th, 0), tm)
            elif op == "m" and len(a) == 2:
                cur = start = _apply(ctm, float(a[0]), float(a[1]))
            elif op == "l" and len(a) == 2 and cur is not None:
                p = _apply(ctm, float(a[0]), float(a[1]))
                path.append((cur[0], cur[1], p[0], p[1]))
                cur = p
            elif op in ("c", "v", "y"):
                if len(a) >= 2:
                    cur = _apply(ctm, float(a[-2]), float(a[-1]))
            elif op == "h" and cur is not None and start is not None:
                path.append((cur[0], cur[1], start[0], start[1]))
                cur = start
            elif op == "re" and len(a) == 4:
                x, y, w, h = (float(v) for v in a)
                pts = [_apply(ctm, x, y), _apply(ctm, x + w, y), _apply(ctm, x + w, y + h), _apply(ctm, x, y + h)]
                for k in range(4):
                    path.append((*pts[k], *pts[(k + 1) % 4]))
                cur = start = pts[0]
            elif op in ("S", "s", "B", "B*", "b", "b*", "f", "F", "f*", "n"):
                if op in ("S", "s", "B", "B*", "b", "b*"):
                    for x0, y0, x1, y1 in path:
                        if abs(y0 - y1) <= 1.0 or abs(x0 - x1) <= 1.0:
                            page.lines.append(PdfLine(min(x0, x1), H - max(y0, y1), max(x0, x1), H - min(y0, y1)))
                elif op in ("f", "F", "f*"):
                    # thin filled rectangles are drawn rules too (common table borders)
                    xs = [p[0] for p in path] + [p[2] for p in path]
                    ys = [p[1] for p in path] + [p[3] for p in path]
                    if xs and (max(ys) - min(ys) <= 2.0 or max(xs) - min(xs) <= 2.0):
                        page.lines.append(PdfLine(min(xs), H - max(ys), max(xs), H - min(ys)))
                path = []
                cur = start = None
            elif op == "Do" and a:
                ref = xobjs.get(str(a[0]))
                xo = doc.resolve(ref)
                if not isinstance(xo, dict) or not isinstance(ref, Ref):
                    continue
                if xo.get("Subtype") == "Image":
                    corners = [_apply(ctm, u, v) for u, v in ((0, 0), (1, 0), (0, 1), (1, 1))]
                    xs, ys = [p[0] for p in corners], [p[1] for p in corners]
                    pil = decode_image(doc, ref[0], xo) if decode_images else None
                    page.images.append(PdfImage(str(a[0]), min(xs), H - max(ys), max(xs), H - min(ys),
                                                int(doc.resolve(xo.get("Width", 0)) or 0),
                                                int(doc.resolve(xo.get("Height", 0)) or 0), pil))
                elif xo.get("Subtype") == "Form":
                    m = doc.resolve(xo.get("Matrix")) or [1, 0, 0, 1, 0, 0]
                    sub_res = doc.resolve(xo.get("Resources")) or res
                    _interpret(doc, doc.stream_data(ref[0]), sub_res, page,
                               _mul(tuple(float(v) for v in m), ctm), decode_images, depth + 1)
        except (TypeError, ValueError, ZeroDivisionError):
            continue   # malformed operands: skip the operator, keep the page


# ------------------------------------------------------------------------- layout helpers
@dataclass
class TextLine:
    text: str
    x0: float
    x1: float
    top: float
    bottom: float


def text_lines(chars: List[PdfChar]) -> List[TextLine]:
    """Chars -> reading-order lines (same baseline band, left to right), with a space where
    the gap between glyphs exceeds 0.25 em."""
    if not chars:
        return []
    cs = sorted(chars, key=lambda c: (round(c.bottom, 0), c.x0))
    rows: List[List[PdfChar]] = []
    for c in cs:
        if rows and abs(rows[-1][-1].bottom - c.bottom) <= 0.3 * max(c.size, 1.0):
            rows[-1].append(c)
        else:
            rows.append([c])
    out = []
    for r in rows:
        r.sort(key=lambda c: c.x0)
        parts = [r[0].text]
        for p, c in zip(r, r[1:]):
            if c.x0 - p.x1 > 0.25 * max(c.size, 1.0) and not parts[-1].endswith(" ") and c.text != " ":
                parts.append(" ")
            parts.append(c.text)
        txt = re.sub(r"\s+", " ", "".join(parts)).strip()
        if txt:
            out.append(TextLine(txt, min(c.x0 for c in r), max(c.x1 for c in r), min(c.top for c in r),
                                max(c.bottom for c in r)))
    out.sort(key=lambda ln: (ln.top, ln.x0))
    return out


@dataclass
class Table:
    bbox: Tuple[float, float, float, float]   # x0, top, x1, bottom
    rows: List[List[str]]
    lines: List[PdfLine]


def _cluster(vals: List[float], tol: float) -> List[float]:
    out: List[List[float]] = []
    for v in sorted(vals):
        if out and v - out[-1][-1] <= tol:
            out[-1].append(v)
        else:
            out.append([v])
    return [sum(g) / len(g) for g in out]


def find_tables(page: PdfPage, tol: float = 3.0) -> List[Table]:
    """Ruled tables (pdfplumber's ``lines_strict`` strategy: only drawn rules count): the
    stroked horizontal and vertical segments are grouped into connected components; each
    component with >= 3 horizontal and >= 2 vertical rule positions (>= 2 rows x 1 column of
    cells, or 1 x 2) becomes a grid whose cells take the text whose centre they contain."""
    hs = [ln for ln in page.lines if ln.horizontal and ln.x1 - ln.x0 > tol]
    vs = [ln for ln in page.lines if not ln.horizontal and ln.bottom - ln.top > tol]
    segs = hs + vs
    if len(hs) < 2 or len(vs) < 2:
        return []
    parent = list(range(len(segs)))

    def find(i):
        while parent[i] != i:
            parent[i] = parent[parent[i]]
            i = parent[i]
        return i

    def touch(a: PdfLine, b: PdfLine) -> bool:
        return (a.x0 - tol <= b.x1 and b.x0 - tol <= a.x1 and a.top - tol <= b.bottom and b.top - tol <= a.bottom)

    for i in range(len(segs)):
        for j in range(i + 1, len(segs)):
            if touch(segs[i], segs[j]):
                parent[find(i)] = find(j)
    groups: Dict[int, List[PdfLine]] = {}
    for i, s in enumerate(segs):
        groups.setdefault(find(i), []).append(s)
    tables = []
    for g in groups.values():
        gh = [s for s in g if s.horizontal]
        gv = [s for s in g if not s.horizontal]
        ys = _cluster([s.top for s in gh], tol)
        xs = _cluster([s.x0 for s in gv], tol)
        if len(ys) < 2 or len(xs) < 2 or (len(ys) - 1) * (len(xs) - 1) < 2:
            continue
        rows = []
        for r in range(len(ys) - 1):
            row = []
            for c in range(len(xs) - 1):
                cell = [ch for ch in page.chars
                        if xs[c] <= (ch.x0 + ch.x1) / 2 <= xs[c + 1] and ys[r] <= (ch.top + ch.bottom) / 2 <= ys[r + 1]]
                row.append(" ".join(ln.text for ln in text_lines(cell)))
            rows.append(row)
        tables.append(Table((xs[0], ys[0], xs[-1], ys[-1]), rows, g))
    tables.sort(key=lambda t: (t.bbox[1], t.bbox[0]))
    return tables


def render_region(page: PdfPage, bbox, dpi: int = 109, lines: Optional[List[PdfLine]] = None):
    """Rasterise a page region (drawn rules, text, placed images) to a PIL RGB image at
    ``dpi`` — the table picture DePlot reads (the reference crops the rendered page at 109 dpi:
    custom_pdf_parser.py:190-193)."""
    from PIL import Image, ImageDraw, ImageFont

    s = dpi / 72.0
    x0, top, x1, bottom = bbox
    W, H = max(1, int((x1 - x0) * s) + 2), max(1, int((bottom - top) * s) + 2)
    img = Image.new("RGB", (W, H), "white")
    for im in page.images:
        if im.pil is None or im.x1 < x0 or im.x0 > x1 or im.bottom < top or im.top > bottom:
            continue
        w, h = max(1, int(im.width * s)), max(1, int(im.height * s))
        img.paste(im.pil.resize((w, h)), (int((im.x0 - x0) * s), int((im.top - top) * s)))
    d = ImageDraw.Draw(img)
    for ln in (lines if lines is not None else page.lines):
        d.line([((ln.x0 - x0) * s, (ln.top - top) * s), ((ln.x1 - x0) * s, (ln.bottom - top) * s)],
               fill="black", width=max(1, int(s)))
    font = ImageFont.load_default()
    for tl in text_lines([c for c in page.chars if x0 <= c.x0 <= x1 and top <= c.top <= bottom]):
        d.text(((tl.x0 - x0) * s, (tl.top - top) * s), tl.text, fill="black", font=font)
    return img
