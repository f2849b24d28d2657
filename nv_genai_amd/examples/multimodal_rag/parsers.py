"""PDF / PPTX parsing of the multimodal example — the behaviour of the reference's
``vectorstore/custom_pdf_parser.py`` and ``custom_powerpoint_parser.py``
(RetrievalAugmentedGeneration/examples/multimodal_rag/), on this framework's own layout PDF
reader (:mod:`nv_genai_amd.rag.pdf_layout`) and OOXML parts instead of pdfplumber /
python-pptx / LibreOffice.

Per PDF page (``get_pdf_documents``, ref custom_pdf_parser.py:263-310):

1. header / footer crop: text above 10 % and below 90 % of the page height is dropped
   (:285-292);
2. no text layer left -> OCR fallback (:142-165). tesseract is not installed, so the page's
   largest image goes to the vision model with a transcription prompt; parity unpinned;
3. ruled tables (pdfplumber ``lines_strict``, :167-218): cell text, the reference's
   ``text_to_table`` / ``stringify_table`` forms, a CSV under ``table_references/`` (the
   reference writes .xlsx; openpyxl is not installed), the table region rasterised at 109 dpi
   and sent through DePlot + the LLM (``process_graph``), caption = text above + description
   + text below, or the column names when the table has no adjacent text;
4. images (:221-261): skipped below 5 % of the page width or height and when no caption text
   sits next to them (logos); the rest are re-encoded to JPEG quality 20 (``get_b64_image``,
   :29-34), asked "is it a chart?" and, if so, described by DePlot + the LLM;
5. text in <= 500-character groups of lines, leaving out lines inside detected tables.

Per PPTX slide (``process_ppt_file``, custom_powerpoint_parser.py:66-106): the slide's shape
texts joined by spaces, its speaker notes (``ppt/notesSlides``), and the chart check on the
slide picture. LibreOffice is not installed, so the slide's largest embedded image stands in
for the rendered slide. As in the reference the notes go into the ``caption`` metadata, and
the page content is "This is a slide with the text: " + text + description.

The reference's ``extract_text_around_item`` compares pdfplumber char objects against mixed
bbox indices and returns single characters; this implementation does what it is named for:
the nearest text line above and below the item within 10 % of the page height.
"""
from __future__ import annotations

import csv
import io
import os
import re
import tempfile
import zipfile
from typing import Callable, List, Optional, Sequence, Tuple
from xml.etree import ElementTree

from ...index.vectorstore import Document
from ...rag import pdf_layout as pl

HEADER_FRAC, FOOTER_FRAC = 0.1, 0.9
GROUP_CHARS = 500
CHART_WORDS = ("graph", "plot", "chart")


def ref_dir(kind: str) -> str:
    """Where table / image / OCR references are written (the reference uses /tmp-data/...)."""
    base = os.environ.get("APP_MULTIMODAL_REFDIR") or os.path.join(tempfile.gettempdir(), "nga-multimodal")
    d = os.path.join(base, kind)
    os.makedirs(d, exist_ok=True)
    return d


def jpeg_q20(img) -> bytes:
    """``get_b64_image`` minus the base64: RGB, JPEG quality 20 (custom_pdf_parser.py:29-34)."""
    buf = io.BytesIO()
    img.convert("RGB").save(buf, format="JPEG", quality=20)
    return buf.getvalue()


# ------------------------------------------------------------------ reference table forms
def stringify_table(table_text: Sequence[Sequence[str]]) -> str:
    """Every cell followed by ',', one line per row (custom_pdf_parser.py:72-78)."""
    return "".join("".join(c + "," for c in row) + "\n" for row in table_text)


def text_to_table(table_text: Sequence[Sequence[str]]) -> Tuple[List[str], List[List[str]]]:
    """The reference's DataFrame construction (custom_pdf_parser.py:79-93), kept as it is:
    the column names are the FIRST CELL OF EVERY ROW and row i collects cell i of every row
    (the extracted grid is read transposed). Returns (columns, rows); a ragged grid stops
    where the reference's try block would."""
    columns = [row[0] for row in table_text if row]
    rows = []
    try:
        for i in range(1, len(table_text[0])):
            rows.append([table_text[j][i] for j in range(len(columns))])
    except (IndexError, TypeError):
        pass
    return columns, rows


# ------------------------------------------------------------------ layout helpers
def text_around(lines: List[pl.TextLine], bbox, page_height: float, frac: float = 0.1) -> Tuple[str, str]:
    """Nearest text line above (ending within frac x page height of the item's top) and
    below (starting within that distance of its bottom) that overlaps the item horizontally
    or sits within 10 % of its width of it."""
    x0, top, x1, bottom = bbox
    vt = page_height * frac
    ht = (x1 - x0) * frac
    before = after = ""
    best_b = best_a = None
    for ln in lines:
        if ln.x1 < x0 - ht or ln.x0 > x1 + ht:
            continue
        if ln.bottom <= top + 1e-6 and top - ln.bottom <= vt and (best_b is None or ln.bottom > best_b):
            best_b, before = ln.bottom, ln.text
        elif ln.top >= bottom - 1e-6 and ln.top - bottom <= vt and (best_a is None or ln.top < best_a):
            best_a, after = ln.top, ln.text
    return before, after


def group_lines(lines: List[pl.TextLine], limit: int = GROUP_CHARS) -> List[List[pl.TextLine]]:
    """Consecutive lines in groups of <= ``limit`` characters (process_text_blocks, :103-128)."""
    groups: List[List[pl.TextLine]] = []
    n = 0
    for ln in lines:
        if groups and n + len(ln.text) <= limit:
            groups[-1].append(ln)
            n += len(ln.text)
        else:
            groups.append([ln])
            n = len(ln.text)
    return groups


def _inside(ln: pl.TextLine, bbox, tol: float = 1.0) -> bool:
    x0, top, x1, bottom = bbox
    cx, cy = (ln.x0 + ln.x1) / 2, (ln.top + ln.bottom) / 2
    return x0 - tol <= cx <= x1 + tol and top - tol <= cy <= bottom + tol


# ------------------------------------------------------------------ PDF
def get_pdf_documents(path: str, is_graph: Callable[[bytes], bool], process_graph: Callable[[bytes], str],
                      ocr: Optional[Callable[[bytes], str]] = None) -> List[List[Document]]:
    """Documents of every page of the PDF at ``path`` (a list per page). ``is_graph`` /
    ``process_graph`` take JPEG bytes (NeVA's chart check; DePlot + LLM explanation); ``ocr``
    transcribes a page picture (default: no OCR documents)."""
    with open(path, "rb") as f:
        pages = pl.parse_pages(f.read())
    src = os.path.basename(path)
    out = []
    for page in pages:
        docs: List[Document] = []
        H, W = page.height, page.width
        crop_chars = [c for c in page.chars if c.top >= H * HEADER_FRAC and c.bottom <= H * FOOTER_FRAC]
        lines = pl.text_lines(crop_chars)
        if not lines and ocr is not None and page.images:
            big = max((im for im in page.images if im.pil is not None), key=lambda im: im.width * im.height,
                      default=None)
            if big is not None:
                img_path = os.path.join(ref_dir("ocr_references"), f"page{page.number}.jpg")
                data = jpeg_q20(big.pil)
                with open(img_path, "wb") as f:
                    f.write(data)
                text = ocr(data)
                docs.append(Document("This is a page with text: " + text,
                                     {"x1": 0, "y1": 0, "x2": 0, "x3": 0, "source": src, "image": img_path,
                                      "caption": text, "type": "image", "page_num": page.number}))
        tables = pl.find_tables(page)
        for tno, tb in enumerate(tables, start=1):
            columns, _rows = text_to_table(tb.rows)
            tdir = ref_dir("table_references")
            csv_path = os.path.join(tdir, f"table{tno}-page{page.number}.csv")
            with open(csv_path, "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(columns)
                w.writerows(_rows)
            before, after = text_around(lines, tb.bbox, H)
            img_path = os.path.join(tdir, f"table{tno}-page{page.number}.jpg")
            pic = pl.render_region(page, tb.bbox, 109, tb.lines)
            data = jpeg_q20(pic)
            with open(img_path, "wb") as f:
                f.write(data)
            description = process_graph(data)
            caption = before.replace("\n", " ") + description + after.replace("\n", " ")
            if not before and not after:
                caption = " ".join(columns)
            all_cols = ", ".join(columns)
            docs.append(Document("This is a table with the caption: " + caption +
                                 f"\nThe columns are {all_cols} and the table data is {stringify_table(tb.rows)}",
                                 {"x1": 0, "y1": 0, "x2": 0, "x3": 0, "source": src, "dataframe": csv_path,
                                  "image": img_path, "caption": caption, "type": "table",
                                  "page_num": page.number + 1}))
        for ino, im in enumerate(page.images):
            if im.width < W / 20 or im.height < H / 20:
                continue   # very small images
            if im.pil is None:
                continue   # codec this reader does not decode (JPX, JBIG2, CCITT)
            before, after = text_around(lines, (im.x0, im.top, im.x1, im.bottom), H)
            if not before and not after:
                continue   # no caption: likely a logo or decoration
            img_path = os.path.join(ref_dir("image_references"), f"image{ino}-page{page.number}.jpg")
            data = jpeg_q20(im.pil)
            with open(img_path, "wb") as f:
                f.write(data)
            desc = process_graph(data) if is_graph(data) else " "
            caption = before.replace("\n", " ") + desc + after.replace("\n", " ")
            docs.append(Document("This is an image with the caption: " + caption,
                                 {"x1": 0, "y1": 0, "x2": 0, "x3": 0, "source": src, "image": img_path,
                                  "caption": caption, "type": "image", "page_num": page.number}))
        body = [ln for ln in lines if not any(_inside(ln, tb.bbox) for tb in tables)]
        for grp in group_lines(body):
            h = grp[0]
            docs.append(Document("\n".join(ln.text for ln in grp),
                                 {"x1": h.x0, "y1": h.top, "x2": h.x1, "x3": h.bottom, "type": "text",
                                  "page_num": page.number, "source": src}))
        out.append(docs)
    return out


# ------------------------------------------------------------------ PPTX
_NS_A = "{http://schemas.openxmlformats.org/drawingml/2006/main}"
_NS_P = "{http://schemas.openxmlformats.org/presentationml/2006/main}"
_NS_R = "{http://schemas.openxmlformats.org/officeDocument/2006/relationships}"
_NS_REL = "{http://schemas.openxmlformats.org/package/2006/relationships}"


def _shape_texts(root) -> List[Tuple[str, Optional[str]]]:
    """(text, placeholder type) of every text-bearing shape: paragraphs joined by newlines,
    runs concatenated (python-pptx ``shape.text``)."""
    out = []
    for sp in root.iter(_NS_P + "sp"):
        body = sp.find(_NS_P + "txBody")
        if body is None:
            continue
        paras = []
        for p in body.iter(_NS_A + "p"):
            paras.append("".join(t.text or "" for t in p.iter(_NS_A + "t")))
        ph = sp.find(f"{_NS_P}nvSpPr/{_NS_P}nvPr/{_NS_P}ph")
        out.append(("\n".join(paras), ph.get("type") if ph is not None else None))
    return out


def _rels(z: zipfile.ZipFile, part: str):
    d, base = os.path.split(part)
    rp = f"{d}/_rels/{base}.rels"
    if rp not in z.namelist():
        return []
    root = ElementTree.fromstring(z.read(rp))
    res = []
    for r in root.iter(_NS_REL + "Relationship"):
        tgt = os.path.normpath(os.path.join(d, r.get("Target", ""))).replace("\\", "/")
        res.append((r.get("Type", "").rsplit("/", 1)[-1], tgt))
    return res


def slides(path: str) -> List[dict]:
    """Per slide in presentation order: text (shape texts joined by ' '), speaker notes (the
    notes slide's body placeholder), and the bytes of each embedded picture."""
    with zipfile.ZipFile(path) as z:
        names = set(z.namelist())
        order = []
        if "ppt/presentation.xml" in names:
            pres = ElementTree.fromstring(z.read("ppt/presentation.xml"))
            rels = {rid: tgt for rid, tgt in
                    ((r.get("Id"), r.get("Target")) for r in
                     ElementTree.fromstring(z.read("ppt/_rels/presentation.xml.rels")).iter(_NS_REL + "Relationship"))} \
                if "ppt/_rels/presentation.xml.rels" in names else {}
            for s in pres.iter(_NS_P + "sldId"):
                t = rels.get(s.get(_NS_R + "id"))
                if t:
                    order.append(os.path.normpath(os.path.join("ppt", t)).replace("\\", "/"))
        if not order:
            def key(n):
                m = re.search(r"(\d+)\.xml$", n)
                return int(m.group(1)) if m else 0
            order = sorted((n for n in names if re.fullmatch(r"ppt/slides/slide\d+\.xml", n)), key=key)
        out = []
        for part in order:
            if part not in names:
                continue
            texts = _shape_texts(ElementTree.fromstring(z.read(part)))
            notes, images = "", []
            for typ, tgt in _rels(z, part):
                if typ == "notesSlide" and tgt in names:
                    nt = _shape_texts(ElementTree.fromstring(z.read(tgt)))
                    notes = "\n".join(t for t, ph in nt if ph == "body")
                elif typ == "image" and tgt in names:
                    images.append(z.read(tgt))
            out.append({"text": " ".join(t for t, _ in texts), "notes": notes, "images": images})
        return out


def process_ppt_file(path: str, is_graph: Callable[[bytes], bool],
                     process_graph: Callable[[bytes], str]) -> List[Document]:
    """One document per slide (custom_powerpoint_parser.py:86-106)."""
    from PIL import Image

    src = os.path.basename(path)
    docs = []
    for num, sl in enumerate(slides(path)):
        notes = sl["notes"]
        if notes:
            notes = "\n\nThe speaker notes for this slide are: " + notes
        image_description = " "
        img_path = ""
        pics = []
        for b in sl["images"]:
            try:
                im = Image.open(io.BytesIO(b))
                im.load()
                pics.append(im)
            except Exception:  # noqa: BLE001 - EMF / WMF / unknown media: not a picture here
                continue
        if pics:
            big = max(pics, key=lambda im: im.size[0] * im.size[1])
            data = jpeg_q20(big)
            img_path = os.path.join(ref_dir("ppt_references"), f"{os.path.splitext(src)[0]}_{num:04d}.jpg")
            with open(img_path, "wb") as f:
                f.write(data)
            if is_graph(data):
                image_description = process_graph(data)
        caption = sl["text"] + image_description + notes
        docs.append(Document("This is a slide with the text: " + sl["text"] + image_description,
                             {"x1": 0, "y1": 0, "x2": 0, "x3": 0, "source": src, "image": img_path,
                              "caption": caption, "type": "image", "page_num": num}))
    return docs
