"""Multimodal ingestion parity (reference RetrievalAugmentedGeneration/
examples/multimodal_rag/vectorstore/custom_pdf_parser.py, custom_powerpoint_parser.py) on
generated PDFs / PPTX: Flate images decoded by their dictionary and re-encoded JPEG q=20, the
5 %-of-page size filter and the caption rule, header/footer crop, ruled tables through DePlot
+ the LLM as table documents, PPTX speaker notes, and the OCR fallback for text-less pages."""
import io
import os
import zipfile
import zlib

import pytest
from PIL import Image

from nv_genai_amd.examples.multimodal_rag import parsers
from nv_genai_amd.rag import pdf_layout as pl


# ------------------------------------------------------------------ PDF writer for the tests
def _png_predict(raw: bytes, row: int) -> bytes:
    """PNG 'Up' filter on every row (Predictor 12 family; the decoder handles all five)."""
    out = bytearray()
    prev = bytes(row)
    for y in range(len(raw) // row):
        cur = raw[y * row:(y + 1) * row]
        out.append(2)
        out += bytes((c - p) & 0xFF for c, p in zip(cur, prev))
        prev = cur
    return bytes(out)


def _gradient(w, h):
    im = Image.new("RGB", (w, h))
    im.putdata([((x * 255) // max(1, w - 1), (y * 255) // max(1, h - 1), 128) for y in range(h) for x in range(w)])
    return im


def make_pdf(pages):
    """pages: list of dicts {"ops": [content lines], "images": {name: (kind, PIL image)}}; kind
    "flate" (FlateDecode RGB + PNG predictor), "flate-gray" or "dct" (JPEG)."""
    objs = {}
    nxt = [4]

    def new(body: bytes) -> int:
        n = nxt[0]
        nxt[0] += 1
        objs[n] = body
        return n

    kids = []
    for pg in pages:
        xo = {}
        for name, (kind, im) in pg.get("images", {}).items():
            w, h = im.size
            if kind == "dct":
                buf = io.BytesIO()
                im.save(buf, format="JPEG", quality=90)
                data = buf.getvalue()
                d = f"<< /Type /XObject /Subtype /Image /Width {w} /Height {h} /ColorSpace /DeviceRGB " \
                    f"/BitsPerComponent 8 /Filter /DCTDecode /Length {len(data)} >>"
            elif kind == "flate-gray":
                data = zlib.compress(im.convert("L").tobytes())
                d = f"<< /Type /XObject /Subtype /Image /Width {w} /Height {h} /ColorSpace /DeviceGray " \
                    f"/BitsPerComponent 8 /Filter /FlateDecode /Length {len(data)} >>"
            else:
                data = zlib.compress(_png_predict(im.convert("RGB").tobytes(), 3 * w))
                d = f"<< /Type /XObject /Subtype /Image /Width {w} /Height {h} /ColorSpace /DeviceRGB " \
                    f"/BitsPerComponent 8 /Filter /FlateDecode /DecodeParms << /Predictor 12 /Colors 3 " \
                    f"/BitsPerComponent 8 /Columns {w} >> /Length {len(data)} >>"
            xo[name] = new(d.encode() + b"\nstream\n" + data + b"\nendstream")
        cs = zlib.compress("\n".join(pg["ops"]).encode("latin-1"))
        cid = new(b"<< /Length %d /Filter /FlateDecode >>\nstream\n" % len(cs) + cs + b"\nendstream")
        xres = " ".join(f"/{k} {v} 0 R" for k, v in xo.items())
        pid = new(f"<< /Type /Page /Parent 2 0 R /MediaBox [0 0 612 792] /Resources << /Font << /F1 3 0 R >> "
                  f"/XObject << {xres} >> >> /Contents {cid} 0 R >>".encode())
        kids.append(pid)
    objs[1] = b"<< /Type /Catalog /Pages 2 0 R >>"
    objs[2] = f"<< /Type /Pages /Kids [{' '.join(f'{k} 0 R' for k in kids)}] /Count {len(kids)} >>".encode()
    objs[3] = b"<< /Type /Font /Subtype /Type1 /BaseFont /Helvetica >>"
    buf = io.BytesIO()
    buf.write(b"%PDF-1.5\n")
    offs = {}
    for oid in sorted(objs):
        offs[oid] = buf.tell()
        buf.write(f"{oid} 0 obj\n".encode() + objs[oid] + b"\nendobj\n")
    x = buf.tell()
    n = max(objs) + 1
    buf.write(f"xref\n0 {n}\n0000000000 65535 f \n".encode())
    for oid in range(1, n):
        buf.write(f"{offs.get(oid, 0):010d} 00000 n \n".encode())
    buf.write(f"trailer << /Size {n} /Root 1 0 R >>\nstartxref\n{x}\n%%EOF\n".encode())
    return buf.getvalue()


def text(x, y, s, size=12):
    s = s.replace("\\", "\\\\").replace("(", "\\(").replace(")", "\\)")
    return f"BT /F1 {size} Tf {x} {y} Td ({s}) Tj ET"


def place(name, x, y, w, h):
    return f"q {w} 0 0 {h} {x} {y} cm /{name} Do Q"


def ruled_table(x, y_top, col_w, row_h, cells):
    """Stroked grid (re + S for the outline, l + S for inner rules) with one text per cell."""
    nr, nc = len(cells), len(cells[0])
    W, H = nc * col_w, nr * row_h
    ops = [f"{x} {y_top - H} {W} {H} re S"]
    for r in range(1, nr):
        yy = y_top - r * row_h
        ops.append(f"{x} {yy} m {x + W} {yy} l S")
    for c in range(1, nc):
        xx = x + c * col_w
        ops.append(f"{xx} {y_top} m {xx} {y_top - H} l S")
    for r, row in enumerate(cells):
        for c, s in enumerate(row):
            ops.append(text(x + c * col_w + 4, y_top - (r + 1) * row_h + 5, s, 10))
    return ops


@pytest.fixture
def refdir(tmp_path, monkeypatch):
    monkeypatch.setenv("APP_MULTIMODAL_REFDIR", str(tmp_path / "refs"))
    return tmp_path / "refs"


class Recorder:
    def __init__(self, chart=True):
        self.chart = chart
        self.seen = []

    def is_graph(self, jpeg):
        self.seen.append(("neva", jpeg))
        return self.chart

    def process_graph(self, jpeg):
        self.seen.append(("deplot", jpeg))
        return " [chart: revenue rises] "

    def ocr(self, jpeg):
        self.seen.append(("ocr", jpeg))
        return "scanned words"


def _rich_pdf():
    chart = _gradient(120, 90)
    page1 = {
        "ops": [text(72, 760, "ACME CONFIDENTIAL HEADER"),        # top 10 %: cropped
                text(72, 30, "Page 1 footer"),                   # bottom 10 %: cropped
                text(72, 700, "Quarterly report body text about widgets."),
                place("Im1", 72, 400, 240, 180),                  # 240x180 pt: kept
                text(72, 385, "Figure 1: Revenue by quarter"),    # caption under it
                place("Logo", 500, 650, 20, 20),                  # < 5 % of the page: skipped
                place("Im3", 350, 450, 200, 120),                 # large, no text nearby: skipped
                text(72, 330, "Table 1: Units by region")]
              + ruled_table(72, 320, 100, 20, [["Region", "Units"], ["North", "10"], ["South", "32"]]),
        "images": {"Im1": ("flate", chart), "Logo": ("flate", _gradient(16, 16)),
                   "Im3": ("flate-gray", _gradient(64, 40))},
    }
    page2 = {"ops": [place("Scan", 50, 100, 500, 600)], "images": {"Scan": ("dct", _gradient(100, 120))}}
    return make_pdf([page1, page2]), chart


def test_layout_reader_recovers_text_images_and_rules():
    data, chart = _rich_pdf()
    pages = pl.parse_pages(data)
    assert len(pages) == 2 and pages[0].width == 612 and pages[0].height == 792
    lines = [ln.text for ln in pl.text_lines(pages[0].chars)]
    assert "ACME CONFIDENTIAL HEADER" in lines and "Figure 1: Revenue by quarter" in lines
    ims = {im.name: im for im in pages[0].images}
    im1 = ims["Im1"]
    assert (round(im1.x0), round(im1.top), round(im1.width), round(im1.height)) == (72, 792 - 580, 240, 180)
    # the Flate + PNG-predictor RGB stream decodes to the original pixels exactly
    assert im1.pil.size == (120, 90) and im1.pil.tobytes() == chart.tobytes()
    assert ims["Im3"].pil.mode == "RGB" and ims["Im3"].pil.size == (64, 40)
    assert pages[1].images[0].pil.size == (100, 120)            # DCT
    assert len([ln for ln in pages[0].lines if ln.horizontal]) >= 4
    tabs = pl.find_tables(pages[0])
    assert len(tabs) == 1 and tabs[0].rows == [["Region", "Units"], ["North", "10"], ["South", "32"]]


def test_pdf_documents_follow_reference_rules(refdir):
    data, chart = _rich_pdf()
    path = refdir.parent / "report.pdf"
    path.write_bytes(data)
    rec = Recorder()
    pages = parsers.get_pdf_documents(str(path), rec.is_graph, rec.process_graph, ocr=rec.ocr)
    assert len(pages) == 2
    d1 = pages[0]
    texts = [d for d in d1 if d.metadata["type"] == "text"]
    body = "\n".join(d.page_content for d in texts)
    assert "Quarterly report body text" in body
    assert "HEADER" not in body and "footer" not in body              # header/footer crop
    assert "North" not in body                                        # table cells are the table's
    # exactly one image document: the captioned chart (logo too small, Im3 uncaptioned)
    imgs = [d for d in d1 if d.metadata["type"] == "image"]
    assert len(imgs) == 1
    cap = imgs[0].metadata["caption"]
    assert "Figure 1: Revenue by quarter" in cap and "[chart: revenue rises]" in cap
    assert imgs[0].page_content.startswith("This is an image with the caption: ")
    # the vision models received JPEG q=20 of the decoded chart pixels, not the raw stream
    jpegs = [b for k, b in rec.seen if k == "neva"]
    assert jpegs and all(b[:2] == b"\xff\xd8" for b in jpegs)
    got = Image.open(io.BytesIO(jpegs[0]))
    assert got.format == "JPEG" and got.size == (120, 90)
    # the ruled table: DePlot + LLM description, the reference's column / data strings
    tabs = [d for d in d1 if d.metadata["type"] == "table"]
    assert len(tabs) == 1
    t = tabs[0]
    assert t.metadata["page_num"] == 1 and os.path.exists(t.metadata["dataframe"])
    assert "Table 1: Units by region" in t.metadata["caption"] and "[chart: revenue rises]" in t.metadata["caption"]
    # text_to_table reads the grid transposed: the columns are every row's first cell
    assert "The columns are Region, North, South" in t.page_content
    assert "Region,Units,\nNorth,10,\nSouth,32,\n" in t.page_content
    assert Image.open(t.metadata["image"]).format == "JPEG"
    # page 2 has no text layer: the OCR fallback reads its picture
    d2 = pages[1]
    assert [d.metadata["type"] for d in d2] == ["image"]
    assert d2[0].page_content == "This is a page with text: scanned words"


def test_reference_table_helpers():
    grid = [["a", "b", "c"], ["1", "2", "3"]]
    assert parsers.stringify_table(grid) == "a,b,c,\n1,2,3,\n"
    cols, rows = parsers.text_to_table(grid)
    assert cols == ["a", "1"] and rows == [["b", "2"], ["c", "3"]]


def test_uncaptioned_table_takes_column_names(refdir):
    pg = {"ops": ruled_table(72, 500, 90, 18, [["k", "v"], ["x", "1"]])}
    path = refdir.parent / "t.pdf"
    path.write_bytes(make_pdf([pg]))
    rec = Recorder()
    docs = parsers.get_pdf_documents(str(path), rec.is_graph, rec.process_graph)[0]
    t = [d for d in docs if d.metadata["type"] == "table"][0]
    assert t.metadata["caption"] == "k x"


def _pptx(path, slides):
    """Minimal PPTX: presentation order, shape texts, a picture and a notes slide per slide."""
    ns = ('xmlns:a="http://schemas.openxmlformats.org/drawingml/2006/main" '
          'xmlns:p="http://schemas.openxmlformats.org/presentationml/2006/main" '
          'xmlns:r="http://schemas.openxmlformats.org/officeDocument/2006/relationships"')
    rel_ns = 'xmlns="http://schemas.openxmlformats.org/package/2006/relationships"'
    T = "http://schemas.openxmlformats.org/officeDocument/2006/relationships/"

    def sp(paras, ph=None):
        phx = f'<p:nvSpPr><p:cNvPr id="2" name="s"/><p:cNvSpPr/><p:nvPr><p:ph type="{ph}"/></p:nvPr></p:nvSpPr>' \
            if ph else '<p:nvSpPr><p:cNvPr id="2" name="s"/><p:cNvSpPr/><p:nvPr/></p:nvSpPr>'
        body = "".join(f"<a:p>{''.join(f'<a:r><a:t>{r}</a:t></a:r>' for r in p)}</a:p>" for p in paras)
        return f"<p:sp>{phx}<p:txBody>{body}</p:txBody></p:sp>"

    with zipfile.ZipFile(path, "w") as z:
        ids = "".join(f'<p:sldId id="{256 + i}" r:id="rId{i + 1}"/>' for i in range(len(slides)))
        z.writestr("ppt/presentation.xml", f"<p:presentation {ns}><p:sldIdLst>{ids}</p:sldIdLst></p:presentation>")
        # presentation order deliberately differs from file-name order
        order = list(reversed(range(len(slides))))
        z.writestr("ppt/_rels/presentation.xml.rels", f"<Relationships {rel_ns}>" + "".join(
            f'<Relationship Id="rId{i + 1}" Type="{T}slide" Target="slides/slide{order[i] + 1}.xml"/>'
            for i in range(len(slides))) + "</Relationships>")
        for i, s in enumerate(slides):
            k = order.index(i) + 1   # file number of presentation slide i
            z.writestr(f"ppt/slides/slide{k}.xml", f"<p:sld {ns}><p:cSld><p:spTree>" +
                       "".join(sp(x) for x in s["shapes"]) + "</p:spTree></p:cSld></p:sld>")
            rels = []
            if s.get("notes"):
                z.writestr(f"ppt/notesSlides/notesSlide{k}.xml", f"<p:notes {ns}><p:cSld><p:spTree>" +
                           sp([["Slide image"]], "sldImg") + sp([[s["notes"]]], "body") +
                           "</p:spTree></p:cSld></p:notes>")
                rels.append(f'<Relationship Id="rId2" Type="{T}notesSlide" Target="../notesSlides/notesSlide{k}.xml"/>')
            if s.get("image") is not None:
                buf = io.BytesIO()
                s["image"].save(buf, format="PNG")
                z.writestr(f"ppt/media/image{k}.png", buf.getvalue())
                rels.append(f'<Relationship Id="rId3" Type="{T}image" Target="../media/image{k}.png"/>')
            z.writestr(f"ppt/slides/_rels/slide{k}.xml.rels", f"<Relationships {rel_ns}>" + "".join(rels)
                       + "</Relationships>")


def test_pptx_slides_notes_and_chart_check(refdir):
    path = refdir.parent / "deck.pptx"
    _pptx(path, [{"shapes": [[["Intro ", "slide"]], [["Agenda"]]], "notes": "Say hello first"},
                 {"shapes": [[["Sales ", "chart"]]], "image": _gradient(80, 60), "notes": "Point at Q4"}])
    sl = parsers.slides(str(path))
    assert [s["text"] for s in sl] == ["Intro slide Agenda", "Sales chart"]
    assert [s["notes"] for s in sl] == ["Say hello first", "Point at Q4"]
    rec = Recorder()
    docs = parsers.process_ppt_file(str(path), rec.is_graph, rec.process_graph)
    assert [d.metadata["page_num"] for d in docs] == [0, 1]
    assert docs[0].page_content == "This is a slide with the text: Intro slide Agenda "
    assert docs[0].metadata["caption"].endswith("\n\nThe speaker notes for this slide are: Say hello first")
    assert docs[1].page_content == "This is a slide with the text: Sales chart [chart: revenue rises] "
    assert "Point at Q4" in docs[1].metadata["caption"]
    # only the slide with a picture went to the vision model, as JPEG q=20
    assert [k for k, _ in rec.seen] == ["neva", "deplot"]
    assert Image.open(io.BytesIO(rec.seen[0][1])).format == "JPEG"


def test_vision_client_never_mislabels_bytes():
    from nv_genai_amd.connectors.vision import as_web_image

    buf = io.BytesIO()
    _gradient(10, 10).save(buf, format="GIF")
    out, fmt = as_web_image(buf.getvalue())
    assert fmt == "jpeg" and Image.open(io.BytesIO(out)).format == "JPEG"
    png = io.BytesIO()
    _gradient(10, 10).save(png, format="PNG")
    assert as_web_image(png.getvalue())[1] == "png"
    with pytest.raises(ValueError):
        as_web_image(zlib.compress(b"\x00" * 300))                # a raw Flate pixel stream


def test_multimodal_example_ingests_pdf_end_to_end(refdir, monkeypatch):
    """The chain-server example ingests the generated PDF through the parsers with local
    stand-in vision models (register_local_vision) and the fake LLM, then retrieves the
    table document."""
    monkeypatch.setenv("APP_LLM_MODELENGINE", "fake")
    monkeypatch.setenv("APP_EMBEDDINGS_MODELENGINE", "hash")
    monkeypatch.setenv("APP_EMBEDDINGS_DIMENSIONS", "256")
    from nv_genai_amd.chain_server import utils
    from nv_genai_amd.connectors import vision
    from nv_genai_amd.examples.multimodal_rag.chains import MultimodalRAG

    class Neva:
        def describe(self, image, prompt="", max_tokens=0, **kw):
            assert image[:2] == b"\xff\xd8"
            return "a bar chart" if "Describe" in prompt else "ocr text"

    class Deplot:
        def describe(self, image, prompt="", max_tokens=0, **kw):
            return "Region | Units <0x0A> North | 10"

    monkeypatch.setattr(vision, "_LOCAL", {"ai-neva-22b": Neva(), "ai-google-deplot": Deplot()})
    utils.reset()
    try:
        data, _ = _rich_pdf()
        path = refdir.parent / "report.pdf"
        path.write_bytes(data)
        ex = MultimodalRAG()
        ex.ingest_docs(str(path), "report.pdf")
        assert "report.pdf" in ex.get_documents()
        hits = ex.document_search("Table 1: Units by region", 4)
        assert hits and all(h["source"] == "report.pdf" for h in hits)
    finally:
        utils.reset()
