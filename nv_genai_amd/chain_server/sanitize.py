"""HTML sanitising for user-supplied fields (the ``bleach.clean(value, strip=True)`` the
reference applies to every request field — RetrievalAugmentedGeneration/common/server.py:60-113).

Same default policy as bleach: a small allow-list of inline tags is kept (attributes other than
``href``/``title`` on ``a`` and ``title`` on abbr/acronym dropped), every other tag is removed
(its text kept), comments are removed, and text is HTML-escaped (``&`` -> ``&amp;``, ``<`` ->
``&lt;``, ``>`` -> ``&gt;``).
"""
from __future__ import annotations

import html
from html.parser import HTMLParser

ALLOWED_TAGS = {"a", "abbr", "acronym", "b", "blockquote", "code", "em", "i", "li", "ol", "strong", "ul"}
ALLOWED_ATTRS = {"a": {"href", "title"}, "abbr": {"title"}, "acronym": {"title"}}


class _Cleaner(HTMLParser):
    def __init__(self):
        super().__init__(convert_charrefs=False)
        self.out = []

    def handle_starttag(self, tag, attrs):
        if tag in ALLOWED_TAGS:
            keep = [(k, v) for k, v in attrs if k in ALLOWED_ATTRS.get(tag, set()) and v is not None]
            a = "".join(f' {k}="{html.escape(v, quote=True)}"' for k, v in keep)
            self.out.append(f"<{tag}{a}>")

    def handle_endtag(self, tag):
        if tag in ALLOWED_TAGS:
            self.out.append(f"</{tag}>")

    def handle_data(self, data):
        self.out.append(html.escape(data, quote=False))

    def handle_entityref(self, name):
        self.out.append(f"&{name};")

    def handle_charref(self, name):
        self.out.append(f"&#{name};")

    def handle_comment(self, data):
        pass

    def unknown_decl(self, data):
        pass


def clean(value: str) -> str:
    if not value or ("<" not in value and "&" not in value and ">" not in value):
        return value
    c = _Cleaner()
    c.feed(value)
    c.close()
    rest = c.rawdata if hasattr(c, "rawdata") else ""
    return "".join(c.out) + html.escape(rest, quote=False)
