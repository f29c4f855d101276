"""Offline parser for the results table the reference scrapes (layer L3).

Reference (``Main.java:60-67,86-102``): ``Jsoup.parse(body)``, first element with
CSS class ``"table table-bordered table-condensed table-striped text-center table-hover"``,
``child(0).children()`` (the rows of its first section), drop row 0 ("info row"),
then per row: ``td[0]`` parsed with ``"E, MMM d, yyyy"`` (e.g. ``"Fri, Jun 12, 2020"``),
every other cell's text taken verbatim.

Jsoup's ``hasClass`` matches a multi-word class string when it equals the whole
``class`` attribute (case-insensitive); a single word matches any class token.  The
date is parsed with an English locale explicitly (the reference used the JVM default
locale: defect D-i).  There is no network here: pass the page as a string or file.
"""
from __future__ import annotations

import datetime as _dt
import re
from html.parser import HTMLParser

import numpy as np

from ..config import REFERENCE_TABLE_CLASS
from .draws import DrawSet

_SECTIONS = ("thead", "tbody", "tfoot")


class _TableGrab(HTMLParser):
    def __init__(self, want_class: str):
        super().__init__(convert_charrefs=True)
        self.want = want_class.strip().lower()
        self.depth = 0  # nesting depth inside the matched table
        self.found = False
        self.done = False
        self.first_child: str | None = None
        self.section_depth = 0
        self.rows: list[list[str]] = []
        self.cur_row: list[str] | None = None
        self.cur_cell: list[str] | None = None
        self.in_first_section = False
        self.first_section_closed = False

    def _match(self, attrs) -> bool:
        cls = dict(attrs).get("class")
        if cls is None:
            return False
        cls_l = " ".join(cls.split()).lower()
        if " " in self.want:
            return cls_l == self.want
        return self.want in cls_l.split()

    def handle_starttag(self, tag, attrs):
        if self.done:
            return
        if not self.found:
            if tag == "table" and self._match(attrs):
                self.found = True
                self.depth = 1
            return
        if tag == "table":
            self.depth += 1
            return
        if self.depth != 1 and not (self.depth == 1):
            return
        if self.first_child is None:
            self.first_child = tag
            if tag in _SECTIONS:
                self.in_first_section = True
        if tag in _SECTIONS and self.first_child in _SECTIONS and tag != self.first_child and self.rows:
            self.first_section_closed = True
        if self.first_section_closed:
            return
        if tag == "tr":
            self.cur_row = []
        elif tag in ("td", "th") and self.cur_row is not None:
            self.cur_cell = []

    def handle_endtag(self, tag):
        if not self.found or self.done:
            return
        if tag == "table":
            self.depth -= 1
            if self.depth == 0:
                self.done = True
            return
        if tag in _SECTIONS and self.first_child == tag:
            self.first_section_closed = True
        if tag in ("td", "th") and self.cur_cell is not None and self.cur_row is not None:
            self.cur_row.append(" ".join("".join(self.cur_cell).split()))
            self.cur_cell = None
        elif tag == "tr" and self.cur_row is not None:
            self.rows.append(self.cur_row)
            self.cur_row = None

    def handle_data(self, data):
        if self.cur_cell is not None:
            self.cur_cell.append(data)


def extract_rows(html: str, table_class: str = REFERENCE_TABLE_CLASS) -> list[list[str]]:
    """Rows (cell texts) of the first section of the first matching table, info row dropped."""
    p = _TableGrab(table_class)
    p.feed(html)
    p.close()
    if not p.found:
        raise ValueError(f"no table with class {table_class!r}")  # the reference NPEs here (Main.java:62-64)
    rows = p.rows
    if not rows:
        return []
    return rows[1:]  # "Getting rid of the info row" (Main.java:66-67)


_DATE_FMT = "%a, %b %d, %Y"  # Java "E, MMM d, yyyy" in an English locale


def parse_date(text: str) -> _dt.date:
    t = " ".join(text.split())
    try:
        return _dt.datetime.strptime(t, _DATE_FMT).date()
    except ValueError:
        # tolerate full weekday/month names ("Friday, June 12, 2020")
        return _dt.datetime.strptime(t, "%A, %B %d, %Y").date()


def parse_results_table(html: str, table_class: str = REFERENCE_TABLE_CLASS) -> DrawSet:
    rows = extract_rows(html, table_class)
    nums, dates = [], []
    for cells in rows:
        if not cells:
            continue
        d = parse_date(cells[0])
        vals: list[int] = []
        for c in cells[1:]:
            vals += [int(x) for x in re.findall(r"\d+", c)]
        if len(vals) < 7:
            raise ValueError(f"row {cells!r}: expected 5 numbers + 2 stars")
        nums.append(vals[:7] + [0])
        dates.append(np.datetime64(d, "D"))
    arr = np.array(nums, dtype=np.uint8).reshape(-1, 8)
    ds = DrawSet(arr, np.array(dates, dtype="datetime64[D]"), {"source": "html"})
    # the site lists newest first; keep the site order (the reference splits in site order)
    return ds


def render_results_table(ds: DrawSet, table_class: str = REFERENCE_TABLE_CLASS) -> str:
    """Inverse of :func:`parse_results_table` — used to build offline fixtures."""
    out = [f'<html><body><table class="{table_class}"><tbody>',
           "<tr><td colspan=\"8\">Euromillions winning numbers</td></tr>"]
    for i in range(len(ds)):
        d = ds.dates[i].astype(_dt.date)
        cells = [d.strftime(_DATE_FMT)] + [str(int(v)) for v in ds.numbers[i, :7]]
        out.append("<tr>" + "".join(f"<td>{c}</td>" for c in cells) + "</tr>")
    out.append("</tbody></table></body></html>")
    return "\n".join(out)
