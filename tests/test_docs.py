"""CPU: every section reference in the code and tests resolves (DESIGN.md
split into the contract and PERF_LOG.md, the per-round log).

A reference is "DESIGN.md §4.3", "DESIGN.md 4.2b", "DESIGN.md §3, §5" or "DESIGN.md "Title""
(likewise PERF_LOG.md); each must name a heading of that file (a numbered section, or words of a
heading's title)."""
import glob
import os
import re

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SOURCES = sorted(
    set(glob.glob(os.path.join(REPO, "convolutionalencdec_amd", "**", "*.*"), recursive=True)
        + glob.glob(os.path.join(REPO, "tests", "*.py")) + glob.glob(os.path.join(REPO, "tools", "*.*"))
        + glob.glob(os.path.join(REPO, "include", "*.h")) + glob.glob(os.path.join(REPO, "oracle", "*.[ch]"))
        + [os.path.join(REPO, f) for f in ("bench.py", "__graft_entry__.py", "INTEGRATION.md", "README.md")]))
SOURCES = [p for p in SOURCES if p.endswith((".py", ".hip", ".h", ".c", ".sh", ".md")) and os.path.isfile(p)
           and os.path.basename(p) != "test_docs.py"]


def headings(doc):
    """(section numbers, heading titles) of a markdown file."""
    nums, titles = set(), []
    for ln in open(os.path.join(REPO, doc), encoding="utf-8"):
        m = re.match(r"^#{2,4}\s+(.*)$", ln)
        if not m:
            continue
        t = m.group(1).strip()
        titles.append(t.lower())
        n = re.match(r"^(\d+(?:\.\d+)?[a-z]?)\.?\s", t)
        if n:
            nums.add(n.group(1))
    return nums, titles


# (a continuation after a comma needs a § or a dotted number: "§4.2b, 65,536 x 2,048 bits" is one)
REF = re.compile(r"(DESIGN|PERF_LOG)\.md,?\s*((?:§\s*\d+(?:\.\d+)?[a-z]?|\d+(?:\.\d+)?[a-z]?\b)"
                 r"(?:\s*(?:,|and)\s*(?:§\s*\d+(?:\.\d+)?[a-z]?|\d+\.\d+[a-z]?)\b)*)")
TITLE = re.compile(r"(DESIGN|PERF_LOG)\.md,?\s*\"([^\"]+)\"")


def refs():
    out = []
    for p in SOURCES:
        text = open(p, encoding="utf-8", errors="replace").read()
        text = re.sub(r"\s*\n\s*(#|//|\*)?\s*", " ", text)  # references may wrap across comment lines
        for m in REF.finditer(text):
            for n in re.findall(r"\d+(?:\.\d+)?[a-z]?", m.group(2)):
                out.append((os.path.relpath(p, REPO), m.group(1), "num", n))
        for m in TITLE.finditer(text):
            out.append((os.path.relpath(p, REPO), m.group(1), "title", m.group(2)))
    return out


def test_references_found():
    kinds = {(d, k) for _, d, k, _ in refs()}
    assert ("DESIGN", "num") in kinds and ("PERF_LOG", "num") in kinds


@pytest.mark.parametrize("doc", ["DESIGN", "PERF_LOG"])
def test_every_reference_resolves(doc):
    nums, titles = headings(doc + ".md")
    bad = []
    for src, d, kind, what in refs():
        if d != doc:
            continue
        if kind == "num" and what not in nums:
            bad.append((src, what))
        if kind == "title" and not any(what.lower() in t for t in titles):
            bad.append((src, what))
    assert not bad, f"{doc}.md references without a section: {sorted(set(bad))[:20]}"


def test_design_is_a_contract():
    """DESIGN.md stays the short contract (the log lives in PERF_LOG.md)."""
    n = sum(1 for _ in open(os.path.join(REPO, "DESIGN.md"), encoding="utf-8"))
    assert n <= 450, n
    text = open(os.path.join(REPO, "DESIGN.md"), encoding="utf-8").read()
    for must in ("Frame-length limits", "Metric formulation", "Traceback rule", "Roofline", "switches"):
        assert must in text, must
