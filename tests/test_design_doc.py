"""DESIGN.md's quoted headline figures match the evidence they name (CPU).

DESIGN §0 holds a table between `<!-- headline -->` markers: an evidence tag (a bench line
`profiles/<tag>_bench.json`), then figures with the JSON path they come from, or the GPU test log
`profiles/<tag>_gpu_tests.txt`.  Every figure must equal its source within 1%, the tag must be the
newest evidence (the one profiles/pmc_summary.json was collected with, as tests/test_roofline.py
picks it), and no other "N GPU tests" count in DESIGN may differ from the log's.  A doc that drifts
from its evidence fails here.
"""
import json
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")
DESIGN = os.path.join(ROOT, "DESIGN.md")


def headline():
    text = open(DESIGN).read()
    m = re.search(r"<!-- headline -->(.*?)<!-- /headline -->", text, re.S)
    assert m, "DESIGN.md has no headline table"
    rows = []
    for line in m.group(1).strip().splitlines():
        cells = [c.strip() for c in line.strip().strip("|").split("|")]
        if len(cells) != 3 or cells[0] in ("Figure",) or set(cells[0]) <= set("-"):
            continue
        rows.append((cells[0], cells[1], cells[2].strip("`")))
    return rows


def gpu_tests_passed(tag):
    f = os.path.join(PROF, f"{tag}_gpu_tests.txt")
    text = open(f).read()
    m = re.findall(r"(\d+) passed", text)
    return int(m[-1]) if m else sum(1 for ln in text.splitlines() if " PASSED" in ln)


def lookup(obj, path):
    for k in path.split("."):
        obj = obj[k]
    return obj


def test_headline_figures_match_their_evidence():
    rows = headline()
    tag = dict((a, b) for a, b, _ in rows)["evidence tag"]
    bench = json.load(open(os.path.join(PROF, f"{tag}_bench.json")))
    checked = 0
    for name, value, source in rows:
        if name == "evidence tag":
            continue
        want = float(value)
        if source.endswith("_gpu_tests.txt"):
            got = gpu_tests_passed(tag)
        else:
            got = float(lookup(bench, source))
        assert abs(got - want) <= 0.01 * abs(got), f"DESIGN headline '{name}': {want} vs {got} in {tag}:{source}"
        checked += 1
    assert checked >= 5


def test_headline_tag_is_the_newest_evidence():
    """The tag is the bench line profiles/pmc_summary.json's run produced (collect_profiles.sh
    installs both from one run)."""
    tag = dict((a, b) for a, b, _ in headline())["evidence tag"]
    src = json.load(open(os.path.join(PROF, "pmc_summary.json")))["source"]
    assert src.split("/")[1] == tag, (tag, src)


def test_no_other_gpu_test_count_in_design():
    tag = dict((a, b) for a, b, _ in headline())["evidence tag"]
    n = gpu_tests_passed(tag)
    text = open(DESIGN).read()
    counts = {int(c) for c in re.findall(r"(\d+) (?:GPU )?tests(?: green| passed)?\b", text)
              if int(c) > 50}  # (counts of GPU tests; small numbers are other things)
    counts |= {int(c) for c in re.findall(r"-m gpu`?, (\d+) tests", text)}
    assert counts <= {n}, f"DESIGN quotes GPU test counts {sorted(counts)}; the evidence has {n}"
