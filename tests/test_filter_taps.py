"""Tap tables of the product and of the oracle against the reference's own tables
(tests/golden/filter_taps.json, extracted from InterpolationFilter.cpp:82-100, :187-221 by
tools/extract_filter_taps.py)."""
import json
import os
import re

from helpers import GOLDEN, ROOT


def _golden():
    return json.load(open(os.path.join(GOLDEN, "filter_taps.json")))


def _parse_macro(text, name):
    lines = text[text.index("#define " + name):].splitlines()
    body = []
    for ln in lines:
        body.append(ln)
        if not ln.rstrip().endswith("\\"):
            break
    body = " ".join(body).replace("\\", "")
    return [[int(v) for v in r.split(",") if v.strip()] for r in re.findall(r"\{([^{}]*)\}", body)]


def test_product_taps_match_reference():
    g = _golden()
    text = open(os.path.join(ROOT, "vvc-extension-mm_amd", "csrc", "mm_filter.h")).read()
    assert _parse_macro(text, "MM_LUMA_TAPS_INIT") == g["luma"]
    assert _parse_macro(text, "MM_CHROMA_TAPS_INIT") == g["chroma"]


def test_oracle_taps_match_reference():
    g = _golden()
    text = open(os.path.join(ROOT, "oracle", "mm_oracle.c")).read()
    for name, key in (("LUMA", "luma"), ("CHROMA", "chroma")):
        m = re.search(r"static const int16_t " + name + r"\[\d+\]\[\d+\] = \{(.*?)\};", text, re.S)
        rows = [[int(v) for v in r.split(",") if v.strip()] for r in re.findall(r"\{([^{}]*)\}", m.group(1))]
        assert rows == g[key]


def test_taps_sum_to_64():
    g = _golden()
    assert all(sum(r) == 64 for r in g["luma"] + g["chroma"])
