"""Extract the VVC interpolation tap tables from the reference source text into a fixture.

Reads /root/reference/source/Lib/CommonLib/InterpolationFilter.cpp (text only) and writes
tests/golden/filter_taps.json with m_lumaFilter[16][8] (:82-100) and m_chromaFilter[32][4]
(:187-221).  Run once in the survey container; the JSON is committed.
"""
import json
import os
import re
import sys

SRC = "/root/reference/source/Lib/CommonLib/InterpolationFilter.cpp"
OUT = os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "filter_taps.json")


def table(text, name):
    m = re.search(r"InterpolationFilter::" + name + r"\[[^\]]*\]\[[^\]]*\]\s*=\s*\{(.*?)\};", text, re.S)
    if not m:
        raise SystemExit(f"{name} not found")
    line = text[: m.start()].count("\n") + 1
    rows = re.findall(r"\{([^{}]*)\}", m.group(1))
    return line, [[int(v) for v in r.split(",") if v.strip()] for r in rows]


def main():
    text = open(SRC).read()
    ll, luma = table(text, "m_lumaFilter")
    cl, chroma = table(text, "m_chromaFilter")
    assert len(luma) == 16 and all(len(r) == 8 for r in luma)
    assert len(chroma) == 32 and all(len(r) == 4 for r in chroma)
    json.dump({"source": "source/Lib/CommonLib/InterpolationFilter.cpp", "luma_line": ll, "chroma_line": cl,
               "luma": luma, "chroma": chroma}, open(OUT, "w"), indent=1)
    print("wrote", OUT)


if __name__ == "__main__":
    sys.exit(main())
