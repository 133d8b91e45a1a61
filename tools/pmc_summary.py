"""Summarise rocprofv3 --pmc CSVs per kernel (mean counter value per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict


def summarise(paths):
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].split("(")[0].replace("(anonymous namespace)::", "")
            if "anonymous" in r["Kernel_Name"]:
                k = r["Kernel_Name"].split("::")[1].split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
    return out


if __name__ == "__main__":
    paths = []
    for a in sys.argv[1:]:
        paths += glob.glob(a)
    for k, cs in summarise(paths).items():
        print(k)
        for c, v in sorted(cs.items()):
            print(f"    {c:32s} {v:16.1f}")
