"""Per-launch HBM traffic of k_mc_dev from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_run.sh
pmc_fetch pmc_write) -> profiles/<name>.json, keyed by the sha256 of the library that was profiled.
bench.py reports it as roofline.traffic when its own library has the same hash.

FETCH_SIZE / WRITE_SIZE are in KB.  MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half the
bytes of 16-B-per-lane coalesced reads; k_mc's window reads are 8-16 B per lane, so the
fetch figure is doubled here (calibration outside the guide's measured pattern -- see DESIGN.md)."""
import csv
import glob
import hashlib
import json
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
OUT = sys.argv[2] if len(sys.argv) > 2 else "profiles/r04_traffic.json"
PICTURES = 4  # bench.py --pictures default, used by the pmc passes of tools/gpu_run.sh
KERNELS = ("k_mc_dev", "k_mc_pair_dev")  # the picture path's interpolation kernel, whichever is built


def per_dispatch(pattern, counter):
    vals = {}
    for p in glob.glob(pattern):
        for r in csv.DictReader(open(p)):
            if any(k in r["Kernel_Name"] for k in KERNELS) and r["Counter_Name"] == counter:
                vals.setdefault(r["Dispatch_Id"], 0.0)
                vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
    return sum(vals.values()) / len(vals), len(vals)


fetch_kb, nf = per_dispatch(f"{ROOT}/pmc_fetch/*counter_collection.csv", "FETCH_SIZE")
write_kb, nw = per_dispatch(f"{ROOT}/pmc_write/*counter_collection.csv", "WRITE_SIZE")
sha = hashlib.sha256(open("vvc-extension-mm_amd/lib/libmm360.so", "rb").read()).hexdigest()
d = {"kernel": "/".join(KERNELS), "lib_sha256": sha, "pictures": PICTURES, "dispatches": [nf, nw],
     "fetch_size_kb": round(fetch_kb, 1), "write_size_kb": round(write_kb, 1),
     "traffic_bytes_per_launch": int(2 * fetch_kb * 1024 + write_kb * 1024),
     "note": "2 x FETCH_SIZE + WRITE_SIZE per k_mc_dev launch (rocprofv3 --pmc, separate passes)"}
json.dump(d, open(OUT, "w"), indent=1)
print(json.dumps(d))
