"""VALU utilisation of k_me_sad (the C5 candidate kernel) from a rocprofv3 --pmc pass over the C5
bench (tools/gpu_run.sh pmc_c5) -> profiles/r04_c5_pmc.json, keyed by the sha256 of the library
that was profiled; bench.py's C3 line reports it as c5.bound when its own library has that hash.

SQ_ACTIVE_INST_VALU counts, per wave, the quad-cycles in which the wave issued a VALU instruction
(MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* are quad-cycle counts); one SIMD issues at
most one wave64 VALU instruction per 2 cycles (SIMD-32).  valu_busy = the SIMD-cycles VALU issue
took over the SIMD-cycles the kernel ran: SQ_INSTS_VALU x 2 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8
per XCD-summed cycle count) -- the share of the chip's VALU issue slots the kernel used."""
import csv
import glob
import hashlib
import json
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
OUT = sys.argv[2] if len(sys.argv) > 2 else "profiles/r04_c5_pmc.json"
KERNEL = "k_me_sad"


def per_dispatch(counter):
    vals = {}
    for p in glob.glob(f"{ROOT}/pmc_c5*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.setdefault((p, r["Dispatch_Id"]), 0.0)
                vals[(p, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return (sum(vals.values()) / len(vals), len(vals)) if vals else (None, 0)


insts, n = per_dispatch("SQ_INSTS_VALU")
active, _ = per_dispatch("SQ_ACTIVE_INST_VALU")
waves, _ = per_dispatch("SQ_WAVES")
wave_cycles, _ = per_dispatch("SQ_WAVE_CYCLES")
grbm, _ = per_dispatch("GRBM_GUI_ACTIVE")
sha = hashlib.sha256(open("vvc-extension-mm_amd/lib/libmm360.so", "rb").read()).hexdigest()
cycles = grbm / 8 if grbm else None  # GRBM_GUI_ACTIVE is summed over the 8 XCDs
d = {"kernel": KERNEL, "lib_sha256": sha, "dispatches": n,
     "sq_insts_valu": insts, "sq_active_inst_valu": active, "sq_waves": waves, "sq_wave_cycles": wave_cycles,
     "grbm_gui_active": grbm,
     "valu_insts_per_wave": round(insts / waves, 1) if insts and waves else None,
     "valu_busy": round(insts * 2 / (1024 * cycles), 3) if insts and cycles else None,
     "valu_utilization": round(active * 4 / wave_cycles / 4, 3) if active and wave_cycles else None,
     "note": "valu_busy = SQ_INSTS_VALU x 2 cycles / (1024 SIMDs x kernel cycles): the share of the chip's VALU "
             "issue slots k_me_sad used; valu_utilization = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES: the share of a "
             "resident wave's cycles in which it issued VALU"}
json.dump(d, open(OUT, "w"), indent=1)
print(json.dumps(d))
