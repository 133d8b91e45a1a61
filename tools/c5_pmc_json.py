"""VALU utilisation of k_me_sad (the C5 candidate kernel) from a rocprofv3 --pmc pass over the C5
bench (tools/gpu_run.sh pmc_c5) -> profiles/r04_c5_pmc.json, keyed by the sha256 of the library
that was profiled; bench.py's C3 line reports it as c5.bound when its own library has that hash.

SQ_ACTIVE_INST_VALU counts, per wave, the quad-cycles in which the wave issued a VALU instruction
(MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_ACTIVE_INST_* are quad-cycle counts).  Two figures:
valu_active_share = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x kernel cycles), the share of the SIMDs'
time with a VALU quad-cycle in progress (one per instruction on this kernel); valu_busy_2cyc = the
same with 2 cycles per instruction, the guide's SIMD-32 throughput of v_fma_f32 when waves
interleave -- the share of issue slots used lies between the two.  Kernel cycles =
GRBM_GUI_ACTIVE / 8 (summed over the XCDs)."""
import csv
import glob
import hashlib
import json
import sys

ROOT = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
OUT = sys.argv[2] if len(sys.argv) > 2 else "profiles/r05_c5_pmc.json"
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
     "valu_active_share": round(active * 4 / (1024 * cycles), 3) if active and cycles else None,
     "valu_busy_2cyc": round(insts * 2 / (1024 * cycles), 3) if insts and cycles else None,
     "note": "valu_active_share = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x kernel cycles); valu_busy_2cyc = "
             "SQ_INSTS_VALU x 2 / (1024 SIMDs x kernel cycles) (the guide's SIMD-32 rate): the share of VALU "
             "issue slots k_me_sad used lies between the two"}
json.dump(d, open(OUT, "w"), indent=1)
print(json.dumps(d))
