"""Summarise the rocprofv3 --pmc passes of tools/pmc_traffic.sh for the k_flow launch into
profiles/pmc_summary.json (one entry per problem, key "<m>x<n>_b<b>[_f32]"):
  traffic   bytes = 2 x FETCH_SIZE(KB) x 1024 + WRITE_SIZE(KB) x 1024 (gfx950: FETCH_SIZE reports
            half the bytes of wide streaming reads, MI355X_MICROARCH.md 'HBM');
  MFMA      executed flops = (SQ_INSTS_VALU_MFMA_MOPS_F64 + _F32) x 512 (counter_defs.yaml
            'MFMA_FLOPS_F64': the MOPS counters count flops / 512); MFMA-pipe utilisation
            = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) (GRBM_GUI_ACTIVE is
            reported summed over the 8 XCDs, MI355X_MICROARCH.md 'DVFS give-back');
            effective clock = GRBM_GUI_ACTIVE / 8 / kernel duration.
Usage: python3 tools/pmc_summary.py <pmc dir> [key]"""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
key = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] else "16384x16384_b256"


def kflow_rows(pass_name):
    files = glob.glob(os.path.join(root, pass_name, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter csv for {pass_name} under {root}"
    rows = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_flow" in row["Kernel_Name"]:
                    d = rows.setdefault(int(row["Dispatch_Id"]), {})
                    d[row["Counter_Name"]] = float(row["Counter_Value"])
                    d["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    assert rows, f"no k_flow rows in {pass_name}"
    return rows[max(rows)], files  # the last k_flow launch of the run


fetch = kflow_rows("FETCH_SIZE")[0]["FETCH_SIZE"]
write = kflow_rows("WRITE_SIZE")[0]["WRITE_SIZE"]
mf = kflow_rows("MFMA")[0]
mops = mf.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) + mf.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)
gui = mf["GRBM_GUI_ACTIVE"]
busy = mf["SQ_VALU_MFMA_BUSY_CYCLES"]
entry = {
    "fetch_size_kb_raw": fetch,
    "write_size_kb_raw": write,
    "fetch_bytes": int(2 * fetch * 1024),
    "write_bytes": int(write * 1024),
    "update_hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
    "sq_insts_valu_mfma_mops_f64": mf.get("SQ_INSTS_VALU_MFMA_MOPS_F64"),
    "sq_insts_valu_mfma_mops_f32": mf.get("SQ_INSTS_VALU_MFMA_MOPS_F32"),
    "sq_insts_valu_mfma_f64": mf.get("SQ_INSTS_VALU_MFMA_F64"),
    "sq_valu_mfma_busy_cycles": busy,
    "grbm_gui_active": gui,
    "kernel_ns_profiled": mf["_ns"],
    "executed_mfma_flops": mops * 512.0,
    "mfma_util": busy / (gui / 8.0 * 1024.0),
    "effective_clock_ghz": gui / 8.0 / mf["_ns"],
}
path = "profiles/pmc_summary.json"
out = json.load(open(path)) if os.path.exists(path) else {}
out["_doc"] = ("PMC summary of one k_flow launch per problem (tools/pmc_traffic.sh: rocprofv3 --pmc passes "
               "over python3 bench.py --no-cpu-baseline --no-host-api --steps 1 --warmup 1, the last (warm) k_flow launch; CSVs under profiles/r05/final4/pmc*/). "
               + __doc__.split("\n", 2)[1].strip() + " See tools/pmc_summary.py for every formula.")
out[key] = entry
os.makedirs("profiles", exist_ok=True)
with open(path, "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps({key: entry}))
