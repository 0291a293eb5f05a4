"""Summarise tools/pmc_stall.sh: the k_flow launch's wave cycles by state (SQ counters count
quad-cycles per wave, summed over waves; MI355X_MICROARCH.md 'rocprofv3 PMC slots')."""
import csv, glob, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_stall"
pas = sys.argv[2] if len(sys.argv) > 2 else "stall"
rows = {}
for f in glob.glob(os.path.join(root, pas, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            if "k_flow" in row["Kernel_Name"]:
                d = rows.setdefault(int(row["Dispatch_Id"]), {})
                d[row["Counter_Name"]] = float(row["Counter_Value"])
                d["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
assert rows, "no k_flow rows"
d = rows[max(rows)]
if pas == "lds":
    gui = d["GRBM_GUI_ACTIVE"] / 8.0  # summed over the 8 XCDs -> cycles
    print(f"k_flow {d['_ns'] / 1e6:.1f} ms; GRBM_GUI_ACTIVE/8 {gui:.4g} cycles")
    for k, v in sorted(d.items()):
        if k.startswith("SQ_"):
            print(f"  {k:26s} {v:.4g}   per CU-cycle {v / (gui * 256):.3f}")
    sys.exit(0)
wc = d["SQ_WAVE_CYCLES"]
print(f"k_flow {d['_ns'] / 1e6:.1f} ms; SQ_WAVE_CYCLES {wc:.4g}")
for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM",
          "SQ_WAIT_INST_LDS"):
    print(f"  {k:22s} {d[k]:.4g}  {100 * d[k] / wc:5.1f} % of wave cycles")
print(f"  SQ_VALU_MFMA_BUSY_CYCLES {d['SQ_VALU_MFMA_BUSY_CYCLES']:.4g}")
