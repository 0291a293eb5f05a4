"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc_traffic.sh) for the k_flow
launch into profiles/pmc_summary.json. bytes = 2 x FETCH_SIZE(KB) x 1024 + WRITE_SIZE(KB) x 1024
(gfx950: FETCH_SIZE reports half the bytes of wide streaming reads, MI355X_MICROARCH.md 'HBM')."""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"


def kflow_value(counter):
    files = glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter csv for {counter} under {root}"
    vals = []
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and "k_flow" in row["Kernel_Name"]:
                    vals.append(float(row["Counter_Value"]))
    assert vals, f"no k_flow rows for {counter}"
    return vals[-1], files


fetch, ff = kflow_value("FETCH_SIZE")
write, wf = kflow_value("WRITE_SIZE")
out = {
    "_doc": "HBM-side traffic of one k_flow launch (the whole 16384x16384 b=256 factorisation) from "
            "rocprofv3 --pmc, one counter per run (tools/pmc_traffic.sh, profiles/r01/pmc_v16/*.csv: rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE -- "
            "python3 bench.py --no-cpu-baseline --steps 1 --warmup 0). bytes = 2 x FETCH_SIZE(KB) x 1024 + "
            "WRITE_SIZE(KB) x 1024 (gfx950 FETCH_SIZE correction, MI355X_MICROARCH.md 'HBM'); Infinity-Cache "
            "hits are included by these counters.",
    "16384x16384_b256": {
        "fetch_size_kb_raw": fetch,
        "write_size_kb_raw": write,
        "fetch_bytes": int(2 * fetch * 1024),
        "write_bytes": int(write * 1024),
        "update_hbm_bytes_per_launch": int(2 * fetch * 1024 + write * 1024),
    },
}
os.makedirs("profiles", exist_ok=True)
with open("profiles/pmc_summary.json", "w") as fh:
    json.dump(out, fh, indent=1)
print(json.dumps(out["16384x16384_b256"]))
