"""Join the rocprofv3 --pmc passes of tools/tile_bench_pmc.sh with the tile_bench JSON lines:
one line per (dtype, op, b) — the configuration's last k_update launch (tile_bench launches each
configuration 3 times, in the order of its JSON lines). Formulas as tools/pmc_summary.py:
  hbm_bytes   = 2 x FETCH_SIZE(KB) x 1024 + WRITE_SIZE(KB) x 1024 (gfx950 FETCH_SIZE correction);
  exec_flops  = (SQ_INSTS_VALU_MFMA_MOPS_F64 + _F32) x 512;
  mfma_util   = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) — of the whole chip,
                so a batch smaller than the chip reads low;
  alg_bytes   = the batch's tiles read and written once (TSMQR 2 tiles, UNMQR 1 tile, per copy).
The launches are the wave engine's standalone k_update (fp64 arithmetic for both storage types,
hence the MOPS_F64 counts for fp32), not the persistent engine's chains.
Usage: python3 tools/tile_bench_pmc.py <dir>   (JSON lines on stdout)"""
import csv, glob, json, os, sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tile_pmc"
REPS = 3


def launches(pass_name):
    files = glob.glob(os.path.join(root, pass_name, "**", "*counter_collection.csv"), recursive=True)
    assert files, f"no counter csv for {pass_name} under {root}"
    rows = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_update" in row["Kernel_Name"]:
                    d = rows.setdefault(int(row["Dispatch_Id"]), {})
                    d[row["Counter_Name"]] = float(row["Counter_Value"])
                    d["_ns"] = int(row["End_Timestamp"]) - int(row["Start_Timestamp"])
    return [rows[k] for k in sorted(rows)]


def configs(pass_name):
    with open(os.path.join(root, pass_name + ".jsonl")) as fh:
        return [json.loads(x) for x in fh if x.startswith("{")]


cfg = [c for c in configs("MFMA") if "status" not in c]  # (a rejected configuration launches nothing)
passes = {p: launches(p) for p in ("FETCH_SIZE", "WRITE_SIZE", "MFMA")}
for p, ls in passes.items():
    assert len(ls) == REPS * len(cfg), f"{p}: {len(ls)} k_update launches for {len(cfg)} configurations"
for i, c in enumerate(cfg):
    last = REPS * i + REPS - 1
    fe, wr, mf = passes["FETCH_SIZE"][last], passes["WRITE_SIZE"][last], passes["MFMA"][last]
    es = 8 if c["dtype"] == "f64" else 4
    rows = 2 if c["op"] == "TSMQR" else 1
    b, nb = c["b"], c["tiles"]
    alg_flops = (4.0 if rows == 2 else 2.0) * b ** 3 * nb
    exec_flops = (mf.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) + mf.get("SQ_INSTS_VALU_MFMA_MOPS_F32", 0.0)) * 512
    gui = mf.get("GRBM_GUI_ACTIVE", 0.0)
    util = mf["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui / 8 * 1024) if gui else None
    hbm = 2 * fe["FETCH_SIZE"] * 1024 + wr["WRITE_SIZE"] * 1024
    alg_bytes = 2 * rows * b * b * es * nb
    out = dict(c)
    out.update({"kernel_ms_profiled": round(mf["_ns"] / 1e6, 4), "mfma_util": round(util, 4) if util is not None else None,
                "exec_flops": exec_flops, "alg_flops": alg_flops, "exec_over_alg": round(exec_flops / alg_flops, 3),
                "hbm_bytes": int(hbm), "alg_bytes": alg_bytes, "hbm_over_alg": round(hbm / alg_bytes, 3),
                "hbm_gbs": round(hbm / (fe["_ns"] * 1e-9) / 1e9, 1),
                # the JSON line's ms / gflops come from HIP events around the launch, which under
                # the profiler include its per-dispatch counter collection; these are the kernel's
                "gflops_profiled": round(alg_flops / (mf["_ns"] * 1e-9) / 1e9, 1)})
    print(json.dumps(out))
