"""Sweep the flow plan's cost model / segment length / lookahead (env TQR_TG, TQR_SEGLEN, TQR_LAZY, TQR_LA, TQR_LAC) at one size."""
import os, subprocess, sys, json
m = sys.argv[1] if len(sys.argv) > 1 else "16384"
grid = [(s, t, l, a, c, g) for s in (os.environ.get("SEGS") or "8").split(",") for t in (os.environ.get("TGS") or "1.0,1.4").split(",")
        for l in (os.environ.get("LAZYS") or "0,0.5,1").split(",") for a in (os.environ.get("LAS") or "0").split(",")
        for c in (os.environ.get("LACS") or "0").split(",") for g in (os.environ.get("SEGLAS") or s).split(",")]
for seg, tg, lz, la, lac, sgla in grid:
    if True:
        env = dict(os.environ, TQR_TG=tg, TQR_SEGLEN=seg, TQR_LAZY=lz, TQR_LA=la, TQR_LAC=lac, TQR_SEGLEN_LA=sgla)
        r = subprocess.run([sys.executable, "bench.py", "--no-cpu-baseline", "--steps", "3", "--warmup", "1", "--rows", m, "--cols", m],
                           env=env, capture_output=True, text=True, timeout=120)
        try:
            j = json.loads(r.stdout.strip().splitlines()[-1])
            print(f"seglen {seg:>3} la-col {sgla:>3} Tg {tg:>4} lazy {lz:>4} la {la:>4} lac {lac:>4}: {j['ms_per_step']:8.2f} ms  {j['value']/1e3:6.2f} TF/s", flush=True)
        except Exception:
            print("failed", seg, tg, r.stderr[-500:], flush=True)
            sys.exit(1)
