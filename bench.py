#!/usr/bin/env python3
"""bench.py — fp64 tiled-QR GFLOP/s on MI355X (BASELINE.json metric), one JSON line.

Workload (N = 1): BASELINE.json configs[2], the north-star roofline run — a 16384 x 16384
fp64 matrix, tile size 256, factorised in place by the flat-tree tiled Householder QR
(reference s10m/GPU-Tiled-QR-Decomposition: qrdecomp.c / gridscheduler.c DAG). Synthetic
RANDZO-distributed input generated on the device (the reference's distribution,
qrdecomp.c:1383). A step = restore the input from a resident HBM copy (device-to-device,
included in the step) + one whole factorisation. GFLOP/s uses the algorithmic count
2mn^2 - 2n^3/3.

N > 1 (torchrun, one process per GPU): ONE matrix, BASELINE.json configs[3] by default
(65536 x 16384 fp64, tile 256), factorised by all ranks together — tile column j on rank
j % N, the owner of each panel forwarding its reflector groups' V/T images to the peers over
xGMI inside the persistent launch. Total work is fixed ("scaling": "strong");
value = the matrix's algorithmic flops / max-over-ranks time. Each step restores the rank's
own tile columns from a resident copy, resets its counters, barriers, and factorises.

Extra objects on the line:
  roofline      — the dominant kernel (trailing-update: TSMQR/UNMQR strips on
                  v_mfma_f64_4x4x4_4b_f64): algorithmic flops of its launches / their summed
                  device time (HIP events on its own stream, a separate profiled pass),
                  against the fp64 MFMA peak 78.6 TFLOP/s (MI355X datasheet);
                  traffic = HBM bytes per launch from the committed rocprofv3 PMC summary.
  cpu_baseline  — the reference's own host path (oracle/_ref, 8 pthreads, as qrdecomp.c:21)
                  on a bounded sample, rank 0, N = 1 only; falls back to the oracle port.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gpu-tiled-qr-decomposition_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X datasheet fp64 matrix peak (DESIGN.md "Roofline")
METRIC = "fp64 QR GFLOP/s and %MFMA-peak, dense m×n, at 1/2/4/8 MI355X"


def qr_flops(m, n):
    return 2.0 * m * n * n - 2.0 * n ** 3 / 3.0 if m >= n else 2.0 * n * m * m - 2.0 * m ** 3 / 3.0


def update_flops(m, n, b):
    """Algorithmic flops of all trailing-update tasks: 4b^3 per TSMQR, 2b^3 per UNMQR."""
    p, q = m // b, n // b
    f = 0.0
    for k in range(min(p, q)):
        f += (p - k - 1) * (q - k - 1) * 4.0 * b ** 3 + (q - k - 1) * 2.0 * b ** 3
    return f


def cpu_baseline(sample_n=6144, b=256, threads=8):
    import ctypes

    import numpy as np
    P = ctypes.c_void_p
    ref = os.path.join(REPO, "oracle", "_ref", "libref_f64_fix.so")
    m = n = sample_n
    A = np.zeros((n, m), dtype=np.float64)
    F = np.zeros_like(A)
    T = np.zeros_like(A)
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        L.ref_factor.restype = ctypes.c_double
        L.ref_randzo(A.ctypes.data_as(P), m, n, m, 5)
        t = L.ref_factor(A.ctypes.data_as(P), F.ctypes.data_as(P), T.ctypes.data_as(P), m, n, b, m, threads)
        kind = "reference"
    else:
        lib = os.path.join(REPO, "oracle", "liboracle.so")
        L = ctypes.CDLL(lib)
        L.oracle_randzo_d(A.ctypes.data_as(P), m, n, m, 5)
        t0 = time.perf_counter()
        L.oracle_factor_threads_d(A.ctypes.data_as(P), F.ctypes.data_as(P), T.ctypes.data_as(P), m, n, b, m, threads)
        t = time.perf_counter() - t0
        kind = "port"
    cpu = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(qr_flops(m, n) / t / 1e9, 3), "unit": "GFLOP/s", "cores": threads, "kind": kind,
            "sample": f"{m}x{n} fp64 b={b} RANDZO seed 5, full factorisation, {threads} pthreads "
                      f"(reference taskQRP_threads worker loop, -O2), {t:.2f} s on {cpu}"}


def load_traffic(m, n, b):
    """HBM bytes per trailing-update launch from the committed rocprofv3 PMC summary."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    try:
        d = json.load(open(path))
        e = d.get(f"{m}x{n}_b{b}")
        return e["update_hbm_bytes_per_launch"] if e else None
    except (OSError, ValueError, KeyError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # (no --m/--n: torch.distributed.run's parser would claim them as abbreviations)
    ap.add_argument("--rows", type=int, default=None, help="m (default 16384 at N=1, 65536 at N>1)")
    ap.add_argument("--cols", type=int, default=None, help="n (default 16384)")
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--storage", choices=["f64", "f32"], default="f64",
                    help="matrix element type (arithmetic is fp64 either way; f32 = BASELINE configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=6144)
    args = ap.parse_args()

    import torch
    import tqr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # TQR_BENCH_DEVICE / TQR_BENCH_BACKEND: rehearse N > 1 with all ranks on one GPU over gloo
    dev = int(os.environ.get("TQR_BENCH_DEVICE", local_rank))
    torch.cuda.set_device(dev)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("TQR_BENCH_BACKEND", "nccl")  # nccl = RCCL on ROCm
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    m = args.rows or (16384 if world == 1 else 65536)
    n = args.cols or 16384
    b = args.tile
    dt = torch.float64 if args.storage == "f64" else torch.float32
    q = n // b

    A0 = torch.empty((n, m), dtype=dt, device="cuda")
    tqr.fill_randzo(A0, m, n, 5)
    A = torch.empty_like(A0)
    A.copy_(A0)
    tau = torch.zeros((min(m, n) // b, m), dtype=dt, device="cuda")
    plan = tqr.TiledQR(m, n, b, dt) if world == 1 else tqr.DistTiledQR(m, n, b, dt)
    stream = torch.cuda.current_stream().cuda_stream
    # this rank's tile columns (all of them at N = 1): rows j*b..j*b+b-1 of the (n, m) array
    own_A = A.view(q, b, m)[rank::world]
    own_A0 = A0.view(q, b, m)[rank::world]

    def step():
        own_A.copy_(own_A0)
        plan.execute(A, tau, stream=stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    el = t1 - t0
    if dist:
        tt = torch.tensor([el], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    if hasattr(plan, "status"):
        plan.status(stream)
    ms_step = el / args.steps * 1e3
    total_flops = qr_flops(m, n) * args.steps
    value = total_flops / el / 1e9

    # profiled pass (outside the timed region): per-launch device time of the dominant kernel
    plan.set_profile(True)
    own_A.copy_(own_A0)
    plan.execute(A, tau, stream=stream)
    torch.cuda.synchronize()
    st = plan.stats()
    plan.set_profile(False)
    uf = update_flops(m, n, b)
    # per GPU: its share of the update flops (1/N of the job at N > 1) over its launch time
    achieved = uf / world / (st["ms_update"] * 1e-3) / 1e12 if st["ms_update"] > 0 else None
    traffic = load_traffic(m, n, b)
    roof = {
        "bound": "mfma",
        "kernel": "k_flow (persistent engine; TSMQR/UNMQR strips on v_mfma_f64_4x4x4_4b_f64)",
        "achieved": round(achieved, 3) if achieved else None,
        "peak": FP64_MFMA_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP64_MFMA_PEAK_TFLOPS, 4) if achieved else None,
        "traffic": traffic,
        "launches": st["n_update"],
        "avg_launch_ms": round(st["ms_update"] / max(1, st["n_update"]), 4),
        "algorithmic_flops_per_launch": round(uf / max(1, st["n_update"])),
        "panel_kernel_ms_total": round(st["ms_panel"], 3),
        "whole_factorisation_frac_of_peak": round(value / 1e3 / (world * FP64_MFMA_PEAK_TFLOPS), 4),
    }
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_sample, b)

    cfg = 2 if (m, n) == (16384, 16384) else 3 if (m, n) == (65536, 16384) else 1 if (m, n) == (4096, 4096) else "custom"
    if args.storage == "f32":
        cfg = 4 if (m, n) == (32768, 32768) else "custom"
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (RANDZO distribution, device-generated)",
            "config": {"workload": f"tiled QR {m}x{n} {args.storage} storage, tile {b} (BASELINE configs[{cfg}])", "m": m, "n": n,
                       "tile": b, "parallelism": "single GPU" if world == 1 else
                       f"{world} GPUs, tile-column cyclic, panel V/T forwarded over xGMI"},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
