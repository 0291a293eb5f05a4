#!/usr/bin/env python3
"""bench.py — fp64 tiled-QR GFLOP/s on MI355X (BASELINE.json metric), one JSON line.

Workload (N = 1): BASELINE.json configs[2], the north-star roofline run — a 16384 x 16384
fp64 matrix, tile size 256, factorised in place by the flat-tree tiled Householder QR
(reference s10m/GPU-Tiled-QR-Decomposition: qrdecomp.c / gridscheduler.c DAG). Synthetic
RANDZO-distributed input generated on the device (the reference's distribution,
qrdecomp.c:1383). A step = restore the input from a resident HBM copy (device-to-device,
included in the step) + one whole factorisation. GFLOP/s uses the algorithmic count
2mn^2 - 2n^3/3.

N > 1 (one process per GPU): ONE matrix, BASELINE.json configs[3] by default
(65536 x 16384 fp64, tile 256), factorised by all ranks together — tile columns dealt to the
ranks in snake order, the owner of each panel forwarding its reflector groups' V/T images to the
peers over xGMI inside the persistent launch. Total work is fixed ("scaling":
"strong"); value = the matrix's algorithmic flops / max-over-ranks time. A plain
`python bench.py --gpus N` starts the N ranks itself (torch.distributed.run as a child process,
before anything touches the GPU; launch_plan / spawn_ranks); under an external launcher
(WORLD_SIZE set) --gpus must agree with it.

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
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "gpu-tiled-qr-decomposition_amd"))

FP64_MFMA_PEAK_TFLOPS = 78.6  # MI355X datasheet fp64 matrix peak (DESIGN.md "Roofline")
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X fp32 matrix peak (MI355X_MICROARCH.md; 152-155 measured)
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


def _host_threads():
    """Host cores available to this process (the GPU box exports OMP_NUM_THREADS = its CPU share;
    os.cpu_count() there is the whole machine)."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit() and int(v) > 0:
        return int(v)
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def _cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_factor(m, n, b, threads, f32=False):
    """One full factorisation on the host: the reference's own host path (oracle/_ref, its
    pthr_doTasks worker loop + gridscheduler.c; fp32 = the unmodified source, fp64 = the same with
    -Dfloat=double) when built, else the oracle port. Returns (seconds, kind)."""
    import ctypes

    import numpy as np
    P = ctypes.c_void_p
    dt, sfx = (np.float32, "s") if f32 else (np.float64, "d")
    A = np.zeros((n, m), dtype=dt)
    F = np.zeros_like(A)
    T = np.zeros_like(A)
    ref = os.path.join(REPO, "oracle", "_ref", "libref_f32_fix.so" if f32 else "libref_f64_fix.so")
    if os.path.exists(ref):
        L = ctypes.CDLL(ref)
        L.ref_factor.restype = ctypes.c_double
        L.ref_randzo(A.ctypes.data_as(P), m, n, m, 5)
        return L.ref_factor(A.ctypes.data_as(P), F.ctypes.data_as(P), T.ctypes.data_as(P), m, n, b, m, threads), "reference"
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    getattr(L, f"oracle_randzo_{sfx}")(A.ctypes.data_as(P), m, n, m, 5)
    t0 = time.perf_counter()
    getattr(L, f"oracle_factor_threads_{sfx}")(A.ctypes.data_as(P), F.ctypes.data_as(P), T.ctypes.data_as(P), m, n, b, m, threads)
    return time.perf_counter() - t0, "port"


def cpu_baseline(sample_n=6144, b=256, f32=False, target=(16384, 16384), full_target=True):
    """the reference host path at 8 threads (qrdecomp.c:21) and at all host cores
    this process may use. Timed in full: configs[0] (512^2, b=64), configs[1] (4096^2, b=128; fp64
    only) and a sample^2 b=256 sample of the bench workload (same tile size, same kernels). The fp64
    workload up to 16384^2 is timed in full at both thread counts (round 6: the 8-thread run, ≈130 s,
    is the line's value, not extrapolated; `--no-full-cpu-target` skips both full runs and falls back
    to the sample's rate, marked extrapolated). f32: the reference's fp32 build (its native
    precision) for the fp32 line (configs[4]), whose 32768^2 workload is extrapolated from the
    sample."""
    nproc = _host_threads()
    legs = {}
    kind = "reference"
    tm, tn = target
    prec = "fp32" if f32 else "fp64"
    for name, thr in (("threads_8", 8), ("threads_nproc", nproc)):
        leg = {"threads": thr}
        t1, kind = _cpu_factor(512, 512, 64, thr, f32)
        leg["c1_512x512_b64_s"] = round(t1, 4)
        leg["c1_gflops"] = round(qr_flops(512, 512) / t1 / 1e9, 3)
        if not f32:
            t2, kind = _cpu_factor(4096, 4096, 128, thr, f32)
            leg["c2_4096x4096_b128_s"] = round(t2, 3)
            leg["c2_gflops"] = round(qr_flops(4096, 4096) / t2 / 1e9, 3)
        ts, kind = _cpu_factor(sample_n, sample_n, b, thr, f32)
        rate = qr_flops(sample_n, sample_n) / ts
        leg[f"sample_{sample_n}x{sample_n}_b{b}_s"] = round(ts, 3)
        leg["sample_gflops"] = round(rate / 1e9, 3)
        leg[f"target_{tm}x{tn}_b{b}_s_extrapolated"] = round(qr_flops(tm, tn) / rate, 1)
        if not f32 and tm * tn <= 16384 * 16384 and full_target:
            # the headline workload itself, in full (≈130 s at 8 threads, ≈67 s at 16 on the GPU box)
            tt, kind = _cpu_factor(tm, tn, b, thr, f32)
            leg[f"target_{tm}x{tn}_b{b}_s"] = round(tt, 2)
            leg["target_gflops"] = round(qr_flops(tm, tn) / tt / 1e9, 3)
        legs[name] = leg
    t8 = legs["threads_8"]
    full = "target_gflops" in t8
    what = f"{tm}x{tn}" if full else f"{sample_n}x{sample_n}"
    return {"value": t8["target_gflops"] if full else t8["sample_gflops"], "unit": "GFLOP/s", "cores": 8, "kind": kind,
            "sample": f"{what} {prec} b={b} RANDZO seed 5, full factorisation, 8 pthreads "
                      f"(reference taskQRP_threads worker loop, -O2) on {_cpu_model()}",
            "config": ("configs[0] 512x512 b=64 timed in full" + ("" if f32 else ", configs[1] 4096x4096 b=128 timed in full")
                       + (f"; the bench workload {tm}x{tn} b={b} timed in full at 8 and {nproc} threads" if full else
                          f"; the bench workload {tm}x{tn} b={b} extrapolated from the {sample_n}^2 b={b} sample rate")),
            "extrapolated": not full,
            "threads_8": legs["threads_8"], "threads_nproc": legs["threads_nproc"]}


def load_pmc(m, n, b, storage):
    """The committed rocprofv3 PMC summary of the k_flow launch (tools/pmc_summary.py): HBM bytes
    per launch, executed MFMA flops, MFMA-pipe utilisation. None where not measured."""
    path = os.path.join(REPO, "profiles", "pmc_summary.json")
    key = f"{m}x{n}_b{b}" + ("_f32" if storage == "f32" else "")
    try:
        return json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None


def check_output(A0, A, m, n):
    """Cheap correctness check of the final factorisation (outside the timed region): Q is
    orthogonal, so every column of R has the norm of the same column of A."""
    import torch
    R = torch.triu(A.T.double()).T  # (n, m) storage: zero below the diagonal
    na = torch.linalg.vector_norm(A0.double(), dim=1)
    nr = torch.linalg.vector_norm(R[:, :m], dim=1)
    rel = ((na - nr).abs() / na.clamp_min(1e-300)).max().item()
    tol = 1e-10 if A.dtype == torch.float64 else 1e-4
    if not rel <= tol:
        raise RuntimeError(f"bench: factorisation check failed (column-norm error {rel:.3e} > {tol})")
    return rel


def check_owned_columns(A0, A, m, n, b, rank, world, owned=None, packed=False):
    """The same check for one rank of a multi-GPU factorisation: every column of R lives in its
    tile column, and a tile column is finished by its owner (panel and all its updates), so each
    rank checks the columns it owns on its own device. owned: those tile columns as the plan deals
    them (DistTiledQR.owned_cols); default the snake partition (tqr.owned_tile_cols). packed: A0 and
    A hold only the owned tile columns, in order (the multi-GPU storage; else full (n, m) arrays)."""
    import torch
    import tqr
    q = n // b
    if owned is None:
        owned = tqr.owned_tile_cols(q, rank, world)
    own = torch.tensor(owned, device=A.device, dtype=torch.long)
    cols = torch.arange(n, device=A.device).view(q, b)[own].reshape(-1)  # global matrix columns
    rows = torch.arange(len(owned) * b, device=A.device) if packed else cols  # where they are stored
    Ao = A[rows].double()  # (n, m) storage: row c = matrix column c
    keep = torch.arange(m, device=A.device)[None, :] <= cols[:, None]  # R: rows r <= c
    nr = torch.linalg.vector_norm(Ao * keep, dim=1)
    na = torch.linalg.vector_norm(A0[rows].double(), dim=1)
    rel = ((na - nr).abs() / na.clamp_min(1e-300)).max().item()
    tol = 1e-10 if A.dtype == torch.float64 else 1e-4
    if not rel <= tol:
        raise RuntimeError(f"bench: rank {rank}: factorisation check failed (column-norm error {rel:.3e} > {tol})")
    return rel


def stage_budget(torch, share=1):
    """Bytes of HBM the bench may spend on staged inputs (one resident copy per timed step): three
    quarters of what is free on this device, split between the processes sharing it (a one-GPU
    rehearsal), at most 200 GiB. At 65536 x 16384 fp64 with the driver's 20 steps that is 160 GiB,
    so both strong-scaling legs time factorisations only."""
    free, _ = torch.cuda.mem_get_info()
    return min(200 << 30, int(0.75 * free) // max(1, share))


def single_gpu_leg(tqr, torch, m, n, b, dt, steps, warmup):
    """t(1 GPU) of the strong-scaling ratio: the N > 1 workload on this GPU alone, timed like the
    N-rank leg (staged inputs when steps copies fit in stage_budget, else a restore inside each
    step)."""
    A0 = torch.empty((n, m), dtype=dt, device="cuda")
    tqr.fill_randzo(A0, m, n, 5)
    A = A0.clone()
    tau = torch.zeros((min(m, n) // b, m), dtype=dt, device="cuda")
    plan = tqr.TiledQR(m, n, b, dt)
    staged = steps * A0.numel() * A0.element_size() <= stage_budget(torch)
    As = [A0.clone() for _ in range(steps)] if staged else []
    for _ in range(warmup):
        A.copy_(A0)
        plan.execute(A, tau)
    torch.cuda.synchronize()
    plan.status()
    t0 = time.perf_counter()
    for s in range(steps):
        if staged:
            plan.execute(As[s], tau)
        else:
            A.copy_(A0)
            plan.execute(A, tau)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    plan.status()
    rel = check_output(A0, As[-1] if staged and steps else A, m, n)
    del As, A, A0, tau, plan
    torch.cuda.empty_cache()
    return {"t1_ms": round(el / steps * 1e3, 3), "t1_inputs": "staged" if staged else "restored in step",
            "t1_column_norm_rel_err": rel}


def seglen_of(world, full=True):
    """The engine's chain segment length for a plan of `world` ranks (engine.hip env_seglen); full:
    each rank's launch covers its whole device (not a one-GPU rehearsal's share)."""
    e = os.environ.get("TQR_SEGLEN")
    return max(1, int(e)) if e else (2 if world >= 4 and full else 8)


def launch_plan(gpus, env, ndev):
    """How `bench.py --gpus N` runs: ("run", None) in this process (N = 1, or already one rank of an
    external torch.distributed.run), ("spawn", None) = start N ranks as a child launcher, or
    ("error", message). ndev: visible devices (a callable, so that it is only asked when needed;
    torch.cuda.device_count() does not initialise the GPU). TQR_BENCH_DEVICE pins every rank to one
    device (a one-GPU rehearsal), so the device count does not bound N then."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: must be >= 1"
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            return "error", f"--gpus {gpus} disagrees with WORLD_SIZE={ws} set by the launcher"
        return "run", None
    if gpus == 1:
        return "run", None
    if "TQR_BENCH_DEVICE" not in env:
        have = ndev()
        if gpus > have:
            return "error", f"--gpus {gpus} but only {have} device(s) are visible"
    return "spawn", None


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(gpus, argv, popen=None):
    """Run this script as `gpus` ranks under torch.distributed.run, as a CHILD process (nothing here
    has touched the GPU, and no exec replaces this process). The child's stdout is relayed line by
    line: the rank-0 JSON line to our stdout, everything else to stderr. Returns the exit code to
    use: the child's, or 1 if it exited 0 without printing a JSON line."""
    import subprocess
    popen = popen or subprocess.Popen
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    print(f"bench: launching {gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    child = popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    got = False
    for ln in child.stdout:
        s = ln.strip()
        if s.startswith("{") and '"metric"' in s:
            print(s, flush=True)
            got = True
        else:
            print(ln.rstrip("\n"), file=sys.stderr, flush=True)
    rc = child.wait()
    if rc == 0 and not got:
        print("bench: the ranks exited without a result line", file=sys.stderr, flush=True)
        return 1
    return rc


def main():
    # (before any torch / GPU call: N > 1 without an external launcher starts the ranks as a child)
    gi = None
    for x, a in enumerate(sys.argv[1:]):
        if a == "--gpus" and x + 2 < len(sys.argv):
            gi = sys.argv[x + 2]
        elif a.startswith("--gpus="):
            gi = a.split("=", 1)[1]
    if gi is not None:
        def ndev():
            import torch
            return torch.cuda.device_count()
        how, msg = launch_plan(int(gi), os.environ, ndev)
        if how == "error":
            print(f"bench: {msg}", file=sys.stderr, flush=True)
            sys.exit(2)
        if how == "spawn":
            sys.exit(spawn_ranks(int(gi), sys.argv[1:]))
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    # (no --m/--n: torch.distributed.run's parser would claim them as abbreviations)
    ap.add_argument("--rows", type=int, default=None, help="m (default 16384 at N=1, 65536 at N>1)")
    ap.add_argument("--cols", type=int, default=None, help="n (default 16384)")
    ap.add_argument("--tile", type=int, default=256)
    ap.add_argument("--storage", choices=["f64", "f32"], default="f64",
                    help="matrix element type: f64 (fp64 MFMA chains) or f32 (fp32 MFMA chains, fp64 panel "
                         "factorisation; BASELINE configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-api", action="store_true",
                    help="skip the PCIe-inclusive host-pointer timing (tqr_*geqrt_host)")
    ap.add_argument("--cpu-sample", type=int, default=6144)
    ap.add_argument("--no-full-cpu-target", action="store_true",
                    help="cpu_baseline: skip the full-size host factorisations of the workload (8 and all threads)")
    ap.add_argument("--no-single-leg", action="store_true",
                    help="N > 1: skip rank 0's single-GPU timing of the same matrix (strong_scaling)")
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
    rehearsal = world > 1 and "TQR_BENCH_DEVICE" in os.environ
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    if rehearsal and "TQR_FLOW_GRID" not in os.environ:
        # ranks sharing one GPU: each persistent launch gets its share of the CUs (all ranks' launches
        # must be resident together — a rank's chains wait for its peers' panels inside the launch)
        os.environ["TQR_FLOW_GRID"] = str(max(1, ncu // world))
    full_grid = int(os.environ.get("TQR_FLOW_GRID", ncu)) >= ncu  # (engine.hip: the segment-length rule)

    # strong scaling, self-contained: before the N-rank region, rank 0 factorises the same m x n
    # matrix on its GPU alone (single-GPU engine, same steps / warmup / input handling); the others wait
    single = None
    if dist:
        if rank == 0 and not args.no_single_leg:
            single = single_gpu_leg(tqr, torch, m, n, b, dt, args.steps, args.warmup)
        dist.barrier()

    if world == 1:
        plan = tqr.TiledQR(m, n, b, dt)
        A0 = torch.empty((n, m), dtype=dt, device="cuda")
        tqr.fill_randzo(A0, m, n, 5)
        tau = torch.zeros((min(m, n) // b, m), dtype=dt, device="cuda")
    else:
        # a rank stores only its own tile columns (packed, include/tqr.h "multi-GPU"): its share of
        # the same global RANDZO matrix, generated in place
        plan = tqr.DistTiledQR(m, n, b, dt)
        A0, tau = plan.alloc_local()
        plan.fill_randzo_local(A0, 5)
    A = torch.empty_like(A0)
    A.copy_(A0)
    stream = torch.cuda.current_stream().cuda_stream
    local_bytes = A0.numel() * A0.element_size()

    def step():
        A.copy_(A0)
        plan.execute(A, tau, stream=stream)

    # The factorisation is in place, so every timed step needs a fresh input: when HBM allows, one
    # resident copy per timed step is staged before the timed region (the timed region then holds
    # factorisations only); otherwise each step restores its input with a device copy inside it.
    nbytes = A0.numel() * A0.element_size()
    staged = args.steps * nbytes <= stage_budget(torch, world if rehearsal else 1)
    As = [A0.clone() for _ in range(args.steps)] if staged else []

    # N > 1: an engine error (a cross-device wait that timed out, error word set, workgroups drained)
    # or a failed column check on one rank is recorded in that rank's `status` and reported in the
    # line (value null, exit code 1) instead of raising on one rank while the others wait
    rank_status = "ok"

    def engine_status(where):
        nonlocal rank_status
        if not dist:
            plan.status(stream)
            return
        try:
            plan.status(stream)
        except tqr.TQRError as e:
            if rank_status == "ok":
                rank_status = f"{where}: {e}"

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    engine_status("warmup")  # the engine's error word (outside the timed region)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(args.steps):
        if staged:
            plan.execute(As[s], tau, stream=stream)
        else:
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
    engine_status("timed steps")
    Afin = As[-1] if staged and args.steps else A  # the last timed step's output
    if world == 1:
        ok_rel = check_output(A0, Afin, m, n)
    else:
        try:
            ok_rel = check_owned_columns(A0, Afin, m, n, b, rank, world, plan.owned_cols(), packed=True)
        except RuntimeError as e:
            ok_rel = None
            if rank_status == "ok":
                rank_status = f"check: {e}"
    del As, Afin
    dist_info = None
    failed = []
    if dist:
        # per rank: engine status, forwarded bytes, and with a stamps build
        # (TQR_LIB=libtqr_fst.so) the share of workgroup time the panels spent forwarding
        mine = {"rank": rank, "status": rank_status, "fwd_bytes": plan.fwd_bytes(), "column_norm_rel_err": ok_rel,
                "tile_cols": plan.local_cols(), "matrix_bytes": local_bytes,
                "hbm_in_use_bytes": torch.cuda.memory_allocated()}
        L = tqr.lib()
        if hasattr(L, "tqr_debug_flow_stamps"):
            import ctypes
            nc = L.tqr_debug_flow_stamp_count()
            grid = ctypes.c_int()
            L.tqr_plan_info(plan.h, None, None, None, ctypes.byref(grid))
            stv = (ctypes.c_ulonglong * (nc * grid.value))()
            if L.tqr_debug_flow_stamps(stv, grid.value) == 0:
                tot = sum(stv)
                fwd = sum(stv[w * nc + 23] for w in range(grid.value))  # panels' image forwarding
                mine["fwd_share_of_wg_time"] = round(fwd / tot, 4) if tot else None
                mine["fwd_ms_per_wg"] = round(fwd / grid.value / 1e5, 3)  # s_memrealtime at 100 MHz
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
        dist_info = {"world_size": world, "ranks": ranks}
        failed = [r["rank"] for r in ranks if r["status"] != "ok"]
    ms_step = el / args.steps * 1e3
    if failed:
        if rank == 0:
            print(json.dumps({"metric": METRIC, "value": None, "unit": "GFLOP/s", "n_gpus": world, "steps": args.steps,
                              "warmup": args.warmup, "ms_per_step": round(ms_step, 3), "higher_is_better": True,
                              "scaling": "strong", "vs_baseline": None, "dtype": args.storage,
                              "error": f"rank(s) {failed} failed (see dist.ranks[*].status)",
                              "config": {"workload": f"tiled QR {m}x{n} {args.storage} storage, tile {b}", "m": m,
                                         "n": n, "tile": b},
                              "dist": dist_info}), flush=True)
        dist.destroy_process_group()
        sys.exit(1)
    strong = None
    if single:
        strong = dict(single, tN_ms=round(ms_step, 3), tN_inputs="staged" if staged else "restored in step",
                      speedup=round(single["t1_ms"] / ms_step, 3),
                      efficiency=round(single["t1_ms"] / ms_step / world, 3),
                      note="t1: the same matrix on rank 0's GPU alone (single-GPU engine), timed before the "
                           f"{world}-rank region with the same steps, warmup and input handling" +
                           ("; REHEARSAL: all ranks share one GPU (TQR_BENCH_DEVICE), so this is not a "
                            "multi-GPU measurement" if rehearsal else ""))
    total_flops = qr_flops(m, n) * args.steps
    value = total_flops / el / 1e9

    # profiled pass (outside the timed region): per-launch device time of the dominant kernel
    plan.set_profile(True)
    A.copy_(A0)
    plan.execute(A, tau, stream=stream)
    torch.cuda.synchronize()
    st = plan.stats()
    plan.set_profile(False)
    uf = update_flops(m, n, b)
    # per GPU: its share of the update flops (1/N of the job at N > 1) over its launch time
    achieved = uf / world / (st["ms_update"] * 1e-3) / 1e12 if st["ms_update"] > 0 else None
    peak = FP64_MFMA_PEAK_TFLOPS if args.storage == "f64" else FP32_MFMA_PEAK_TFLOPS
    pmc = load_pmc(m, n, b, args.storage) if world == 1 else None
    traffic = pmc.get("update_hbm_bytes_per_launch") if pmc else None
    roof = {
        "bound": "mfma",
        "kernel": "k_flow (persistent engine; TSMQR/UNMQR strips on " +
                  ("v_mfma_f64_4x4x4_4b_f64)" if args.storage == "f64" else "v_mfma_f32_16x16x4_f32)"),
        "achieved": round(achieved, 3) if achieved else None,
        "peak": peak,
        "unit": "TFLOP/s",
        "frac": round(achieved / peak, 4) if achieved else None,
        "traffic": traffic,
        "executed_flops": pmc.get("executed_mfma_flops") if pmc else None,
        "mfma_util": round(pmc["mfma_util"], 4) if pmc and pmc.get("mfma_util") is not None else None,
        "pmc_source": "profiles/pmc_summary.json (rocprofv3 --pmc, tools/pmc_traffic.sh)" if pmc else None,
        "launches": st["n_update"],
        "avg_launch_ms": round(st["ms_update"] / max(1, st["n_update"]), 4),
        "algorithmic_flops_per_launch": round(uf / max(1, st["n_update"])),
        "panel_kernel_ms_total": round(st["ms_panel"], 3),
        "whole_factorisation_frac_of_peak": round(value / 1e3 / (world * peak), 4),
    }
    host_api = None
    if world == 1 and not args.no_host_api:
        # the reference's calling convention (host matrix in, factorised host matrix out): pageable
        # host array -> pinned staging -> HBM, factorisation, and back (outside the timed region;
        # reported beside, never as, the value)
        import numpy as np
        Ah = A0.cpu().numpy()
        Th = np.zeros_like(Ah)  # the caller's zeroed tau matrix (qrdecomp.c:90), allocated beforehand

        def host_ms(with_tau, mode):
            os.environ["TQR_HOST_XFER"] = mode
            times = []
            for _ in range(3):
                F = Ah.copy()
                t0 = time.perf_counter()
                tqr.geqrt_host(F, b, with_tau=with_tau, tau=Th if with_tau else None)
                times.append(time.perf_counter() - t0)
            os.environ.pop("TQR_HOST_XFER", None)
            return min(times) * 1e3

        th = host_ms(True, "stage")
        th_nt = host_ms(False, "stage")
        th_reg = host_ms(False, "register")
        host_api = {"ms": round(th, 1), "gflops": round(qr_flops(m, n) / th / 1e6, 1),
                    "ms_no_tau": round(th_nt, 1), "ms_registered_no_tau": round(th_reg, 1),
                    "h2d_d2h_bytes": 2 * Ah.nbytes,
                    "note": "tqr_geqrt_host end to end (best of 3), pageable host array in, factorised array "
                            "(+ the reference's m x n tau matrix for 'ms') out; the persistent launch uploads each "
                            "tile column before step 0 needs it and downloads it once final (csrc/xfer.hpp), host "
                            "threads filling / draining a pinned staging buffer meanwhile; ms_registered_no_tau: the "
                            "caller's array page-locked for the call and read / written by the launch directly"}
        del Ah, Th
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # (minutes of host work with no other output: a heartbeat on stderr every 30 s, the ctypes
        # calls release the GIL; stdout carries the one result line only)
        done = threading.Event()

        def heartbeat():
            t0 = time.perf_counter()
            while not done.wait(30.0):
                print(f"bench: cpu_baseline running ({time.perf_counter() - t0:.0f} s)", file=sys.stderr, flush=True)
        hb = threading.Thread(target=heartbeat, daemon=True)
        hb.start()
        try:
            cpu = cpu_baseline(args.cpu_sample, 256, f32=args.storage == "f32", target=(m, n),
                               full_target=not args.no_full_cpu_target)
        finally:
            done.set()
            hb.join()

    cfg = 2 if (m, n) == (16384, 16384) else 3 if (m, n) == (65536, 16384) else 1 if (m, n) == (4096, 4096) else "custom"
    if args.storage == "f32":
        cfg = 4 if (m, n) == (32768, 32768) else "custom"
    if rank == 0:
        part = "cyclic" if os.environ.get("TQR_DIST_PART") == "cyclic" else "snake"
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
            "dtype": args.storage,  # the chains' MFMA arithmetic (the panel factorises in fp64 either way)
            "data": "synthetic (RANDZO distribution, device-generated)",
            "config": {"workload": f"tiled QR {m}x{n} {args.storage} storage, tile {b} (BASELINE configs[{cfg}])", "m": m, "n": n,
                       "tile": b, "parallelism": "single GPU" if world == 1 else
                       (f"{world} ranks on ONE GPU (rehearsal, TQR_BENCH_DEVICE; {os.environ.get('TQR_FLOW_GRID')} "
                        f"workgroups per rank, the single-GPU leg too), tile-column {part}, panel V/T forwarded device to "
                        "device" if rehearsal else
                        f"{world} GPUs, tile-column {part}, panel V/T forwarded over xGMI"),
                       "inputs": "one resident copy per timed step, staged before the timed region" if staged
                       else "input restored by a device copy inside each timed step",
                       # elements per chain task (engine.hip env_seglen: TQR_SEGLEN, else 2 at >= 4 ranks, 8 otherwise)
                       "chain_segment_length": seglen_of(world, full_grid)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "check": {"column_norm_rel_err": ok_rel} if ok_rel is not None else None,
            "dist": dist_info,
            "strong_scaling": strong,
            "host_api": host_api,
        }
        print(json.dumps(line))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
