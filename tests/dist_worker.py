"""Multi-GPU parity worker (launched by tests/test_dist.py under torch.distributed.run).

Every rank factorises its share of the same RANDZO matrix with the tile-column partitioned engine
(tqr.DistTiledQR; each rank stores only its own tile columns, packed, generated in place from the
global matrix's seed); rank 0 also factorises the whole matrix alone (tqr.TiledQR, the single-GPU
engine). The owned tile columns and taus of all ranks are gathered to rank 0 (gloo, host tensors)
and compared with the single-GPU result: the per-tile operation sequence is identical, so the
results must agree bit for bit. Runs the factorisation twice, back to back with no host
synchronisation between the ranks (the epoch-valued flags of consecutive launches).
Prints one JSON line on rank 0. Usage: dist_worker.py m n b f64|f32 [device] [gather|checksum]

mode "checksum" (BASELINE-size shapes, e.g. 65536 x 16384): instead of gathering the matrix,
every rank reduces each owned tile column (and tau column) on the device to two wrapping int64
sums of the raw bit patterns (plain and position-weighted) and only these are gathered —
bit-identical results give identical checksums.
"""
import json
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "gpu-tiled-qr-decomposition_amd"))
import tqr  # noqa: E402


def checksums(blocks):
    """(plain, position-weighted) wrapping int64 sums of each block's raw bits, on the device."""
    out = []
    for x in blocks:
        v = x.contiguous().view(torch.int64 if x.dtype == torch.float64 else torch.int32).to(torch.int64).flatten()
        w = torch.arange(1, v.numel() + 1, device=v.device, dtype=torch.int64)
        out.append((int(v.sum().item()), int((v * w).sum().item())))
    return out


def main():
    m, n, b = (int(x) for x in sys.argv[1:4])
    dt = torch.float64 if sys.argv[4] == "f64" else torch.float32
    dev = int(sys.argv[5]) if len(sys.argv) > 5 else int(os.environ.get("LOCAL_RANK", "0"))
    mode = sys.argv[6] if len(sys.argv) > 6 else "gather"
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    q, kmax = n // b, min(m, n) // b
    # test hooks: rank 1 builds its task list with another segment length (must fail at import);
    # the single-GPU reference with its own segment length (results are bit-identical regardless)
    if rank == 1 and os.environ.get("TQR_TEST_SEGLEN_RANK1"):
        os.environ["TQR_SEGLEN"] = os.environ["TQR_TEST_SEGLEN_RANK1"]
    plan = tqr.DistTiledQR(m, n, b, dt)
    if os.environ.get("TQR_TEST_REF_SEGLEN"):
        os.environ["TQR_SEGLEN"] = os.environ["TQR_TEST_REF_SEGLEN"]
    L0, _ = plan.alloc_local()
    plan.fill_randzo_local(L0, 5)
    own = plan.owned_cols()
    torch.cuda.synchronize()
    if os.environ.get("TQR_DIST_VERBOSE") == "1":
        print(f"[rank {rank}] input ready ({len(own)} tile columns, {L0.numel() * L0.element_size() >> 20} MiB)",
              file=sys.stderr, flush=True)
    out = {"local_cols": plan.local_cols(), "owned": len(own)}

    def full_input():
        A0 = torch.empty((n, m), dtype=dt, device="cuda")
        tqr.fill_randzo(A0, m, n, 5)
        return A0

    # the packed local input is exactly the owned columns of the global matrix
    if mode == "gather":
        A0 = full_input()
        if not all(bool(torch.equal(L0[plan.local_index(j) * b:(plan.local_index(j) + 1) * b], A0[j * b:(j + 1) * b]))
                   for j in own):
            raise SystemExit(f"rank {rank}: the packed local input differs from the global matrix's columns")
        del A0
    verbose = os.environ.get("TQR_DIST_VERBOSE") == "1"

    def say(msg):
        if verbose:
            print(f"[rank {rank}] {msg}", file=sys.stderr, flush=True)

    # two launches back to back (stream-ordered, no host synchronisation in between), then the checks
    As, tau_list = [], []
    for rep in range(2):
        A, tau = plan.alloc_local()
        A.copy_(L0)
        As.append(A)
        tau_list.append(tau)
    # test hook: the last rank starts its launches TQR_TEST_SKEW_S seconds after the others (the
    # others' waits on its flags must outlast the skew: flow.hpp g_flow_wait_limit)
    skew = float(os.environ.get("TQR_TEST_SKEW_S", "0"))
    if skew > 0 and rank == world - 1:
        import time
        say(f"sleeping {skew} s before the first launch")
        time.sleep(skew)
    for rep in range(2):
        say(f"run {rep}: execute")
        plan.execute(As[rep], tau_list[rep])
    for rep in range(2):
        A, tau = As[rep], tau_list[rep]
        plan.status()
        say(f"run {rep}: done")
        lc = lambda j: slice(plan.local_index(j) * b, (plan.local_index(j) + 1) * b)  # noqa: E731
        own_tau = [k for k in range(kmax) if plan.owns(k)]
        if mode == "checksum":
            mine = dict(zip(own, checksums([A[lc(j)] for j in own])))
            mine_tau = dict(zip(own_tau, checksums([tau[plan.local_index(k)] for k in own_tau])))
            del A, tau
            allcs = [None] * world
            dist.all_gather_object(allcs, (mine, mine_tau))
            say(f"run {rep}: checksums gathered")
            if rank == 0:
                ref = tqr.TiledQR(m, n, b, dt)
                R = full_input()
                rtau = torch.zeros((kmax, m), dtype=dt, device="cuda")
                ref.execute(R, rtau)
                ref.status()
                rc = checksums([R[j * b:(j + 1) * b] for j in range(q)])
                rt = checksums([rtau[k] for k in range(kmax)])
                del R, rtau, ref
                cols, taus = {}, {}
                for c_, t_ in allcs:
                    cols.update(c_)
                    taus.update(t_)
                bad = [j for j in range(q) if cols.get(j) != rc[j]] + [-1 - k for k in range(kmax) if taus.get(k) != rt[k]]
                out[f"run{rep}"] = {"cols_covered": len(cols) == q, "mismatched": bad[:16], "exact": not bad}
            dist.barrier()
            torch.cuda.empty_cache()
            continue
        mine = {j: A[lc(j)].cpu().numpy() for j in own}
        mine_tau = {k: tau[plan.local_index(k)].cpu().numpy() for k in own_tau}
        allcols = [None] * world
        dist.all_gather_object(allcols, (mine, mine_tau))
        say(f"run {rep}: gathered")
        if rank == 0:
            ref = tqr.TiledQR(m, n, b, dt)
            R = full_input()
            rtau = torch.zeros((kmax, m), dtype=dt, device="cuda")
            ref.execute(R, rtau)
            torch.cuda.synchronize()
            R = R.cpu().numpy()
            rtau = rtau.cpu().numpy()
            F = np.zeros_like(R)
            T = np.zeros_like(rtau)
            seen = set()
            for cols, taus in allcols:
                for j, blk in cols.items():
                    F[j * b:(j + 1) * b] = blk
                    seen.add(j)
                for k, t in taus.items():
                    T[k] = t
            out[f"run{rep}"] = {
                "cols_covered": len(seen) == q,
                "max_diff": float(np.abs(F - R).max()),
                "max_tau_diff": float(np.abs(T - rtau).max()),
                "exact": bool(np.array_equal(F, R) and np.array_equal(T, rtau)),
            }
        dist.barrier()
    if rank == 0:
        print(json.dumps({"m": m, "n": n, "b": b, "world": world, **out}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
