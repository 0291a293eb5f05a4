"""Python host mirror of the MI355X tiled QR (libtqr.so) — thin ctypes bindings.

The product is the C ABI in include/{tqr,gridscheduler,gpucalc,qrdecomp}.h; this module only
binds it (for tests, bench.py and __graft_entry__), mirroring the reference's interface
(taskQRP_threads / cudaQRTask / SGEQRF ... / the gridscheduler API, reference qrdecomp.h,
include/gpucalc.h, include/gridscheduler.h). There is no Python or CPU compute path here:
every factorisation call goes to the HIP kernels, and loading fails loudly if libtqr.so is
missing.

Array convention: a column-major m x n matrix is a numpy/torch array of shape (n, m)
(row j = column j), so ldm = m and element (i, j) is A[j, i] — the reference's
CO(i,j,ldm) = j*ldm + i.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# TQR_LIB: a diagnostic build of the same library (e.g. libtqr_fst.so, activity stamps) by file name
LIB_PATH = os.path.join(HERE, os.environ.get("TQR_LIB", "libtqr.so"))

TQR_F32, TQR_F64 = 0, 1
QRS, SAPP, QRD, DAPP = 0, 1, 2, 3
TASK_AVAIL, TASK_NONE, TASK_DONE = 0, 1, 2
READY, DOING, DONE, NONE, NOTASKS = 0, 1, 2, 3, 4

_lib = None
_P = ctypes.c_void_p
_I = ctypes.c_int


class TQRError(RuntimeError):
    pass


class Task(ctypes.Structure):
    """reference include/gridscheduler.h:13-17"""
    _fields_ = [("taskType", _I), ("l", _I), ("m", _I), ("k", _I), ("taskStatus", _I)]


class Plan(ctypes.Structure):
    """tqr_plan_t, include/gridscheduler.h"""
    _fields_ = [("M", _I), ("N", _I), ("nlevels", _I), ("ntasks", ctypes.c_long),
                ("tasks", ctypes.POINTER(_I)), ("level_off", ctypes.POINTER(ctypes.c_long))]


def lib():
    """Load libtqr.so (raises if it was not built: no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm wheels dlopen their own bundled libamdhip64.so.7 by path; if libtqr.so were
    # loaded first, the process would hold two HIP runtimes and torch would see no GPU. Loading
    # torch first makes libtqr.so bind (by soname) to the one runtime torch already holds.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(LIB_PATH):
        raise TQRError(f"{LIB_PATH} is missing — build it with __graft_entry__.build() "
                       "(make -C gpu-tiled-qr-decomposition_amd)")
    L = ctypes.CDLL(LIB_PATH)
    L.tqr_strerror.restype = ctypes.c_char_p
    L.tqr_version.restype = ctypes.c_char_p
    L.tqr_total_tasks.restype = ctypes.c_long
    L.tqr_sched_total_tasks.restype = ctypes.c_long
    L.initScheduler.restype = ctypes.POINTER(Task)
    L.tqr_plan_create.argtypes = [ctypes.POINTER(_P), _I, _I, _I, _I]
    L.tqr_plan_execute.argtypes = [_P, _P, _I, _P, _P]
    L.tqr_plan_destroy.argtypes = [_P]
    L.tqr_plan_set_profile.argtypes = [_P, _I]
    L.tqr_plan_stats.argtypes = [_P, ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(_I), ctypes.POINTER(ctypes.c_double)]
    L.tqr_fill_randzo.argtypes = [_I, _P, _I, _I, _I, ctypes.c_ulonglong, _P]
    L.tqr_fill_randzo_cols.argtypes = [_I, _P, _I, _I, _I, ctypes.c_ulonglong, ctypes.c_long, _P]
    L.tqr_dist_local_cols.argtypes = [_P]
    for nm in ("tqr_tile_geqrt", "tqr_tile_unmqr", "tqr_tile_tsqrt", "tqr_tile_tsmqr"):
        getattr(L, nm).restype = _I
    L.tqr_dist_plan_create.argtypes = [ctypes.POINTER(_P), _I, _I, _I, _I, _I, _I]
    L.tqr_dist_handle_bytes.argtypes = [_P]
    L.tqr_dist_handle_bytes.restype = ctypes.c_size_t
    L.tqr_dist_export.argtypes = [_P, ctypes.c_char_p, ctypes.c_size_t]
    L.tqr_dist_import.argtypes = [_P, ctypes.c_char_p, ctypes.c_size_t]
    L.tqr_dist_reset.argtypes = [_P, _P]
    L.tqr_dist_probe.argtypes = [_P, _I, ctypes.POINTER(ctypes.c_ulonglong)]
    L.tqr_plan_status.argtypes = [_P, _P]
    L.tqr_dist_owner.argtypes = [_P, _I]
    L.tqr_dgeqrt_host.argtypes = [_P, _P, _I, _I, _I, _I]
    L.tqr_sgeqrt_host.argtypes = [_P, _P, _I, _I, _I, _I]
    _lib = L
    return L


def check(st, what=""):
    if st != 0:
        raise TQRError(f"{what}: {lib().tqr_strerror(st).decode()} ({st})")


def _ptr(a):
    if hasattr(a, "data_ptr"):
        return _P(a.data_ptr())
    return a.ctypes.data_as(_P)


def _dtype_code(dt):
    dt = np.dtype(dt) if not hasattr(dt, "is_floating_point") else dt
    if str(dt) in ("float64", "torch.float64"):
        return TQR_F64
    if str(dt) in ("float32", "torch.float32"):
        return TQR_F32
    raise TQRError(f"unsupported dtype {dt}")


# ---- scheduler (host C, no GPU needed) ---------------------------------------------------
class Scheduler:
    """The reference gridscheduler API (initScheduler / getNextTask / doneATask)."""

    def __init__(self, M, N):
        self.M, self.N = M, N
        self.grid = lib().initScheduler(M, N)
        if not self.grid:
            raise TQRError("initScheduler failed")

    def next_task(self):
        t = Task()
        r = lib().getNextTask(ctypes.byref(t), self.grid, self.M, self.N)
        return r, t

    def done(self, t):
        lib().doneATask(self.grid, self.M, self.N, t)

    def __del__(self):
        try:
            ctypes.CDLL(None).free(ctypes.cast(self.grid, _P))
        except Exception:
            pass


def sched_plan(M, N):
    """Static wave plan: list of waves, each a list of (type, l, m, k)."""
    p = Plan()
    check(lib().tqr_sched_plan(M, N, ctypes.byref(p)), "tqr_sched_plan")
    tasks = np.ctypeslib.as_array(p.tasks, shape=(p.ntasks * 4,)).reshape(-1, 4).copy()
    offs = np.ctypeslib.as_array(p.level_off, shape=(p.nlevels + 1,)).copy()
    lib().tqr_sched_plan_free(ctypes.byref(p))
    return [tasks[offs[L]:offs[L + 1]] for L in range(len(offs) - 1)]


# ---- device factorisation -------------------------------------------------------------------
class TiledQR:
    """A planned factorisation (tqr_plan): create once, execute on device arrays."""

    def __init__(self, m, n, b, dtype):
        self.m, self.n, self.b = m, n, b
        self.dtype = dtype if isinstance(dtype, int) else _dtype_code(dtype)
        self.kmax = min(m, n) // b
        h = _P()
        check(lib().tqr_plan_create(ctypes.byref(h), m, n, b, self.dtype), "tqr_plan_create")
        self.h = h

    def execute(self, A, tau, ldda=None, stream=None):
        """A, tau: device tensors (torch) — A (n, ldda) column-major, tau (kmax, m) compact."""
        ldda = ldda or self.m
        check(lib().tqr_plan_execute(self.h, _ptr(A), ldda, _ptr(tau), _P(stream or 0)), "tqr_plan_execute")

    def status(self, stream=None):
        """Synchronise `stream` and raise if the engine reported an error (tqr_plan_status)."""
        check(lib().tqr_plan_status(self.h, _P(stream or 0)), "tqr_plan_status")

    def set_profile(self, on=True):
        check(lib().tqr_plan_set_profile(self.h, int(on)))

    def stats(self):
        nu, np_ = _I(), _I()
        mu, mp = ctypes.c_double(), ctypes.c_double()
        check(lib().tqr_plan_stats(self.h, ctypes.byref(nu), ctypes.byref(mu), ctypes.byref(np_), ctypes.byref(mp)))
        return {"n_update": nu.value, "ms_update": mu.value, "n_panel": np_.value, "ms_panel": mp.value}

    def __del__(self):
        try:
            lib().tqr_plan_destroy(self.h)
        except Exception:
            pass


def tile_owner(j, world):
    """Rank owning tile column j in a multi-GPU factorisation (csrc/flow.hpp tile_owner): snake
    order over the ranks, 0..W-1 then W-1..0, so every rank's columns sum to the same index total.
    TQR_DIST_PART=cyclic restores j % W for A/B runs. Host-only helper (tests, planning): code that
    holds a plan asks the plan (DistTiledQR.owner), which read TQR_DIST_PART once, at creation."""
    blk, r = divmod(j, world)
    if os.environ.get("TQR_DIST_PART") == "cyclic":
        return r
    return world - 1 - r if blk % 2 else r


def peer_probe(L, h, rank, world, barrier):
    """The setup's peer-path probe (include/tqr.h tqr_dist_probe): every rank stores its token into
    each peer's probe word, `barrier()` (all ranks), every rank checks it sees each peer's token
    through the load path the chains poll. Raises TQRError naming the ranks whose stores did not
    arrive, before any factorisation could wait on them. Returns the bit mask of peers seen."""
    st = L.tqr_dist_probe(h, 0, None)
    if st != 0:
        raise TQRError(f"DistTiledQR: rank {rank}: peer probe (put) failed: {L.tqr_strerror(st).decode()} ({st})")
    barrier()
    seen = ctypes.c_ulonglong(0)
    st = L.tqr_dist_probe(h, 1, ctypes.byref(seen))
    missing = [r for r in range(world) if r != rank and not (seen.value >> r) & 1]
    if st != 0 or missing:
        raise TQRError(f"DistTiledQR: rank {rank} does not see the flag stores of rank(s) {missing}: "
                       "no working peer path (xGMI / IPC mapping) for the panel flags; "
                       "the factorisation would wait on them and time out")
    return seen.value


def owned_tile_cols(q, rank, world):
    """The tile columns 0..q-1 that `rank` owns."""
    return [j for j in range(q) if tile_owner(j, world) == rank]


class DistTiledQR(TiledQR):
    """One rank's share of a multi-GPU factorisation (tile-column partition, one process per GPU;
    include/tqr.h "multi-GPU"). Tile column j belongs to rank owner(j) (snake order 0..W-1,
    W-1..0, ...), and a rank stores only its own tile columns, packed: global tile column j is
    local tile column j // W (alloc_local / fill_randzo_local). The handle exchange goes over
    torch.distributed (`group`) once; the panel data moves GPU to GPU inside the persistent
    launch (xGMI stores into IPC-opened peer workspaces), and consecutive executes need no host
    synchronisation or barrier (epoch-valued flags on the device)."""

    def __init__(self, m, n, b, dtype, group=None):
        import torch.distributed as dist
        self.m, self.n, self.b = m, n, b
        self.dtype = dtype if isinstance(dtype, int) else _dtype_code(dtype)
        self.kmax = min(m, n) // b
        self.group = group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        verbose = os.environ.get("TQR_DIST_VERBOSE") == "1"

        def say(msg):
            if verbose:
                import sys
                print(f"[rank {self.rank}] DistTiledQR: {msg}", file=sys.stderr, flush=True)

        say("create")
        h = _P()
        check(lib().tqr_dist_plan_create(ctypes.byref(h), m, n, b, self.dtype, self.rank, self.world),
              "tqr_dist_plan_create")
        self.h = h
        if self.world > 1:
            say("export")
            hb = lib().tqr_dist_handle_bytes(self.h)
            buf = ctypes.create_string_buffer(hb)
            check(lib().tqr_dist_export(self.h, buf, hb), "tqr_dist_export")
            blocks = [None] * self.world
            say("all_gather")
            dist.all_gather_object(blocks, bytes(buf.raw), group=group)
            allb = b"".join(blocks)
            say("import")
            check(lib().tqr_dist_import(self.h, allb, len(allb)), "tqr_dist_import")
            # every rank must deal the tile columns the same way (TQR_DIST_PART is read per process
            # at plan creation): a disagreement would deadlock the launch, so fail here instead
            mine = self.owners()
            every = [None] * self.world
            dist.all_gather_object(every, mine, group=group)
            if any(o != mine for o in every):
                raise TQRError("DistTiledQR: ranks disagree on the tile-column partition (TQR_DIST_PART)")
            say("probe")
            peer_probe(lib(), self.h, self.rank, self.world, lambda: dist.barrier(group=group))
            say("ready")

    def owner(self, tile_col):
        """Rank owning tile column tile_col, as this plan partitions (tqr_dist_owner)."""
        r = lib().tqr_dist_owner(self.h, tile_col)
        if r < 0:
            check(r, "tqr_dist_owner")
        return r

    def owners(self):
        return [self.owner(j) for j in range(self.n // self.b)]

    def owned_cols(self):
        """The tile columns this rank owns (its panels and all their updates)."""
        return [j for j, r in enumerate(self.owners()) if r == self.rank]

    def owns(self, tile_col):
        return self.owner(tile_col) == self.rank

    def local_cols(self):
        """Number of tile columns this rank stores (tqr_dist_local_cols)."""
        c = lib().tqr_dist_local_cols(self.h)
        if c < 0:
            check(c, "tqr_dist_local_cols")
        return c

    def local_index(self, tile_col):
        """Local tile column of an owned global tile column."""
        return tile_col // self.world

    def alloc_local(self, device="cuda"):
        """(A, tau) device arrays of this rank's storage: A (local_cols * b, m) — row c = local
        matrix column c — and the compact tau (local_cols, m)."""
        import torch
        dt = torch.float64 if self.dtype == TQR_F64 else torch.float32
        nl = self.local_cols()
        return (torch.empty((nl * self.b, self.m), dtype=dt, device=device),
                torch.zeros((nl, self.m), dtype=dt, device=device))

    def fill_randzo_local(self, A, seed, stream=None):
        """This rank's tile columns of the global RANDZO matrix (tqr_fill_randzo_cols)."""
        b = self.b
        for j in self.owned_cols():
            lj = self.local_index(j)
            fill_randzo(A[lj * b:(lj + 1) * b], self.m, b, seed, stream=stream, col0=j * b)

    def fwd_bytes(self):
        """Bytes this rank forwards to its peers per factorisation (panel V/T images over xGMI)."""
        lib().tqr_plan_fwd_bytes.restype = ctypes.c_longlong
        return int(lib().tqr_plan_fwd_bytes(self.h))

    def execute(self, A, tau, ldda=None, stream=None):
        """Launch (stream-ordered) on this rank's packed storage (alloc_local). Every rank calls it
        the same number of times; no host synchronisation or barrier is needed between calls."""
        ldda = ldda or self.m
        check(lib().tqr_plan_execute(self.h, _ptr(A), ldda, _ptr(tau), _P(stream or 0)), "tqr_plan_execute")


def dist_plan_check(M, N, b, rank, world, seglen=8):
    """Host-only: (ntasks, n_forwarding_members) of one rank's task list (its panel tasks forward
    their images to the peers when world > 1)."""
    nt, nf = _I(), _I()
    check(lib().tqr_dist_plan_check(M, N, b, seglen, rank, world, ctypes.byref(nt), ctypes.byref(nf)),
          "tqr_dist_plan_check")
    return nt.value, nf.value


def fill_randzo(A, m, n, seed, ldda=None, stream=None, col0=0):
    """RANDZO input on the device (columns col0 .. col0 + n - 1 of the global matrix)."""
    check(lib().tqr_fill_randzo_cols(_dtype_code(A.dtype), _ptr(A), m, n, ldda or m, seed, col0, _P(stream or 0)),
          "tqr_fill_randzo_cols")


def geqrt_host(A, b, with_tau=True, m=None, tau=None):
    """Factorise a host column-major array (shape (n, ldm)) in place on the GPU; returns the
    reference's m x n tau matrix (shape (n, ldm), zero except columns k*b; written into `tau` if
    given, else a new zeroed array), or None with with_tau=False (the reference's cudaQRTask
    discards tau). m: rows (default ldm)."""
    n, ldm = A.shape
    m = m or ldm
    if with_tau and tau is None:
        tau = np.zeros_like(A)
    if with_tau:
        assert tau.shape == A.shape and tau.dtype == A.dtype and tau.flags.c_contiguous
    fn = lib().tqr_dgeqrt_host if A.dtype == np.float64 else lib().tqr_sgeqrt_host
    check(fn(_ptr(A), _ptr(tau) if with_tau else None, m, n, ldm, b), "tqr_geqrt_host")
    return tau


def cache_clear():
    """Release the cached plans and host-API staging buffers (tqr_cache_clear)."""
    check(lib().tqr_cache_clear(), "tqr_cache_clear")


def expand_tau(tau_compact, m, n, b):
    """compact (kmax, m) -> the reference's m x n tau matrix as an (n, m) array."""
    T = np.zeros((n, m), dtype=tau_compact.dtype)
    for k in range(min(m, n) // b):
        T[k * b, k * b:] = tau_compact[k, k * b:]
    return T


# ---- single tile ops (host pointers; the reference's SGEQRF/SLARFT/STSQRF/SSSRFT) --------
def _tile_ptr(M, r, c, b):
    """pointer to tile (r,c) of a column-major matrix stored as (n, m) numpy array"""
    ldm = M.shape[1]
    return _P(M.ctypes.data + (c * b * ldm + r * b) * M.itemsize)


def tile_geqrt(M, b, tau):
    check(lib().tqr_tile_geqrt(_dtype_code(M.dtype), _tile_ptr(M, 0, 0, b), _ptr(tau), b, M.shape[1]), "tile_geqrt")


def tile_unmqr(M, b, tau):
    """C = tile (0,1) updated with V, tau of tile (0,0)"""
    check(lib().tqr_tile_unmqr(_dtype_code(M.dtype), _tile_ptr(M, 0, 1, b), _tile_ptr(M, 0, 0, b), _ptr(tau), b,
                               M.shape[1]), "tile_unmqr")


def tile_tsqrt(M, b, tau):
    """[R tile (0,0); tile (1,0)]"""
    check(lib().tqr_tile_tsqrt(_dtype_code(M.dtype), _tile_ptr(M, 0, 0, b), _tile_ptr(M, 1, 0, b), _ptr(tau), b,
                               M.shape[1]), "tile_tsqrt")


def tile_tsmqr(M, b, tau):
    """V = tile (1,0), A = tile (0,1), B = tile (1,1)"""
    check(lib().tqr_tile_tsmqr(_dtype_code(M.dtype), _tile_ptr(M, 1, 0, b), _tile_ptr(M, 0, 1, b),
                               _tile_ptr(M, 1, 1, b), _ptr(tau), b, M.shape[1]), "tile_tsmqr")


def flops(m, n):
    """Algorithmic Householder QR flop count 2mn^2 - 2n^3/3 (m >= n)."""
    if m >= n:
        return 2.0 * m * n * n - 2.0 * n ** 3 / 3.0
    return 2.0 * n * m * m - 2.0 * m ** 3 / 3.0
