"""Host-side model of the persistent engine (k_flow): simulates the in-order dequeue of a flow task
list on W workgroups with the kernel's waits (flow.hpp: panel members pipelined per reflector group
through Rr/Rc/Rt, chain elements waiting per group for the panel images of the NEXT group, Tc for the
tile's previous step, Ac for the previous segment's head rows) and per-group durations taken from
the activity stamps (tools/flowstamps.py). Usage: python tools/sched_sim.py [M]
Multi-GPU model (tile-column cyclic partition, panel images forwarded to the peers):
    python tools/sched_sim.py dist [M] [N] [world ...]   -> makespans, S(world), the panel cost S(8) >= 6 needs"""
import ctypes, heapq, os, sys
import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-tiled-qr-decomposition_amd"))

P = dict(f=29.0, bt=9.3, io_in=4.0, io_wb=2.0, io_img=4.0, t=15.5, c=16.0, e_ld=7.0, e_st=7.0, disp=1.5, W=256, NG=8)


def export_list(M, N, b=256, seglen=8):
    import tqr
    L = tqr.lib()
    n = L.tqr_flow_plan_export(M, N, b, seglen, None, 0)
    buf = (ctypes.c_int * (4 * n))()
    L.tqr_flow_plan_export(M, N, b, seglen, buf, n)
    return np.frombuffer(buf, dtype=np.int32).reshape(n, 4).copy()


def simulate(items, M, N, ns=2, prm=P, waits=None):
    NG, W = prm["NG"], prm["W"]
    wt = waits if waits is not None else {}
    acc = lambda c, v: wt.__setitem__(c, wt.get(c, 0.0) + max(0.0, v))
    Rr, Rc, E = {}, {}, {}       # panel (i,k) -> per-group times
    Tc = {}                      # (i, j, s, k) -> element end (tile (i,j) strip s done at step k)
    G = {}                       # (k, j, s, e) -> last element's group times (head rows for next segment)
    workers = [0.0] * W
    heapq.heapify(workers)
    busy = 0.0
    starts = np.zeros(len(items))
    ends = np.zeros(len(items))
    for x, (ts, l, m, kk) in enumerate(items):
        t0 = heapq.heappop(workers) + prm["disp"]
        typ = ts & 0xff
        if typ != 4:  # panel member (l, k); l == k: GEQRT
            i, k = l, kk
            t = t0
            if k > 0:
                t = max([t] + [Tc[(i, k, s, k - 1)] for s in range(ns)])
            acc("panel Tc wait", t - t0)
            rr, rc, ee = [0.0] * NG, [0.0] * NG, [0.0] * NG
            prev = (i - 1, k) if i > k else None
            for g in range(NG):
                gs = t if g == 0 else ee[g - 1]
                if prev:
                    acc("panel Rr wait", Rr[prev][g] + prm.get("hop", 0.0) - gs)
                    gs = max(gs, Rr[prev][g] + prm.get("hop", 0.0))
                rr[g] = gs + prm["io_in"] + prm["f"] + prm["io_wb"]
                rc[g] = rr[g] + prm["bt"] + prm["io_img"]
                if prev:
                    acc("panel Rt wait", E[prev][g] - rc[g])
                ee[g] = (max(rc[g], E[prev][g]) if prev else rc[g]) + prm["t"]
            Rr[(i, k)], Rc[(i, k)], E[(i, k)] = rr, rc, ee
            end = ee[-1]
        else:
            s = (ts >> 8) & 0xff
            i0, i1 = l & 0xffff, l >> 16
            k, e = kk & 0xffff, kk >> 16
            j = m
            rows = ([k] if e == 0 else []) + list(range(i0, i1))
            t = t0
            if e > 0:
                pg = G[(k, j, s, e - 1)]
            last = None
            la = "la" if j == k + 1 else "other"
            for idx, i in enumerate(rows):
                if k > 0:
                    acc("chain Tc wait", Tc[(i, j, s, k - 1)] - t)
                    t = max(t, Tc[(i, j, s, k - 1)])
                t += prm["e_ld"]
                rc = Rc[(i, k)]
                nxt = Rc[(rows[idx + 1], k)][0] if idx + 1 < len(rows) else 0.0
                g_t = [0.0] * NG
                for g in range(NG):
                    need = rc[g + 1] if g + 1 < NG else nxt
                    st = max(t, rc[g], need)
                    acc(f"chain Rc wait {la} {'start' if g == 0 and idx == 0 else 'in-elem'}", st - t)
                    if e > 0 and idx == 0:
                        acc("chain Ac wait", pg[min(g + 1, NG - 1)] - st)
                        st = max(st, pg[min(g + 1, NG - 1)])
                    t = st + prm["c"]
                    g_t[g] = t
                t += prm["e_st"]
                Tc[(i, j, s, k)] = t
                last = g_t
            G[(k, j, s, e)] = last
            end = t
        starts[x], ends[x] = t0, end
        busy += end - t0
        heapq.heappush(workers, end)
    return ends.max(), starts, ends


def tasks_of(M, N, ns=2, seglen=8, seglen_la=None):
    """All tasks: ('P', i, k) and ('C', k, j, s, e, i0, i1) with the engine's segmenting."""
    seglen_la = seglen_la or seglen
    T = []
    K = min(M, N)
    for k in range(K):
        for i in range(k, M):
            T.append(("P", i, k))
        for j in range(k + 1, N):
            sl = seglen_la if j == k + 1 else seglen
            nseg = max(1, (M - k - 1 + sl - 1) // sl)
            for e in range(nseg):
                i0, i1 = k + 1 + e * sl, min(M, k + 1 + (e + 1) * sl)
                if M - k - 1 == 0:
                    i0 = i1 = M
                for s in range(ns):
                    T.append(("C", k, j, s, e, i0, i1))
    return T


def to_items(order):
    out = []
    for t in order:
        if t[0] == "P":
            out.append((0 if t[1] == t[2] else 2, t[1], t[2], t[2]))
        else:
            _, k, j, s, e, i0, i1 = t
            out.append((4 | (s << 8), i0 | (i1 << 16), j, k | (e << 16)))
    return np.array(out, dtype=np.int64)


def greedy_order(M, N, ns=2, seglen=8, seglen_la=None, prm=P, prio="panel"):
    """List scheduling against the model: each next list slot goes to the earliest-free
    workgroup; among tasks whose wait targets are all earlier in the list, a task whose first
    useful work could start by then is preferred by (class, step, column) — panels, then the
    lookahead column's chains, then other chains — else the one that can start soonest."""
    seglen_la = seglen_la or seglen
    NG, W = prm["NG"], prm["W"]
    T = tasks_of(M, N, ns, seglen, seglen_la)
    segl = lambda k, j: seglen_la if j == k + 1 else seglen
    segof = lambda k, j, i: (i - k - 1) // segl(k, j)
    # dependency (wait-target) lists
    deps = {}
    for t in T:
        if t[0] == "P":
            _, i, k = t
            d = []
            if i > k:
                d.append(("P", i - 1, k))
            if k > 0:
                d += [("Cx", k - 1, k, s, segof(k - 1, k, i)) for s in range(ns)]
            deps[t] = d
        else:
            _, k, j, s, e, i0, i1 = t
            d = [("P", k, k)] if e == 0 else [("Cx", k, j, s, e - 1)]
            rows = ([k] if e == 0 else []) + list(range(i0, i1))
            for i in rows:
                if i > k:
                    d.append(("P", i, k))
                if k > 0:
                    d.append(("Cx", k - 1, j, s, segof(k - 1, j, i)))
            deps[t] = d
    key = lambda t: ("Cx",) + t[1:5] if t[0] == "C" else t
    succ = {}
    ndep = {}
    for t in T:
        ds = set(deps[t])
        ndep[key(t)] = len(ds)
        for d in ds:
            succ.setdefault(d, []).append(t)
    Rr, Rc, E, Tc, G = {}, {}, {}, {}, {}
    workers = [0.0] * W
    heapq.heapify(workers)
    notready, ready = [], []
    cnt = 0

    def ready_time(t):
        if t[0] == "P":
            _, i, k = t
            r = 0.0
            if k > 0:
                r = max(Tc[(i, k, s, k - 1)] for s in range(ns))
            if i > k:
                r = max(r, Rr[(i - 1, k)][0] - prm["io_in"] - prm["f"] - prm["io_wb"])
            return r
        _, k, j, s, e, i0, i1 = t
        i = k if e == 0 else i0
        r = max(Rc[(i, k)][0], Rc[(i, k)][1])
        if k > 0:
            r = max(r, Tc[(i, j, s, k - 1)])
        if e > 0:
            r = max(r, G[(k, j, s, e - 1)][1])
        return r

    def prio_key(t):
        if t[0] == "P":
            return (0, t[2], t[1])
        _, k, j, s, e, i0, i1 = t
        return (1 if j == k + 1 else 2, k, j, e, s)

    def push(t):
        nonlocal cnt
        cnt += 1
        heapq.heappush(notready, (ready_time(t), cnt, t))

    for t in T:
        if ndep[key(t)] == 0:
            push(t)
    order = []
    while notready or ready:
        tw = workers[0] + prm["disp"]
        while notready and notready[0][0] <= tw:
            r, c, t = heapq.heappop(notready)
            heapq.heappush(ready, (prio_key(t), c, t))
        if ready:
            _, _, t = heapq.heappop(ready)
        else:
            _, _, t = heapq.heappop(notready)
        order.append(t)
        # place t: compute its times with the same rules as simulate()
        t0 = heapq.heappop(workers) + prm["disp"]
        if t[0] == "P":
            _, i, k = t
            tt = t0
            if k > 0:
                tt = max([tt] + [Tc[(i, k, s, k - 1)] for s in range(ns)])
            rr, rc, ee = [0.0] * NG, [0.0] * NG, [0.0] * NG
            prev = (i - 1, k) if i > k else None
            for g in range(NG):
                gs = tt if g == 0 else ee[g - 1]
                if prev:
                    gs = max(gs, Rr[prev][g] + prm.get("hop", 0.0))
                rr[g] = gs + prm["io_in"] + prm["f"] + prm["io_wb"]
                rc[g] = rr[g] + prm["bt"] + prm["io_img"]
                ee[g] = (max(rc[g], E[prev][g]) if prev else rc[g]) + prm["t"]
            Rr[(i, k)], Rc[(i, k)], E[(i, k)] = rr, rc, ee
            end = ee[-1]
        else:
            _, k, j, s, e, i0, i1 = t
            rows = ([k] if e == 0 else []) + list(range(i0, i1))
            tt = t0
            pg = G[(k, j, s, e - 1)] if e > 0 else None
            last = None
            for idx, i in enumerate(rows):
                if k > 0:
                    tt = max(tt, Tc[(i, j, s, k - 1)])
                tt += prm["e_ld"]
                rc = Rc[(i, k)]
                nxt = Rc[(rows[idx + 1], k)][0] if idx + 1 < len(rows) else 0.0
                g_t = [0.0] * NG
                for g in range(NG):
                    need = rc[g + 1] if g + 1 < NG else nxt
                    st = max(tt, rc[g], need)
                    if pg is not None and idx == 0:
                        st = max(st, pg[min(g + 1, NG - 1)])
                    tt = st + prm["c"]
                    g_t[g] = tt
                tt += prm["e_st"]
                Tc[(i, j, s, k)] = tt
                last = g_t
            G[(k, j, s, e)] = last
            end = tt
        heapq.heappush(workers, end)
        for u in succ.get(key(t), []):
            ndep[key(u)] -= 1
            if ndep[key(u)] == 0:
                push(u)
    return order


def owner_of(j, world, kind="cyclic"):
    """rank owning tile column j: snake (0..W-1, W-1..0, ...: every rank's columns sum to the same
    index total, balancing the chain work that grows with j; the engine's partition since round 3)
    or cyclic (j % world, rounds 1-2)."""
    if kind == "snake":
        blk, r = divmod(j, world)
        return r if blk % 2 == 0 else world - 1 - r
    return j % world


def _cg(prm, unmqr, g, NG):
    """a chain group's duration: an UNMQR element's group g runs only the rows below the group
    (round 5: prm["uskip"], phases 1 and 2 from k-step 8 g), at prm["c0"] fixed cost"""
    if unmqr and prm.get("uskip"):
        return prm.get("c0", 1.5) + (prm["c"] - prm.get("c0", 1.5)) * (NG - g) / NG
    return prm["c"]


def simulate_dist(items, M, N, world, ns=2, prm=P, fwd_peer=1.6, hop=3.0, mode="idle", trace=None, pres=0,
                  part="snake", fine=None):
    """The engine on `world` GPUs of W workgroups each: rank r runs the tasks of the global list
    that it owns (chains of tile column j and panel j on owner_of(j)) in list order. A
    chain whose panel lives on another rank waits for the member flags instead of Rc: the owner
    forwards each group's images to the world - 1 peers (fwd_peer us per peer and group) and a
    flag reaches a peer `hop` us after it is set. mode "inline" (round 2): the panel's 512 threads
    copy group g's images between its Rc publish and its trailing update (on the member's serial
    path), flags after its Rt publish; mode "idle" (round 3): waves 4-7 copy group g's images during
    the factorisation of group g+1 (stretching it only if the copy is longer), flags at its end;
    the last group inline. pres > 0: each rank reserves `pres` of its W workgroups for panel tasks
    (a second in-order queue), the others take chain tasks only.
    fine = (df, dt): column-granular member hand-off (a what-if, not the engine): member i+1's
    reflector step C waits for member i's step C (not its whole group): its factorisation of group
    g starts df us after member i's started and ends no earlier than df after member i's ended;
    its trailing update likewise trails member i's by dt (strip-granular). Returns the makespan (us)."""
    NG, W = prm["NG"], prm["W"]
    fw = fwd_peer * (world - 1)
    Rr, Rc, E, FL, Tc, G = {}, {}, {}, {}, {}, {}
    FS, TcR, GR = {}, {}, {}
    x2d = hop + 3.0  # "2d": a strip / head-row hand-over between ranks (flag hop + 256 KiB over xGMI)
    heaps = [[0.0] * (W - pres) for _ in range(world)]
    pheaps = [[0.0] * pres for _ in range(world)]
    span = 0.0
    for (ts, l, m, kk) in items:
        typ = ts & 0xff
        if typ != 4:
            i, k = l, kk
            r = owner_of(k, world, part)
        else:
            k, j = kk & 0xffff, m
            r = owner_of(j, world, "snake" if part == "2d" else part)
            if part == "2d":  # what-if: chain segments spread over the ranks, not by column
                r = (j + (kk >> 16)) % world
        hp = pheaps[r] if (pres and typ != 4) else heaps[r]
        t0 = heapq.heappop(hp) + prm["disp"]
        # split panel (what-if, prm["split_from"]): steps >= it run a member as two co-scheduled
        # tasks, F (factorisation, block in / R, V out) and U (T, images, in-tile trailing update): U
        # updates the next group's block first (prm["u"] us after T), so F's next group starts then
        split = typ != 4 and kk >= prm.get("split_from", 1 << 30) and (not prm.get("split_ge") or l == kk)
        if split:
            t0u = heapq.heappop(hp) + prm["disp"]
        if typ != 4:
            t = t0
            if k > 0:
                t = max([t] + [Tc[(i, k, s, k - 1)] + (x2d if TcR[(i, k, s, k - 1)] != r else 0.0) for s in range(ns)])
            rr, rc, ee, fl = [0.0] * NG, [0.0] * NG, [0.0] * NG, [0.0] * NG
            fs = [0.0] * NG
            prev = (i - 1, k) if i > k else None
            for g in range(NG):
                gs = t if g == 0 else ee[g - 1]
                if split and g > 0:
                    gs = rr[g - 1] + prm["bt"] + prm.get("u", 6.0) + prm["io_in"]
                if prev:
                    gs = max(gs, FS[prev][g] + fine[0]) if fine else max(gs, Rr[prev][g])
                fs[g] = gs
                fct = prm["f"]
                if world > 1 and mode == "idle" and g > 0:
                    fct = max(fct, fw)  # waves 4-7 copy group g-1 meanwhile
                rr[g] = gs + prm["io_in"] + fct + prm["io_wb"]
                if prev and fine:
                    rr[g] = max(rr[g], Rr[prev][g] + fine[0])
                rc[g] = rr[g] + prm["bt"] + prm["io_img"]
                # what-if (prm["rc_late"]: "ge" GEQRT only / "all"): the images stored before the
                # trailing update but published with Rt after its drain — the image drain leaves the
                # member's group cycle, Rc comes t later
                late = prm.get("rc_late") == "all" or (prm.get("rc_late") == "ge" and i == k)
                if late:
                    rc[g] = rr[g] + prm["bt"] + prm.get("io_img_issue", 1.5)
                last = g + 1 == NG
                inline = world > 1 and (mode == "inline" or last)
                ready = rc[g] + (fw if inline else 0.0)
                if prev and fine:
                    ee[g] = max(ready + prm["t"], E[prev][g] + fine[1])
                else:
                    ee[g] = (max(ready, E[prev][g]) if prev else ready) + prm["t"]
                if late:
                    rc[g] = ee[g]
                if world > 1:
                    if inline:
                        fl[g] = ee[g] + hop
                    else:
                        fl[g - 1] = rr[g] + hop if g > 0 else 0.0
                if world > 1 and mode == "idle" and g > 0:
                    fl[g - 1] = rr[g] - prm["io_wb"] + hop
            Rr[(i, k)], Rc[(i, k)], E[(i, k)], FL[(i, k)] = rr, rc, ee, fl
            FS[(i, k)] = fs
            end = ee[-1]
            if split:  # F's workgroup is free after its last write-back, U's after the last trailing
                heapq.heappush(hp, rr[-1])
                span = max(span, rr[-1])
                t0 = max(t0, t0u)
        else:
            s = (ts >> 8) & 0xff
            i0, i1 = l & 0xffff, l >> 16
            e = kk >> 16
            remote = world > 1 and owner_of(k, world, part) != r
            rows = ([k] if e == 0 else []) + list(range(i0, i1))
            t = t0 + prm.get("seg", 0.0)  # per-segment cost (head rows in / out, Ac hand-over)
            pg = G[(k, j, s, e - 1)] if e > 0 else None
            if pg is not None and GR[(k, j, s, e - 1)] != r:
                pg = [x + x2d for x in pg]
            lastg = None
            for idx, i in enumerate(rows):
                if k > 0:
                    t = max(t, Tc[(i, j, s, k - 1)] + (x2d if TcR[(i, j, s, k - 1)] != r else 0.0))
                t += prm["e_ld"]
                av = FL[(i, k)] if remote else Rc[(i, k)]
                nxt = (FL if remote else Rc)[(rows[idx + 1], k)][0] if idx + 1 < len(rows) else 0.0
                g_t = [0.0] * NG
                for g in range(NG):
                    need = av[g + 1] if g + 1 < NG else nxt
                    st = max(t, av[g], need)
                    if pg is not None and idx == 0:
                        st = max(st, pg[min(g + 1, NG - 1)])
                    t = st + _cg(prm, i == k, g, NG)
                    g_t[g] = t
                t += prm["e_st"]
                Tc[(i, j, s, k)] = t
                TcR[(i, j, s, k)] = r
                lastg = g_t
            G[(k, j, s, e)] = lastg
            GR[(k, j, s, e)] = r
            end = t
        span = max(span, end)
        heapq.heappush(hp, end)
        if trace is not None:
            trace.append((r, t0, end, typ, k))
    return span


def simulate_dist_dyn(items, M, N, world, ns=2, prm=P, fwd_peer=1.6, hop=3.0, part="snake", prio="list",
                      waits=None):
    """Dependency-triggered dispatch (the reference's completeATask -> cuda_queue_puttask,
    gpucalc.cu:691-814 / 195-225, per rank): each rank keeps a ready queue fed by completions —
    its local counters and the peers' member flags — and a free workgroup takes the best task whose
    first useful work can start now (its dependencies' times are known and reached), else waits
    for the earliest one. Nothing is dequeued that would hold a workgroup waiting for its start;
    waits inside a task (later groups / elements) remain. prio "list": the engine's list position;
    "class": panels, then the lookahead column's chains, then other chains, each by (step, column).
    Timing rules as simulate_dist (idle-wave forwarding). Returns the makespan (us)."""
    NG, W = prm["NG"], prm["W"]
    fw = fwd_peer * (world - 1)
    wt = waits if waits is not None else {}
    acc = lambda c, v: wt.__setitem__(c, wt.get(c, 0.0) + max(0.0, v))
    tasks = []
    for x, (ts, l, m, kk) in enumerate(items):
        typ = ts & 0xff
        if typ != 4:
            tasks.append(("P", l, kk, x))
        else:
            s = (ts >> 8) & 0xff
            tasks.append(("C", kk & 0xffff, m, s, kk >> 16, l & 0xffff, l >> 16, x))
    rank_of = lambda t: owner_of(t[2], world, part) if t[0] == "P" else owner_of(t[2], world, part)
    segl = {}
    for t in tasks:  # segment index of row i in chain (k, j): from the list's own segments
        if t[0] == "C":
            _, k, j, s, e, i0, i1, _ = t
            for i in range(i0, i1):
                segl[(k, j, i)] = e
    deps = {}
    for t in tasks:
        if t[0] == "P":
            _, i, k, _ = t
            d = [("P", i - 1, k)] if i > k else []
            if k > 0:
                d += [("C", k - 1, k, s, segl[(k - 1, k, i)]) for s in range(ns)]
        else:
            _, k, j, s, e, i0, i1, _ = t
            d = [("P", k, k)] if e == 0 else [("C", k, j, s, e - 1)]
            for i in ([k] if e == 0 else []) + list(range(i0, i1)):
                if i > k:
                    d.append(("P", i, k))
                if k > 0:
                    d.append(("C", k - 1, j, s, segl[(k - 1, j, i)]))
        deps[t] = set(d)
    key = lambda t: t[:3] if t[0] == "P" else t[:5]
    succ, ndep = {}, {}
    for t in tasks:
        ndep[key(t)] = len(deps[t])
        for d in deps[t]:
            succ.setdefault(d, []).append(t)
    Rr, Rc, E, FL, Tc, G = {}, {}, {}, {}, {}, {}

    def ready_time(t):
        if t[0] == "P":
            _, i, k, _ = t
            r = max([Tc[(i, k, s, k - 1)] for s in range(ns)]) if k > 0 else 0.0
            if i > k:
                r = max(r, Rr[(i - 1, k)][0])
            return r
        _, k, j, s, e, i0, i1, _ = t
        i = k if e == 0 else i0
        remote = world > 1 and owner_of(k, world, part) != owner_of(j, world, part)
        av = (FL if remote else Rc)[(i, k)]
        r = max(av[0], av[1] if NG > 1 else av[0])
        if k > 0:
            r = max(r, Tc[(i, j, s, k - 1)])
        if e > 0:
            r = max(r, G[(k, j, s, e - 1)][min(1, NG - 1)])
        return r

    def pkey(t):
        if prio == "list":
            return t[-1]
        if t[0] == "P":
            return (0, t[2], t[1])
        return (1 if t[2] == t[1] + 1 else 2, t[1], t[2], t[4], t[3])

    def place(t, t0):
        if t[0] == "P":
            _, i, k, _ = t
            tt = t0
            if k > 0:
                tt = max([tt] + [Tc[(i, k, s, k - 1)] for s in range(ns)])
            rr, rc, ee, fl = [0.0] * NG, [0.0] * NG, [0.0] * NG, [0.0] * NG
            prev = (i - 1, k) if i > k else None
            for g in range(NG):
                gs = tt if g == 0 else ee[g - 1]
                if prev:
                    acc("panel Rr wait", Rr[prev][g] - gs)
                    gs = max(gs, Rr[prev][g])
                fct = max(prm["f"], fw) if world > 1 and g > 0 else prm["f"]
                rr[g] = gs + prm["io_in"] + fct + prm["io_wb"]
                rc[g] = rr[g] + prm["bt"] + prm["io_img"]
                last = g + 1 == NG
                ready = rc[g] + (fw if world > 1 and last else 0.0)
                if prev:
                    acc("panel Rt wait", E[prev][g] - ready)
                ee[g] = (max(ready, E[prev][g]) if prev else ready) + prm["t"]
                if world > 1:
                    if last:
                        fl[g] = ee[g] + hop
                    if g > 0:
                        fl[g - 1] = rr[g] - prm["io_wb"] + hop
            Rr[(i, k)], Rc[(i, k)], E[(i, k)], FL[(i, k)] = rr, rc, ee, fl
            return ee[-1]
        _, k, j, s, e, i0, i1, _ = t
        remote = world > 1 and owner_of(k, world, part) != owner_of(j, world, part)
        rows = ([k] if e == 0 else []) + list(range(i0, i1))
        tt = t0
        pg = G[(k, j, s, e - 1)] if e > 0 else None
        lastg = None
        for idx, i in enumerate(rows):
            if k > 0:
                acc("chain Tc wait", Tc[(i, j, s, k - 1)] - tt)
                tt = max(tt, Tc[(i, j, s, k - 1)])
            tt += prm["e_ld"]
            av = FL[(i, k)] if remote else Rc[(i, k)]
            nxt = (FL if remote else Rc)[(rows[idx + 1], k)][0] if idx + 1 < len(rows) else 0.0
            g_t = [0.0] * NG
            for g in range(NG):
                need = av[g + 1] if g + 1 < NG else nxt
                st = max(tt, av[g], need)
                if pg is not None and idx == 0:
                    st = max(st, pg[min(g + 1, NG - 1)])
                acc("chain wait inside" if (idx or g) else "chain wait at start", st - tt)
                tt = st + prm["c"]
                g_t[g] = tt
            tt += prm["e_st"]
            Tc[(i, j, s, k)] = tt
            lastg = g_t
        G[(k, j, s, e)] = lastg
        return tt

    workers = [[0.0] * W for _ in range(world)]
    notready = [[] for _ in range(world)]  # (ready_time, n, task): dependencies placed
    ready = [[] for _ in range(world)]     # (pkey, n, ready_time, task): startable
    cnt = 0
    for t in tasks:
        if ndep[key(t)] == 0:
            heapq.heappush(notready[rank_of(t)], (ready_time(t), cnt, t))
            cnt += 1
    left = len(tasks)
    span = 0.0
    while left:
        # the rank whose earliest-free workgroup frees first (and has a known task)
        best = None
        for r in range(world):
            if notready[r] or ready[r]:
                tw = workers[r][0] + prm["disp"]
                if best is None or tw < best[0]:
                    best = (tw, r)
        tw, r = best
        while notready[r] and notready[r][0][0] <= tw:
            rt, c, t = heapq.heappop(notready[r])
            heapq.heappush(ready[r], (pkey(t), c, rt, t))
        # the best startable task, else the one that can start soonest
        if ready[r]:
            _, _, rt, t = heapq.heappop(ready[r])
        else:
            rt, _, t = heapq.heappop(notready[r])
        t0 = max(heapq.heappop(workers[r]) + prm["disp"], rt)
        acc("idle (no startable task)", t0 - tw)
        end = place(t, t0)
        span = max(span, end)
        heapq.heappush(workers[r], end)
        left -= 1
        for u in succ.get(key(t), []):
            ndep[key(u)] -= 1
            if ndep[key(u)] == 0:
                heapq.heappush(notready[rank_of(u)], (ready_time(u), cnt, u))
                cnt += 1
    return span


def main_dist(argv):
    """Multi-GPU model: makespan and S(world) per forwarding mode, fine hand-off, dynamic dispatch and
    the panel cost at which S(8) >= 6. Args: [M] [N] [world ...]"""
    M = int(argv[0]) if len(argv) > 0 else 256
    N = int(argv[1]) if len(argv) > 1 else 64
    worlds = [int(x) for x in argv[2:]] or [1, 2, 4, 8]
    items = export_list(M, N)
    t1 = simulate_dist(items, M, N, 1)
    print(f"{M}x{N} tiles (b=256): {len(items)} tasks; model makespan on 1 GPU {t1 / 1e3:.1f} ms")
    for mode in ("inline", "idle"):
        for w in worlds[1:] if worlds[0] == 1 else worlds:
            tw = simulate_dist(items, M, N, w, mode=mode)
            print(f"  {mode:6s} forwarding, {w} GPUs: {tw / 1e3:7.1f} ms  S = {t1 / tw:5.2f}")
    # what-if: column-granular member hand-off (fine = (df, dt) us)
    for fine in ((4.0, 4.0), (2.0, 2.0)):
        t1f = simulate_dist(items, M, N, 1, fine=fine)
        line = f"  fine member hand-off {fine}: t1 {t1f / 1e3:6.1f} ms"
        for w in worlds[1:] if worlds[0] == 1 else worlds:
            tw = simulate_dist(items, M, N, w, fine=fine)
            line += f", t{w} {tw / 1e3:6.1f} (S {t1f / tw:4.2f})"
        print(line)
    if os.environ.get("TQR_SIM_DYN", "1") == "1":
        t1d = simulate_dist_dyn(items, M, N, 1)
        print(f"  dependency-triggered dispatch (per-rank ready queues), 1 GPU: {t1d / 1e3:.1f} ms")
        for pr in ("list", "class"):
            for w in worlds[1:] if worlds[0] == 1 else worlds:
                tw = simulate_dist_dyn(items, M, N, w, prio=pr)
                print(f"  dyn/{pr:5s} {w} GPUs: {tw / 1e3:7.1f} ms  S = {t1 / tw:5.2f} (vs the in-order 1-GPU model)"
                      f", {t1d / tw:5.2f} (vs dyn 1 GPU)")
    # the panel cost (factor, T, images, trailing, I/O) scale at which S(8) >= 6 (idle forwarding)
    for a in (1.0, 0.9, 0.8, 0.7, 0.6, 0.5, 0.4, 0.3):
        pp = dict(P, f=P["f"] * a, bt=P["bt"] * a, t=P["t"] * a, io_in=P["io_in"] * a, io_wb=P["io_wb"] * a,
                  io_img=P["io_img"] * a)
        t8 = simulate_dist(items, M, N, 8, prm=pp)
        t1a = simulate_dist(items, M, N, 1, prm=pp)
        cyc = a * (P["f"] + P["bt"] + P["t"] + P["io_in"] + P["io_wb"] + P["io_img"])
        print(f"  panel group cycle {cyc:5.1f} us: t1 {t1a / 1e3:6.1f} ms, t8 {t8 / 1e3:6.1f} ms, S(8) = {t1a / t8:4.2f}")


def _panel_scaled(a):
    """every panel cost (factor, T, images, trailing, I/O) scaled by a"""
    return dict(P, f=P["f"] * a, bt=P["bt"] * a, t=P["t"] * a, io_in=P["io_in"] * a, io_wb=P["io_wb"] * a,
                io_img=P["io_img"] * a)


def _mn(argv, m=256, n=64):
    return (int(argv[0]) if len(argv) > 0 else m), (int(argv[1]) if len(argv) > 1 else n)


def main_seglen(argv):
    """Chain segment length (TQR_SEGLEN) in the multi-GPU model: makespan and S(world) per segment
    length, with a per-segment cost (TQR_SIM_SEG us, default 20: calibrated on one MI355X, 65536x16384
    at segment length 2 vs 8 = 635.3 vs 607.6 ms, i.e. 27.7 ms for ~356k extra segments on 256
    workgroups). Args: [M] [N] [seglen ...]"""
    M, N = _mn(argv)
    sls = [int(x) for x in argv[2:]] or [8, 4, 3, 2]
    seg = float(os.environ.get("TQR_SIM_SEG", "20"))
    prm = dict(P, seg=seg)
    print(f"per-segment cost {seg} us")
    for sl in sls:
        items = export_list(M, N, seglen=sl)
        t1 = simulate_dist(items, M, N, 1, prm=prm)
        line = f"seglen {sl}: t1 {t1 / 1e3:6.1f} ms"
        for w in (2, 4, 8):
            tw = simulate_dist(items, M, N, w, prm=prm)
            line += f", t{w} {tw / 1e3:6.1f} (S {t1 / tw:4.2f})"
        print(line, flush=True)


def main_2d(argv):
    """Chain segments spread over the ranks ((j + segment) % world) instead of following their tile
    column's owner, every cross-rank strip / head-row hand-over charged a flag hop plus a 256 KiB
    xGMI copy. Args: [M] [N]"""
    M, N = _mn(argv)
    items = export_list(M, N)
    t1 = simulate_dist(items, M, N, 1)
    for w in (2, 4, 8):
        tc = simulate_dist(items, M, N, w)
        t2 = simulate_dist(items, M, N, w, part="2d")
        print(f"{w} ranks: column partition {tc / 1e3:6.1f} ms (S {t1 / tc:4.2f}); segments spread {t2 / 1e3:6.1f} ms "
              f"(S {t1 / t2:4.2f})", flush=True)


def main_cp(argv):
    """Critical path with unbounded workgroups (1 and 8 ranks), base / column-granular member
    hand-off / a faster panel (x0.3). Args: [M] [N]"""
    M, N = _mn(argv)
    items = export_list(M, N)
    fast = _panel_scaled(0.3)
    for name, prm, fine in (("base", P, None), ("fine", P, (2.0, 2.0)), ("panel x0.3", fast, None),
                            ("fine+panel x0.3", fast, (1.0, 1.0))):
        inf = dict(prm, W=20000)
        cp8 = simulate_dist(items, M, N, 8, prm=inf, fine=fine)
        cp1 = simulate_dist(items, M, N, 1, prm=inf, fine=fine)
        print(f"{name:18s}: critical path (unbounded workgroups) 1 rank {cp1 / 1e3:6.1f} ms, 8 ranks {cp8 / 1e3:6.1f} ms",
              flush=True)


def main_fastpanel(argv):
    """A faster panel (every panel cost scaled by a) under the engine's in-order per-rank dequeue and
    under dependency-triggered dispatch (simulate_dist_dyn), 1 and 8 ranks. Args: [M] [N] [a ...]"""
    M, N = _mn(argv)
    scales = [float(x) for x in argv[2:]] or [1.0, 0.5, 0.3]
    items = export_list(M, N)
    for a in scales:
        pp = _panel_scaled(a)
        t1 = simulate_dist(items, M, N, 1, prm=pp)
        t8 = simulate_dist(items, M, N, 8, prm=pp)
        d1 = simulate_dist_dyn(items, M, N, 1, prm=pp)
        d8 = simulate_dist_dyn(items, M, N, 8, prm=pp)
        print(f"panel x{a:.2f}: in-order t1 {t1 / 1e3:6.1f} t8 {t8 / 1e3:6.1f} S {t1 / t8:4.2f} | dynamic t1 {d1 / 1e3:6.1f} "
              f"t8 {d8 / 1e3:6.1f} S {d1 / d8:4.2f}", flush=True)


def main_waits(argv):
    """Where the workgroups wait under dependency-triggered dispatch, 1 and 8 ranks. Args: [M] [N]"""
    M, N = _mn(argv)
    items = export_list(M, N)
    for w in (1, 8):
        wt = {}
        t = simulate_dist_dyn(items, M, N, w, waits=wt)
        print(f"world {w}: {t / 1e3:.1f} ms")
        for c in sorted(wt):
            print(f"   {c:28s} {wt[c] / (w * 256) / 1e3:7.2f} ms/WG")


def main_xcd(argv):
    """ONE GPU, XCD affinity: the tasks of tile column j dequeued only by the 32 workgroups of XCD x(j)
    (the multi-GPU partition with 8 "ranks" of 32 workgroups, no forwarding), so strips and head rows
    could be stored write-back into that XCD's L2 (element hand-over e_ld / e_st scaled by h).
    Args: [M] [N] [h ...]"""
    M, N = _mn(argv, 64, 64)
    hs = [float(x) for x in argv[2:]] or [1.0, 0.5, 0.25]
    items = export_list(M, N)
    base = simulate_dist(items, M, N, 1)
    print(f"{M}x{N} tiles: one queue, 256 workgroups: {base / 1e3:.1f} ms")
    for h in hs:
        prm = dict(P, W=32, e_ld=P["e_ld"] * h, e_st=P["e_st"] * h)
        t = simulate_dist(items, M, N, 8, prm=prm, fwd_peer=0.0, hop=0.0)
        prm1 = dict(P, e_ld=P["e_ld"] * h, e_st=P["e_st"] * h)
        t1 = simulate_dist(items, M, N, 1, prm=prm1)
        print(f"  element hand-over x{h:.2f}: per-XCD queues {t / 1e3:.1f} ms; one queue with that hand-over "
              f"{t1 / 1e3:.1f} ms", flush=True)


def main_one(argv):
    """One GPU, the current order: makespan, per-workgroup waits, and with free panel compute.
    Args: [M] (square, tiles)"""
    M = int(argv[0]) if len(argv) > 0 else 64
    items = export_list(M, M)
    w = {}
    span, s, e = simulate(items, M, M, waits=w)
    print(f"current order: {len(items)} tasks, simulated makespan {span / 1e3:.1f} ms")
    for c in sorted(w):
        print(f"  {c:28s} {w[c] / P['W'] / 1e3:7.2f} ms/WG")
    p0 = dict(P, f=0.0, bt=0.0, t=0.0)
    span0, _, _ = simulate(items, M, M, prm=p0)
    print(f"  with free panel compute (PANEL0): {span0 / 1e3:.1f} ms")


# round-5 chain costs: the asm chain's group 16.3 us, the element hand-over with
# late strip loads +6 us in the hand-over group and +5 us in the next element's first group, the
# UNMQR element skipping the GE V's zero rows
P5 = dict(P, c=16.3, e_ld=5.0, e_st=6.0, uskip=1, c0=1.5)


def main_dist5(argv):
    """The 8-GPU model with round-5 chain costs (P5): one GPU at the engine's segment length 8, N
    ranks at its multi-rank default 2, and list / segment variants (environment knobs of the task
    list, TQR_*, read by the library's plan export). Args: [M] [N] [world]"""
    M, N = _mn(argv)
    w = int(argv[2]) if len(argv) > 2 else 8
    seg = float(os.environ.get("TQR_SIM_SEG", "20"))
    prm = dict(P5, seg=seg)
    t1 = simulate_dist(export_list(M, N, seglen=8), M, N, 1, prm=prm)
    print(f"{M}x{N} tiles, round-5 costs, per-segment {seg} us: t1 {t1 / 1e3:.1f} ms (segment length 8)", flush=True)
    variants = [("seglen 2 (round 4 default)", {}),
                ("round-5 8-GPU default", {"TQR_TAIL": str(7 * min(M, N) // 16), "TQR_TAIL_SEGLEN": "1", "TQR_LAC": "4"}),
                ("seglen_la 1", {"TQR_SEGLEN_LA": "1"}),
                ("lookahead column keyed 4 earlier", {"TQR_LAC": "4"}), ("panels keyed 2 earlier", {"TQR_LA": "2"}),
                ("seglen 3", {"TQR_SEGLEN": "3"})]
    if os.environ.get("TQR_SIM_VARIANTS"):  # "name:K=V,K=V;name:..." replaces the list
        variants = [(v.split(":")[0], dict(kv.split("=") for kv in v.split(":")[1].split(",") if kv))
                    for v in os.environ["TQR_SIM_VARIANTS"].split(";")]
    for name, env in variants:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            sl = int(os.environ.get("TQR_SEGLEN", "2"))
            items = export_list(M, N, seglen=sl)
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k)
                else:
                    os.environ[k] = v
        tw = simulate_dist(items, M, N, w, prm=prm)
        print(f"  {name:34s} t{w} {tw / 1e3:6.1f} ms  S({w}) = {t1 / tw:4.2f}", flush=True)


def main_split(argv):
    """One GPU, round-5 costs: the panel member split into a factorisation task and an update task
    (F / U, U updating the next group's block first) for the steps >= S. Args: [M] [S ...]"""
    M = int(argv[0]) if argv else 64
    prm = dict(P5, f=29.6, bt=10.6, t=15.9, io_in=4.0, io_wb=4.0, io_img=4.3)
    items = export_list(M, M, seglen=8)
    base = simulate_dist(items, M, M, 1, prm=prm)
    print(f"{M}x{M} tiles, round-5 costs, panel group cycle "
          f"{prm['io_in'] + prm['f'] + prm['io_wb'] + prm['bt'] + prm['io_img'] + prm['t']:.1f} us: {base / 1e3:.2f} ms")
    for sf in [int(x) for x in argv[1:]] or [0, M // 4, M // 2, 3 * M // 4]:
        for u in (6.0, 10.0):
            t = simulate_dist(items, M, M, 1, prm=dict(prm, split_from=sf, u=u))
            print(f"  split from step {sf:3d}, next block {u:4.1f} us after T: {t / 1e3:7.2f} ms ({(t - base) / 1e3:+.2f})")


def _list_env(env, M, N):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return export_list(M, N, seglen=int(os.environ.get("TQR_SEGLEN", "8")))
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


# the round-5 one-GPU measurements at 65536 x 16384 (BASELINE configs[3], profiles/r05/reh5): ranks x
# workgroups per rank, task list, measured ms per factorisation. The rehearsals share one GPU.
REH5 = [("1 rank x 256 (one GPU, c4)", 1, 256, "r4", 581.338),
        ("1 rank x 128 (t1 leg of the 2-rank run)", 1, 128, "r4", 1083.162),
        ("1 rank x 64 (t1 leg of the 4-rank run)", 1, 64, "r4", 2081.133),
        ("1 rank x 64, 8-GPU list (t1 leg)", 1, 64, "r5", 2191.254),
        ("2 ranks x 128 (rehearsal)", 2, 128, "r4", 591.792),
        ("4 ranks x 64 (rehearsal)", 4, 64, "r4", 602.1),
        ("4 ranks x 64, 8-GPU list (rehearsal)", 4, 64, "r5", 621.778)]
# the same shapes measured with the round-6 code on another box (profiles/r06/reh6, tools/reh_round.sh)
REH6 = [("1 rank x 256 (one GPU, c4)", 1, 256, "r4", 587.183),
        ("1 rank x 128 (t1 leg of the 2-rank run)", 1, 128, "r4", 1075.378),
        ("1 rank x 64 (t1 leg of the 4-rank run)", 1, 64, "r4", 2084.127),
        ("1 rank x 64, 8-GPU list (t1 leg)", 1, 64, "r5", 2180.608),
        ("2 ranks x 128 (rehearsal)", 2, 128, "r4", 597.346),
        ("4 ranks x 64 (rehearsal)", 4, 64, "r4", 608.097),
        ("4 ranks x 64, 8-GPU list (rehearsal)", 4, 64, "r5", 632.334)]
LISTS = {"r4": {"TQR_SEGLEN": "8"},  # (the rehearsals' ranks do not cover a device: segment length 8)
         "r4d": {"TQR_SEGLEN": "2"},  # round-4 multi-rank default: 2-element segments
         "r5": {"TQR_SEGLEN": "2", "TQR_TAIL": "28", "TQR_TAIL_SEGLEN": "1", "TQR_LAC": "4"}}  # round 5's


def main_calib(argv):
    """The multi-GPU model against the round-5 one-GPU measurements (profiles/r05/reh5): per shape the
    model's time, the measured one, their ratio; then t(8) on 8 x 256 workgroups for the round-4 and
    round-5 multi-rank task lists, corrected by the rehearsals' fitted ratio. Args: [M] [N]
    (TQR_CALIB_SET=reh6: the round-6 measurements instead)"""
    M, N = _mn(argv)
    reh = REH6 if os.environ.get("TQR_CALIB_SET") == "reh6" else REH5
    seg = float(os.environ.get("TQR_SIM_SEG", "20"))
    prm = dict(P5, seg=seg)
    lists = {k: _list_env(v, M, N) for k, v in LISTS.items()}
    ratios = {}
    print(f"{M}x{N} tiles, round-5 costs, per-segment {seg} us", flush=True)
    for name, world, W, lst, meas in reh:
        t = simulate_dist(lists[lst], M, N, world, prm=dict(prm, W=W)) / 1e3
        ratios[name] = meas / t
        print(f"  {name:42s} model {t:8.1f} ms  measured {meas:8.1f}  ratio {meas / t:5.3f}", flush=True)
    rr = [ratios[n] for n, w, *_ in reh if w > 1]
    one = ratios[reh[0][0]]
    lo, hi = min(rr), max(rr)
    print(f"  multi-rank rehearsals: measured / model {lo:.3f} .. {hi:.3f}; one GPU {one:.3f}")
    t1 = reh[0][4]
    for lst in ("r4d", "r5"):
        t8 = simulate_dist(lists[lst], M, N, 8, prm=dict(prm, W=256)) / 1e3
        print(f"  8 x 256, list {lst:3s}: model t(8) {t8:6.1f} ms, S(8) {t1 / t8:4.2f} uncorrected; corrected t(8) "
              f"{t8 * lo:6.1f} .. {t8 * hi:6.1f} ms, S(8) {t1 / (t8 * hi):4.2f} .. {t1 / (t8 * lo):4.2f}", flush=True)


COMMANDS = {"calib": main_calib, "split": main_split, "dist5": main_dist5, "one": main_one, "dist": main_dist, "seglen": main_seglen, "2d": main_2d, "cp": main_cp,
            "fastpanel": main_fastpanel, "waits": main_waits, "xcd": main_xcd}

if __name__ == "__main__":
    # python tools/sched_sim.py <command> [args]; a bare number (or nothing) is "one"
    if len(sys.argv) > 1 and sys.argv[1] in COMMANDS:
        COMMANDS[sys.argv[1]](sys.argv[2:])
    elif len(sys.argv) > 1 and sys.argv[1] in ("-h", "--help"):
        for k, f in COMMANDS.items():
            print(f"{k:10s} {(f.__doc__ or '').strip().splitlines()[0]}")
    else:
        main_one(sys.argv[1:])
