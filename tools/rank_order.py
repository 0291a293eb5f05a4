"""Model experiment: a rank-aware task order for the multi-GPU engine.

The engine's per-rank lists are the single-GPU list restricted to each rank's tile columns
(snake partition). Here the global list is rebuilt by list scheduling against the dist model
instead: the next slot goes to the rank whose earliest-free workgroup comes first; among that
rank's tasks whose wait targets are already in the list, one whose first useful work can start
by then is preferred by (class, step, column) — panels, the lookahead column's chains, other
chains — else the one that can start soonest. Chains of a remote panel are timed against the
member flags (forwarding on waves 4-7, `hop` after the flag), as in sched_sim.simulate_dist.
The result is still one topological order, so every rank's restriction is deadlock-free like
the engine's. Usage: python tools/rank_order.py [M] [N] [world ...]
"""
import heapq
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import sched_sim as S  # noqa: E402


def greedy_dist(M, N, world, ns=2, seglen=8, prm=S.P, fwd_peer=1.6, hop=3.0, part="snake", prio="class"):
    NG, W = prm["NG"], prm["W"]
    fw = fwd_peer * (world - 1)
    T = S.tasks_of(M, N, ns, seglen)
    segof = lambda k, j, i: (i - k - 1) // seglen
    own = lambda t: S.owner_of(t[2] if t[0] == "P" else t[2], world, part)
    deps, succ, ndep = {}, {}, {}
    key = lambda t: ("Cx",) + t[1:5] if t[0] == "C" else t
    for t in T:
        if t[0] == "P":
            _, i, k = t
            d = ([("P", i - 1, k)] if i > k else []) + ([("Cx", k - 1, k, s, segof(k - 1, k, i)) for s in range(ns)] if k > 0 else [])
        else:
            _, k, j, s, e, i0, i1 = t
            d = [("P", k, k)] if e == 0 else [("Cx", k, j, s, e - 1)]
            for i in ([k] if e == 0 else []) + list(range(i0, i1)):
                if i > k:
                    d.append(("P", i, k))
                if k > 0:
                    d.append(("Cx", k - 1, j, s, segof(k - 1, j, i)))
        ds = set(d)
        ndep[key(t)] = len(ds)
        for x in ds:
            succ.setdefault(x, []).append(t)
    Rr, Rc, E, FL, Tc, G = {}, {}, {}, {}, {}, {}
    workers = [[0.0] * W for _ in range(world)]
    notready = [[] for _ in range(world)]  # (ready time, seq, task): deps listed, not yet startable
    ready = [[] for _ in range(world)]     # (priority, seq, task): startable by the rank's next slot
    cnt = 0

    def remote(t):
        return t[0] == "C" and S.owner_of(t[1], world, part) != S.owner_of(t[2], world, part)

    def ready_time(t):
        if t[0] == "P":
            _, i, k = t
            r = max(Tc[(i, k, s, k - 1)] for s in range(ns)) if k > 0 else 0.0
            if i > k:
                r = max(r, Rr[(i - 1, k)][0] - prm["io_in"] - prm["f"] - prm["io_wb"])
            return r
        _, k, j, s, e, i0, i1 = t
        i = k if e == 0 else i0
        av = FL[(i, k)] if remote(t) else Rc[(i, k)]
        r = max(av[0], av[1])
        if k > 0:
            r = max(r, Tc[(i, j, s, k - 1)])
        if e > 0:
            r = max(r, G[(k, j, s, e - 1)][1])
        return r

    def prio_key(t):
        if prio == "step":  # oldest step first, panels before chains within it
            return (t[2], 0) if t[0] == "P" else (t[1], 1, t[2], t[4], t[3])
        if t[0] == "P":
            return (0, t[2], t[1])
        _, k, j, s, e, i0, i1 = t
        return (1 if j == k + 1 else 2, k, j, e, s)

    def push(t):
        nonlocal cnt
        cnt += 1
        heapq.heappush(notready[own(t)], (ready_time(t), cnt, t))

    for t in T:
        if ndep[key(t)] == 0:
            push(t)
    order = []
    left = len(T)
    while left:
        # the rank whose earliest-free workgroup comes first, among ranks with a listed task
        r = min((workers[q][0], q) for q in range(world) if notready[q] or ready[q])[1]
        tw = workers[r][0] + prm["disp"]
        nr, rd = notready[r], ready[r]
        while nr and nr[0][0] <= tw:
            _, c, x = heapq.heappop(nr)
            heapq.heappush(rd, (prio_key(x), c, x))
        t = heapq.heappop(rd)[2] if rd else heapq.heappop(nr)[2]
        order.append(t)
        left -= 1
        t0 = heapq.heappop(workers[r]) + prm["disp"]
        if t[0] == "P":
            _, i, k = t
            tt = max([t0] + ([Tc[(i, k, s, k - 1)] for s in range(ns)] if k > 0 else []))
            rr, rc, ee, fl = [0.0] * NG, [0.0] * NG, [0.0] * NG, [0.0] * NG
            prev = (i - 1, k) if i > k else None
            for g in range(NG):
                gs = tt if g == 0 else ee[g - 1]
                if prev:
                    gs = max(gs, Rr[prev][g])
                fct = max(prm["f"], fw) if world > 1 and g > 0 else prm["f"]
                rr[g] = gs + prm["io_in"] + fct + prm["io_wb"]
                rc[g] = rr[g] + prm["bt"] + prm["io_img"]
                last = g + 1 == NG
                rdy = rc[g] + (fw if world > 1 and last else 0.0)
                ee[g] = (max(rdy, E[prev][g]) if prev else rdy) + prm["t"]
                if world > 1:
                    if last:
                        fl[g] = ee[g] + hop
                    if g > 0:
                        fl[g - 1] = rr[g] - prm["io_wb"] + hop
            Rr[(i, k)], Rc[(i, k)], E[(i, k)], FL[(i, k)] = rr, rc, ee, fl
            end = ee[-1]
        else:
            _, k, j, s, e, i0, i1 = t
            rows = ([k] if e == 0 else []) + list(range(i0, i1))
            rem = remote(t)
            tt = t0
            pg = G[(k, j, s, e - 1)] if e > 0 else None
            lastg = None
            for idx, i in enumerate(rows):
                if k > 0:
                    tt = max(tt, Tc[(i, j, s, k - 1)])
                tt += prm["e_ld"]
                av = FL[(i, k)] if rem else Rc[(i, k)]
                nxt = (FL if rem else Rc)[(rows[idx + 1], k)][0] if idx + 1 < len(rows) else 0.0
                g_t = [0.0] * NG
                for g in range(NG):
                    need = av[g + 1] if g + 1 < NG else nxt
                    st = max(tt, av[g], need)
                    if pg is not None and idx == 0:
                        st = max(st, pg[min(g + 1, NG - 1)])
                    tt = st + prm["c"]
                    g_t[g] = tt
                tt += prm["e_st"]
                Tc[(i, j, s, k)] = tt
                lastg = g_t
            G[(k, j, s, e)] = lastg
            end = tt
        heapq.heappush(workers[r], end)
        for u in succ.get(key(t), []):
            ndep[key(u)] -= 1
            if ndep[key(u)] == 0:
                push(u)
    return order


def main(argv):
    M = int(argv[0]) if argv else 256
    N = int(argv[1]) if len(argv) > 1 else 64
    worlds = [int(x) for x in argv[2:]] or [2, 4, 8]
    items = S.export_list(M, N)
    t1 = S.simulate_dist(items, M, N, 1)
    print(f"{M}x{N} tiles: engine list on 1 GPU {t1 / 1e3:.1f} ms", flush=True)
    for w in worlds:
        te = S.simulate_dist(items, M, N, w)
        print(f"  {w} GPUs: engine list {te / 1e3:6.1f} ms (S {t1 / te:4.2f})", flush=True)
        for pr in ("class", "step"):
            tr = S.simulate_dist(S.to_items(greedy_dist(M, N, w, prio=pr)), M, N, w)
            print(f"    rank-aware list ({pr} priority) {tr / 1e3:6.1f} ms (S {t1 / tr:4.2f})", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
