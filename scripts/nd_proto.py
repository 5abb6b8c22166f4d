"""Prototype of the camera-side ordering: nested dissection of the image co-visibility graph,
block-level symbolic Cholesky and elimination-tree levels (the wave count bounds the factorisation's
critical path).  Compares with reverse Cuthill-McKee.  Usage: python scripts/nd_proto.py [config] [leaf]"""
import os
import sys
from collections import deque

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "fish-eye_bundle_adjustment_amd"))
import synth  # noqa: E402

NB = 128


def graph(img, pid, n_img):
    order = np.argsort(pid, kind="stable")
    p, e = pid[order], img[order]
    adj = [set() for _ in range(n_img)]
    starts = np.flatnonzero(np.r_[True, p[1:] != p[:-1], True])
    for a, b in zip(starts[:-1], starts[1:]):
        ims = np.unique(e[a:b])
        for x in ims:
            adj[x].update(ims)
    for v in range(n_img):
        adj[v].discard(v)
    return [sorted(s) for s in adj]


def bfs_levels(adj, verts, root):
    vs = set(verts)
    lev = {root: 0}
    q = deque([root])
    while q:
        v = q.popleft()
        for w in adj[v]:
            if w in vs and w not in lev:
                lev[w] = lev[v] + 1
                q.append(w)
    return lev


def bisect(adj, verts):
    vs = set(verts)
    root = min(verts, key=lambda v: (sum(1 for w in adj[v] if w in vs), v))
    for _ in range(3):  # pseudo-peripheral root
        lev = bfs_levels(adj, verts, root)
        far = max(lev, key=lambda v: (lev[v], -v))
        if lev[far] <= max(lev.values()) and far == root:
            break
        root = far
    lev = bfs_levels(adj, verts, root)
    rest = [v for v in verts if v not in lev]
    maxl = max(lev.values())
    counts = np.bincount(list(lev.values()), minlength=maxl + 1)
    half = len(verts) / 2
    cum = np.cumsum(counts)
    # separator level: the one closest to the median, ties toward the smaller level set
    best = min(range(1, maxl) if maxl >= 2 else [0], key=lambda l: (abs(cum[l] - counts[l] / 2 - half), counts[l]))
    A = [v for v in verts if v in lev and lev[v] < best]
    S = [v for v in verts if v in lev and lev[v] == best]
    B = [v for v in verts if v in lev and lev[v] > best] + rest
    # refine: separator vertices with no neighbour in B (A) move to A (B)
    sA, sB = set(A), set(B)
    S2 = []
    for v in S:
        if not any(w in sB for w in adj[v]):
            sA.add(v)
        elif not any(w in sA for w in adj[v]):
            sB.add(v)
        else:
            S2.append(v)
    return sorted(sA), sorted(sB), S2


def rcm(adj, verts):
    vs = set(verts)
    deg = {v: sum(1 for w in adj[v] if w in vs) for v in verts}
    seen, order = set(), []
    for r in sorted(verts, key=lambda v: (deg[v], v)):
        if r in seen:
            continue
        seen.add(r)
        q = deque([r])
        order.append(r)
        while q:
            v = q.popleft()
            for w in sorted((w for w in adj[v] if w in vs and w not in seen), key=lambda w: (deg[w], w)):
                seen.add(w)
                order.append(w)
                q.append(w)
    return order[::-1]


def nd(adj, verts, leaf, out):
    """append the nested-dissection order of verts to out (-1 = padding image)"""
    if len(verts) <= leaf:
        out.extend(rcm(adj, verts))
        return
    A, B, S = bisect(adj, verts)
    if not A or not B:
        out.extend(rcm(adj, verts))
        return
    nd(adj, A, leaf, out)
    # pad so that B starts in a fresh 128-row block
    e = len(out)
    m = -(-6 * e // NB)
    out.extend([-1] * (-(-NB * m // 6) - e))
    nd(adj, B, leaf, out)
    out.extend(rcm(adj, S))


def symbolic(order, adj, n_cam_rows, n_loc):
    n_int = len(order)
    pos = {v: i for i, v in enumerate(order) if v >= 0}
    u_c = 6 * n_int + n_cam_rows
    nb = -(-u_c // NB)
    P = [set() for _ in range(nb + 1)]  # P[j] = block rows i >= j nonzero in column j (nb = RHS)

    def touch(e1, e2):
        for bi in range(6 * e1 // NB, (6 * e1 + 5) // NB + 1):
            for bj in range(6 * e2 // NB, (6 * e2 + 5) // NB + 1):
                if bi >= bj:
                    P[bj].add(bi)
    for v, i in pos.items():
        touch(i, i)
        for w in adj[v]:
            j = pos[w]
            if j < i:
                touch(i, j)
    bl = (6 * n_loc - 1) // NB
    for i in range(bl + 1):
        for j in range(i + 1):
            P[j].add(i)
    T = 6 * n_int // NB
    for j in range(nb):
        P[j].update(range(max(T, j), nb + 1))
    levels = [0] * nb
    tiles = 0
    R = []
    for k in range(nb):
        rk = sorted(i for i in P[k] if i > k)
        R.append(rk)
        tiles += len(rk) * (len(rk) + 1) // 2 - 1  # excluding RHS x RHS
        for a in rk:
            if a < nb:
                P[a].update(b for b in rk if b >= a)
                levels[a] = max(levels[a], levels[k] + 1)
    return nb, max(levels) + 1, tiles, R, levels


def main():
    config = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    leaf = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    n_img, n_tie = synth.CONFIGS[config]
    sc = synth.generate(n_img, n_tie, seed=1000 + config)
    adj = graph(np.asarray(sc["img"]), np.asarray(sc["pid"]), n_img)
    print("images", n_img, "mean degree", np.mean([len(a) for a in adj]))
    cams = 10
    o = rcm(adj, list(range(n_img)))
    nb, h, t, _, _ = symbolic(o, adj, cams, 21)
    print(f"RCM: blocks {nb} waves {h} update tiles {t}")
    for lf in (800, 400, 250, 150, 100):
        out = []
        nd(adj, list(range(n_img)), lf, out)
        nb, h, t, R, lev = symbolic(out, adj, cams, 21)
        npad = sum(1 for v in out if v < 0)
        per = np.bincount(lev)
        print(f"ND leaf {lf}: pad {npad} blocks {nb} waves {h} update tiles {t} cols/wave max {per.max()}"
              f" max |R| {max(len(r) for r in R)}")


if __name__ == "__main__":
    main()
