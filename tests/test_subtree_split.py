"""CPU, world_size 2 over gloo: the subtree-to-rank split of the reduced camera system.

Design check for distributing the factorisation, not a product path (the product replicates the solve,
fba_amd.parallel.ShardedStep).  The images are cut by nested dissection's first level: A | B along the
median of the image centres, the separator = the images of A that share a tie point with B.  No tie
point then sees images of both A and B, so the tie points are sharded with the subtrees: rank 0 owns the
points seeing an image of A (or only separator images), rank 1 those seeing an image of B.  Each rank
accumulates its points' share of the reduced system with the C oracle as the rank engine (this container
has no GPU), and then
  * its subtree block S_oo comes from its own points only -- it never enters the all-reduce;
  * it eliminates its subtree from the bordered system [S G; G' 0] (inner constraints) and forms its
    share of the Schur complement on the top unknowns y = [separator + camera rows, lambda];
  * ONE all-reduce of those shares (gloo here, RCCL on MI355X) gives the replicated top system, solved on
    every rank; the subtree unknowns follow by local back-substitution.
Bar: the split solve reproduces the single-process KKT solve of the summed system to 1e-9 (relative to
the largest correction), and each rank's subtree block is exactly zero on the other rank.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _split(od, u_img, u_c):
    """Unknown index sets (A, B, top) and the owner rank of every observation."""
    n_img = od.numImg
    pos = np.zeros((n_img, 3))
    for e in range(n_img):
        pos[e] = od.eop_fixed[np.argmax(od.ext_index == e), :3]
    in_a = pos[:, 0] < np.median(pos[:, 0])
    tie = od.tie_index
    sets = {}
    for i in np.flatnonzero(tie >= 0):
        sets.setdefault(int(tie[i]), set()).add(int(od.ext_index[i]))
    sep = np.zeros(n_img, bool)
    for imgs in sets.values():
        ia = [e for e in imgs if in_a[e]]
        if ia and any(not in_a[e] for e in imgs):
            sep[ia] = True
    a_img = np.flatnonzero(in_a & ~sep)
    b_img = np.flatnonzero(~in_a)
    s_img = np.flatnonzero(sep)
    cols = lambda imgs: (imgs[:, None] * u_img + np.arange(u_img)[None, :]).ravel()
    top = np.concatenate([cols(s_img), np.arange(u_img * n_img, u_c)])
    point_rank = {t: (1 if any(not in_a[e] for e in imgs) else 0) for t, imgs in sets.items()}
    owner = np.array([point_rank[int(t)] if t >= 0 else 0 for t in tie])
    return cols(a_img), cols(b_img), top, owner


def _worker(rank, world, port, folder, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import scipy.linalg as sla
    import torch
    import torch.distributed as dist
    import fba_oracle
    import fba_cpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    od = fba_oracle.load_folder(folder)
    eng = fba_cpu.CpuAdjustment(od, threads=1)
    u_c = eng.u_c
    a_idx, b_idx, top, owner = _split(od, 6, u_c)  # synth estimates all six EOPs of every image
    eng.set_shard(owner == rank, count_cam=(rank == 0))
    eng.accumulate()
    S, r, G = eng.S, eng.r, eng.G
    own, other = (a_idx, b_idx) if rank == 0 else (b_idx, a_idx)
    other_zero = not np.any(S[np.ix_(other, other)]) and not np.any(S[np.ix_(own, other)])
    # this rank's subtree eliminated from [S G; G' 0]; its share of the top system (G_t once, on rank 0)
    f = sla.cho_factor(S[np.ix_(own, own)], lower=True)
    Sot = S[np.ix_(own, top)]
    X = sla.cho_solve(f, np.column_stack([Sot, G[own], r[own]]))
    nt = len(top)
    Xs, Xg, Xr = X[:, :nt], X[:, nt:nt + 7], X[:, -1]
    Gt = G[top] if rank == 0 else np.zeros((nt, 7))
    M = np.zeros((nt + 7, nt + 7))
    M[:nt, :nt] = S[np.ix_(top, top)] - Sot.T @ Xs
    M[:nt, nt:] = Gt - Sot.T @ Xg
    M[nt:, :nt] = Gt.T - G[own].T @ Xs
    M[nt:, nt:] = -G[own].T @ Xg
    h = np.concatenate([-r[top] + Sot.T @ Xr, G[own].T @ Xr])
    buf = torch.from_numpy(np.concatenate([M.ravel(), h]))
    dist.all_reduce(buf)  # the one exchange: the top system, (nt + 7)^2 + nt + 7 doubles
    M = buf[: (nt + 7) ** 2].numpy().reshape(nt + 7, nt + 7)
    y = sla.solve(M, buf[(nt + 7) ** 2:].numpy(), assume_a="sym")
    x_t, lam = y[:nt], y[nt:]
    x_o = -Xr - Xs @ x_t - Xg @ lam
    np.savez(os.path.join(out_dir, f"split{rank}.npz"), own=own, x_o=x_o, top=top, x_t=x_t,
             other_zero=other_zero, n_top=nt, n_own=len(own))
    dist.barrier()
    dist.destroy_process_group()


def test_subtree_split_matches_single_solve(fba, oracle, tmp_path):
    import torch.multiprocessing as mp
    import fba_cpu
    from fba_amd import synth
    fba_cpu.build()
    folder = synth.write_folder(synth.generate(200, 4000, seed=21), str(tmp_path / "s"))
    mp.start_processes(_worker, args=(2, _free_port(), folder, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    od = oracle.load_folder(folder)
    ref = fba_cpu.CpuAdjustment(od, threads=1)
    ref.accumulate()
    x_ref = ref._solve()
    outs = [np.load(tmp_path / f"split{k}.npz") for k in range(2)]
    assert all(bool(o["other_zero"]) for o in outs)          # subtree blocks never need the all-reduce
    assert all(int(o["n_top"]) < int(o["n_own"]) for o in outs)  # a real dissection: the top is the smaller part
    x = np.full(ref.u_c, np.nan)
    for o in outs:
        x[o["own"]] = o["x_o"]
        np.testing.assert_array_equal(o["top"], outs[0]["top"])
        np.testing.assert_allclose(o["x_t"], outs[0]["x_t"], rtol=0, atol=1e-12 * np.abs(x_ref).max())
    x[outs[0]["top"]] = outs[0]["x_t"]
    assert np.all(np.isfinite(x))
    err = np.abs(x - x_ref).max() / np.abs(x_ref).max()
    assert err < 1e-9, err
