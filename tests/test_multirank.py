"""CPU, world_size 2 over gloo: the multi-GPU orchestration (fba_amd.parallel.ShardedStep) end to end.

One process per rank, as bench.py --gpus N runs on MI355X (there over RCCL): each rank owns the
observations fba_partition assigns it, accumulates its share of the point-reduced normal equations,
ShardedStep all-reduces the shared buffer and the deltasum shares, every rank solves the replicated
camera system and updates its own tie points.  The rank engine here is the C restatement
(oracle/fba_cpu.c, same split-step interface as a libfba context) because this container has no GPU;
the GPU engine's shard algebra is covered by tests/test_gpu_parity.py.

Bar: the summed shards reproduce the single-process iterates (xhat 1e-10 relative per group,
deltasum 1e-9 of the first correction -- the all-reduce adds the partial systems in a different
order than one process does).
"""
import os
import socket
import sys

import numpy as np
import pytest

from conftest import group_rel_err

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, folder, out_dir, steps):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import fba_import
    import fba_oracle
    import fba_cpu
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fba = fba_import.load()
    from fba_amd.parallel import ShardedStep
    ds = fba.load_folder(folder)
    od = fba_oracle.load_folder(folder)
    tie_owner, ctl_owner = fba.capi.partition(ds.pack(), world)
    tie = od.tie_index
    owner = np.where(tie >= 0, tie_owner[np.maximum(tie, 0)], ctl_owner)
    eng = fba_cpu.CpuAdjustment(od, threads=1)
    eng.set_shard(owner == rank, count_cam=(rank == 0))
    step = ShardedStep(eng, buffer=torch.from_numpy(eng.flat))
    d = [step() for _ in range(steps)]
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), d=np.array(d), xhat=eng.xhat,
             own=np.unique(tie[(owner == rank) & (tie >= 0)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_sharded_step_over_gloo(fba, oracle, tmp_path, world):
    import torch.multiprocessing as mp
    import fba_cpu
    from fba_amd import synth
    fba_cpu.build()
    folder = synth.write_folder(synth.generate(16, 400, seed=9, n_control=10), str(tmp_path / "s"))
    steps = 3
    mp.start_processes(_worker, args=(world, _free_port(), folder, str(tmp_path), steps), nprocs=world,
                       join=True, start_method="spawn")
    od = oracle.load_folder(folder)
    ref = fba_cpu.CpuAdjustment(od, threads=1)
    d_ref = [ref.step() for _ in range(steps)]
    outs = [np.load(tmp_path / f"rank{r}.npz") for r in range(world)]
    for o in outs:  # every rank returns the same global deltasum
        np.testing.assert_allclose(o["d"], d_ref, rtol=0, atol=1e-9 * d_ref[0])
    u_c = ref.u_c
    x = outs[0]["xhat"].copy()
    for o in outs:
        assert np.array_equal(o["xhat"][:u_c], x[:u_c])  # replicated camera-side solve
        for j in range(3):
            x[u_c + 3 * o["own"] + j] = o["xhat"][u_c + 3 * o["own"] + j]
    dsc = oracle.build_awg(od, ref.xhat)[3]
    err = group_rel_err(x, ref.xhat, ref.names, dsc)
    assert max(err.values()) <= 1e-10, err
