"""The multi-GPU path as the driver runs it, on the one GPU of a test box: two fresh processes started
by torch.distributed.run (tests/gloo_rank_worker.py), each a rank with its own libfba context,
fba_amd.parallel.ShardedStep moving the reduce buffer and the deltasum share through a real process
group (gloo; RCCL on a multi-GPU node, same calls).  Both solves: the replicated
one (observations sharded by tie point, the summed reduced system factored on every rank) and the
subtree split (each rank factors its own subtrees inside fba_accumulate, only the top blocks travel).

Bar at config 3 (200 images x 5k tie points) and at config 4 (1000 images x 50k tie points: BASELINE's
"sharded across 8 GPUs" workload, here two ranks sharing the one GPU -- unmeasured on a multi-GPU node),
three Gauss-Newton passes: the ranks' owned xhat entries reassemble the single context's xhat to 1e-9 per
element and 1e-10 per parameter group (the all-reduce adds the partial systems in another order than one
context does), and the all-reduced deltasum equals the single context's to 1e-9 of the first correction.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT, dist_scaling_of, elem_rel_err, group_rel_err

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def scene_root(tmp_path_factory):
    return tmp_path_factory.mktemp("mp")


def _scene(root, config):
    from fba_amd import synth
    folder = str(root / f"c{config}")
    if not os.path.exists(os.path.join(folder, ".done")):
        synth.make_config(config, folder)
        open(os.path.join(folder, ".done"), "w").close()
    return folder


@pytest.mark.parametrize("config", [3, 4])
@pytest.mark.parametrize("split", [False, True])
def test_two_rank_processes_match_single_context(fba, scene_root, tmp_path, split, config):
    steps = 3
    folder = _scene(scene_root, config)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "gloo_rank_worker.py"), folder, str(tmp_path), str(steps), "1" if split else "0"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    outs = [np.load(tmp_path / f"rank{k}.npz") for k in range(2)]
    assert all(int(o["split"]) == int(split) for o in outs)  # the solve each rank really ran
    ds = fba.load_folder(folder)
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings))
    try:
        d_single = [ctx.step() for _ in range(steps)]
        x_single = ctx.get_xhat()
    finally:
        ctx.close()
    for o in outs:  # every rank returns the all-reduced deltasum
        assert np.all(np.abs(o["d"] - np.array(d_single)) <= 1e-9 * d_single[0]), (o["d"], d_single)
    xr = outs[0]["xhat"] + outs[1]["xhat"]
    names = fba.xhat_names(ds)
    dsc = dist_scaling_of(__import__("fba_oracle").load_folder(folder))
    err = group_rel_err(xr, x_single, names, dsc)
    assert max(err.values()) <= 1e-10, err
    err = elem_rel_err(xr, x_single, names, dsc)
    assert max(err.values()) <= 1e-9, err
