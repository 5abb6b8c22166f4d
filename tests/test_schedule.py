"""CPU: the camera-side ordering and the level schedule of the block Cholesky (fba_order.cpp).

tests/sched_check.cpp orders a synthetic aerial block by nested dissection, builds the per-level
task lists the GPU kernels run (potrf columns, panel-solve tasks, trailing-update targets with their
source columns, backward-solve levels), EMULATES that schedule on the CPU for a random SPD matrix
with the reduced system's block pattern (local border block and dense camera rows included) and
compares factor, forward-solved RHS rows and backward solution with a dense Cholesky: relative
error < 1e-12.  No GPU involved; the kernels themselves are covered by tests/test_gpu_*.py.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("sched") / "sched_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "sched_check.cpp"),
                    os.path.join(ROOT, "fish-eye_bundle_adjustment_amd", "csrc", "fba_order.cpp"), "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("n_img,seed,leaf,merge,block", [
    (40, 1, None, None, None), (300, 2, None, None, None), (300, 1, 60, None, None),
    (420, 3, 100, None, None), (200, 4, 0, None, None), (300, 2, None, 1, None), (300, 1, 60, 2, None),
    # FBA_FLOW_BLOCK: whole-block update tasks -- every group (1, the default of a throughput-bound
    # factorisation), all but the urgent last group (2), the groups with slack (3): whole-block and
    # quarter writers of one target chained
    (300, 2, None, None, 1), (420, 3, 100, None, 2), (300, 1, 60, 2, 3), (40, 1, None, None, 1),
    (300, 2, None, None, "1s1"), (420, 3, 100, None, "1m8")])
def test_level_schedule_matches_dense_cholesky(checker, n_img, seed, leaf, merge, block):
    env = dict(os.environ)
    env.pop("FBA_ND_LEAF", None)
    env.pop("FBA_FLOW_MERGE", None)
    env.pop("FBA_FLOW_BLOCK", None)
    env.pop("FBA_FLOW_SPLIT", None)
    env.pop("FBA_FLOW_MSPLIT", None)
    if block is not None:  # "1s1": one source per record, "1m8": merged groups of up to 8 sources
        env["FBA_FLOW_BLOCK"] = str(block)[0]
        if str(block)[1:2] == "s":
            env["FBA_FLOW_SPLIT"] = str(block)[2:]
        if str(block)[1:2] == "m":
            env["FBA_FLOW_MSPLIT"] = str(block)[2:]
    if leaf is not None:
        env["FBA_ND_LEAF"] = str(leaf)
    if merge is not None:  # writer groups over consecutive source levels (build_flow)
        env["FBA_FLOW_MERGE"] = str(merge)
    r = subprocess.run([checker, str(n_img), str(seed)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), r.stdout + r.stderr
    fields = dict(f.split("=") for f in r.stdout.split()[1:])
    assert int(fields["levels"]) <= int(fields["blocks"])
    if (n_img, seed, leaf, merge, block) == (300, 2, None, None, None):  # targets with > 2 source columns: split and combined
        assert int(fields["split"]) > 0
    if leaf == 60:  # a dissected scene: independent subtrees share levels
        assert int(fields["levels"]) < int(fields["blocks"])


@pytest.mark.parametrize("n_img,seed,leaf,world", [(300, 2, None, 2), (420, 3, 60, 2), (420, 3, 60, 4), (300, 1, 40, 8)])
def test_subtree_split_schedule(checker, n_img, seed, leaf, world):
    """fba_options.split: the elimination tree cut into top columns and per-rank subtrees.  Every rank's
    flow A (its subtree columns: factor, forward solve, Schur updates of the top blocks) runs on the same
    matrix -- their top-block updates add up in place as the ranks' buffers are summed -- then the top
    flow B; the result matches the dense Cholesky (< 1e-12), every column is factored by exactly one
    flow, and a rank's flow writes only its own subtree's blocks and the top blocks."""
    env = dict(os.environ)
    env.pop("FBA_ND_LEAF", None)
    env.pop("FBA_FLOW_MERGE", None)
    if leaf is not None:
        env["FBA_ND_LEAF"] = str(leaf)
    env["SCHED_SPLIT_WORLD"] = str(world)
    r = subprocess.run([checker, str(n_img), str(seed)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("split"), r.stdout + r.stderr
    fields = dict(f.split("=") for f in r.stdout.split() if "=" in f)
    assert int(fields["top_columns"]) < int(fields["blocks"])

