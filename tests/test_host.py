"""CPU: host logic around the HIP path -- ingest, packing, unknown layout, partition, the C-ABI
library (loads, exports every symbol of include/fba.h, validates before touching the GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import CAM0, ROOT


def test_library_exports_every_declared_symbol(fba):
    header = open(os.path.join(ROOT, "include", "fba.h")).read()
    declared = set(re.findall(r"\b(fba_[a-z_]+)\s*\(", header))
    assert declared == set(fba.capi.EXPORTS)
    lib = ctypes.CDLL(fba.capi.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert fba.capi.lib.fba_abi_version() == 2


def test_ingest_matches_oracle(fba, oracle, cam0_folders):
    for folder in cam0_folders.values():
        ds = fba.load_folder(folder)
        od = oracle.load_folder(folder)
        assert (ds.numImg, ds.numCam, ds.n, ds.numtie, ds.numGCP) == (od.numImg, od.numCam, od.n, od.numtie, od.numGCP)
        np.testing.assert_array_equal(ds.xy[:, 0], od.x)
        np.testing.assert_array_equal(ds.xy[:, 1], od.y)
        np.testing.assert_array_equal(ds.img, od.ext_index)
        np.testing.assert_array_equal(ds.cam, od.cam_num)
        np.testing.assert_array_equal(ds.tie, od.tie_index)
        np.testing.assert_array_equal(ds.xyz_fixed, od.xyz_fixed)
        for k in ("Meas_std", "Meas_std_y", "type", "threshold", "Iteration_Cap", "Inner_Constraints"):
            assert ds.settings[k] == od.settings[k], k
        _, names = oracle.buildxhat(od)
        assert fba.xhat_names(ds) == names


def test_unknown_count_matches_buildxhat(fba, oracle, cam0_folders):
    for folder in cam0_folders.values():
        ds = fba.load_folder(folder)
        pk = ds.pack()
        x, _ = oracle.buildxhat(oracle.load_folder(folder))
        assert fba.capi.count_unknowns(pk, fba.capi.make_settings(ds.settings)) == len(x)


def test_allgcp_tie_order_is_sorted_unique(fba, tmp_path):
    from conftest import variant_folder
    folder = variant_folder(str(tmp_path), "allgcp", {"Estimate_AllGCP": "1"})
    ds = fba.load_folder(folder)
    assert ds.TIE == sorted(set(ds.pho_target))  # main.m:261-264
    assert (ds.tie >= 0).all()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_partition_is_contiguous_balanced_and_complete(fba, world):
    from fba_amd import synth
    sc = synth.generate(20, 400, seed=5)
    n = len(sc["img"])
    pk = fba.capi.PackedProblem(sc["xy"], sc["img"], np.zeros(n), sc["pid"], np.zeros((n, 3)), np.zeros((20, 6)),
                                np.zeros((1, 10)), np.array([[-1, 0, 0, 2048, 2048]]), sc["X0"], 20, 1, 400)
    tie_owner, ctl_owner = fba.capi.partition(pk, world)
    assert tie_owner.min() >= 0 and tie_owner.max() < world
    assert (np.diff(tie_owner) >= 0).all()  # contiguous ranges
    counts = np.bincount(tie_owner, weights=np.bincount(sc["pid"], minlength=400), minlength=world)
    assert counts.max() - counts.min() <= 2 * 10  # within two points' observations
    assert (ctl_owner == -1).all()


def test_partition_control_points_round_robin(fba, oracle):
    ds = fba.load_folder(CAM0)
    pk = ds.pack()
    t, q = fba.capi.partition(pk, 2)
    ctl = q[ds.tie < 0]
    assert len(ctl) == 17 and set(ctl.tolist()) == {0, 1}
    assert (q[ds.tie >= 0] == -1).all()


def test_create_validates_before_gpu(fba):
    ds = fba.load_folder(CAM0)
    pk = ds.pack()
    s = fba.capi.make_settings(ds.settings)
    s.num_radial = 0
    with pytest.raises(fba.FBAError) as e:
        fba.capi.Context(pk, s)
    assert e.value.code == 5
    s = fba.capi.make_settings(ds.settings)
    s.est_kappa = 0  # inner constraints need all six EOPs (BuildAwG.m:525)
    with pytest.raises(fba.FBAError) as e:
        fba.capi.Context(pk, s)
    assert e.value.code == 5
    s = fba.capi.make_settings(ds.settings)
    s.type = 9
    with pytest.raises(fba.FBAError) as e:
        fba.capi.Context(pk, s)
    assert e.value.code == 2
    bad = dict(ds.settings, type="fishy")
    with pytest.raises(fba.FBAError):
        fba.capi.make_settings(bad)


def test_missing_setting_is_an_error(fba, tmp_path):
    from conftest import variant_folder
    folder = variant_folder(str(tmp_path), "bad", {})
    cfg = os.path.join(folder, "config.cfg")
    lines = [ln for ln in open(cfg) if not ln.startswith("Iteration_Cap")]
    open(cfg, "w").writelines(lines)
    with pytest.raises(fba.IngestError):
        fba.load_folder(folder)
    assert fba.main(folder) == 1


def test_missing_meas_std_fails_as_the_reference_text(fba, oracle, tmp_path):
    """A .cfg without Meas_std: main.m:123-127 sets Meas_std = 1 and no_std_y = 1 but never creates a
    Meas_std_y field, so main.m:399's rmfield fails and the reference stops.  The reference's own text run
    on cam0 without that line (tests/golden/make_ref_golden.py -> ref_cam0_nostd.json) fails exactly
    there; ingest (and the oracle's restatement) raise at the same point, and main() returns the error."""
    import json
    from conftest import variant_folder
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "ref_cam0_nostd.json")))
    assert ref["error"] and "rmfield" in ref["error"] and "Meas_std_y" in ref["error"] and "line 399" in ref["error"]
    folder = variant_folder(str(tmp_path), "nostd", {"Meas_std": None, "Meas_std_y": None})
    assert all(not ln.startswith("Meas_std") for ln in open(os.path.join(folder, "config.cfg")))
    with pytest.raises(fba.IngestError, match="main.m:399"):
        fba.load_folder(folder)
    with pytest.raises(ValueError, match="main.m:399"):
        oracle.load_folder(folder)
    assert fba.main(folder) == 1


def test_synthetic_scene_files_roundtrip(fba, oracle, tmp_path):
    from fba_amd import synth
    sc = synth.generate(9, 100, seed=3)
    folder = synth.write_folder(sc, str(tmp_path / "s"))
    ds = fba.load_folder(folder)
    assert ds.numImg == 9 and ds.numtie == 100 and ds.n_pts == 900
    assert ds.settings["type"] == "fisheye" and ds.settings["Inner_Constraints"] == 1
    od = oracle.load_folder(folder)
    A, w, G, dsc = oracle.build_awg(od, oracle.buildxhat(od)[0])
    # initial misclosure is small (model-consistent observations, perturbed start)
    assert np.sqrt(np.mean(w ** 2)) < 50
