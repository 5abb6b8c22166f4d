"""Report writers (fba_amd/report.py, main.m:631-958) on CPU: the .out / .par / .rsd layout, fed with
the oracle's results for cam0 (the writers are host formatting; the numbers come from the device path
in production, from the dense restatement here)."""
import io
import os

import numpy as np
import pytest

from conftest import CAM0


def test_num2str_and_print_cell(fba):
    from fba_amd import report
    assert report.num2str(3.0) == "3"
    assert report.num2str(0.3) == "0.3"
    assert report.num2str(np.pi) == "3.1416"
    assert report.num2str(123.456) == "123.456"
    assert report.num2str(1e-6) == "1e-06"
    assert report.num2str(2.0 / 3.0, 10) == "0.6666666667"
    assert report.num2str("abc") == "abc"
    fh = io.StringIO()
    col = report.print_cell(fh, [("ab", "1"), ("\\line", ""), ("\\n", ""), ("abcd", "x")], "\t")
    # printCell.m measures every first-column string, the '\line' marker (5 characters) included
    assert fh.getvalue() == "\tab ....... 1\n" + "-" * 15 + "\n\n\tabcd ..... x\n"
    assert col == 12


@pytest.fixture(scope="module")
def cam0_outputs(fba, oracle, tmp_path_factory):
    from fba_amd.bundle import Adjustment
    folder = str(tmp_path_factory.mktemp("rep"))
    for f in os.listdir(CAM0):
        os.symlink(os.path.join(CAM0, f), os.path.join(folder, f))
    ds = fba.load_folder(folder)
    od = oracle.load_folder(folder)
    ro = oracle.adjust(od)
    cxd, corr = oracle.covariance(od, ro)
    u_img, u_cam = oracle.counts(od.settings)
    blocks = []
    for e in range(od.numImg):
        k = int(od.cam_num[np.nonzero(od.ext_index == e)[0][0]])
        idx = list(range(e * u_img, (e + 1) * u_img)) + \
            list(range(u_img * od.numImg + k * u_cam, u_img * od.numImg + (k + 1) * u_cam))
        blocks.append(corr[np.ix_(idx, idx)])
    res = Adjustment(xhat=ro.xhat, xhatnames=ro.names, iterations=ro.iterations, deltasum=np.array(ro.deltasum),
                     v=ro.v, rsd=ro.rsd, rms=ro.rms, sigma02=ro.sigma02, seconds=1.25, cx_diag=cxd,
                     corr=np.array(blocks))
    out_dir = str(tmp_path_factory.mktemp("out"))
    path = fba.bundle.write_outputs(ds, res, out_dir)
    return ds, res, path, out_dir


def test_out_report_layout(cam0_outputs):
    ds, res, path, _ = cam0_outputs
    txt = open(path).read()
    heads = ["Version: ", "Settings used:", "Observations/Unknowns Summary", "Estimated EOPs",
             "Estimated IOPs and Distortions for each Camera", "IOP Correlation sub-matrix",
             "Estimated Ground Coordinates of targets", "Corrected Image Measurements",
             "Absolute (positive) mean correlation coefficients between EOPs and IOPs"]
    pos = [txt.index(h) for h in heads]
    assert pos == sorted(pos)
    lines = txt.splitlines()
    # main.m:636-637's header lines, with this build named as the producer (the reference's author line
    # otherwise attributes these numbers to the MATLAB program)
    assert lines[0].startswith("Version: fba_amd") and lines[0].endswith("Fish-eye model Bundle Adjustment")
    assert lines[1].startswith("Results produced by fba_amd") and "Wynand Tredoux" in lines[1] and lines[2] == ""

    def row(name):
        ln = next(x for x in lines if x.startswith(name + " ."))
        return ln.split()[-1]
    # cam0 Stage-3: u = 580, printed degrees of freedom 1,485
    assert row("Total Unknowns") == "580"
    assert row("Total Degrees of Freedom") == "1485"
    assert row("Number of Inner Constraints") == "7"
    assert float(row("A-Posteriori")) == pytest.approx(res.sigma02, rel=1e-9)
    # first image's Xc: value and sqrt(Cx) in %-W.5f columns
    i = lines.index("Estimated EOPs") + 1
    xc = next(x for x in lines[i:] if x.startswith("Xc "))
    v, s = (float(t) for t in xc.split()[1:3])
    assert v == pytest.approx(res.xhat[0], abs=1e-5)
    assert s == pytest.approx(np.sqrt(res.cx_diag[0]), abs=1e-5)
    # omega in degrees
    om = next(x for x in lines[i:] if x.startswith("Omega "))
    assert float(om.split()[1]) == pytest.approx(np.degrees(res.xhat[3]), abs=1e-5)
    # distortion terms in %e
    k1 = next(x for x in lines if x.startswith("k1 "))
    assert "e" in k1.split()[1]
    # one corrected-measurement row per image point
    c0 = lines.index("PointID\tImageID\tCorrected x\tCorrected y") + 2
    assert float(lines[c0].split()[2]) == pytest.approx(ds.xy[0, 0] + res.rsd[0, 1], abs=1e-5)


def test_par_and_rsd(cam0_outputs):
    ds, res, path, out_dir = cam0_outputs
    name = os.path.splitext(ds.settings["Output_Filename"])[0]
    par = open(os.path.join(out_dir, name + ".par")).read().splitlines()
    # 3 heading rows, then per camera: 'Camera' + xp yp c k1..k5 p1 p2
    assert len(par) == 3 + ds.numCam * (1 + 3 + 5 + 2)
    assert par[3].split("\t")[:2] == ["Camera", ds.INT[0][0]]
    assert par[4].split("\t")[0] == "xp"
    rsd = open(os.path.join(out_dir, name + ".rsd")).read().splitlines()
    assert len(rsd) == ds.n_pts
    f = rsd[0].split("\t")
    assert f[:2] == [ds.pho_target[0], ds.pho_image[0]]
    np.testing.assert_allclose([float(x) for x in f[4:]], res.rsd[0], rtol=1e-14)


def test_batch_find_folders(fba, tmp_path):
    """BatchRun.m's findfiles: complete folders found recursively, partial ones reported and skipped,
    a duplicate extension warns and clears the found list (BatchRun.m:92-96)."""
    from fba_amd import batch
    import shutil
    a = tmp_path / "a"
    shutil.copytree(CAM0, a)
    (tmp_path / "b").mkdir()
    for ext in (".pho", ".ext"):
        (tmp_path / "b" / ("x" + ext)).write_text("")
    shutil.copytree(CAM0, tmp_path / "b" / "deep")
    c = tmp_path / "c"
    shutil.copytree(CAM0, c)
    (c / "zz.pho").write_text("")
    msgs = []
    found = batch.find_folders(str(tmp_path), log=msgs.append)
    assert found == [str(a), str(tmp_path / "b" / "deep")]
    assert any(m.startswith("Error: .ext and .pho were found in") and m.endswith("but not .cnt and .int. This folder "
                                                                                    "will be skipped") for m in msgs)
    assert any(m.startswith("Warning: More than 1 .pho file was found in") for m in msgs)
