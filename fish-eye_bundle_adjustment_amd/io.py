"""Reference file interface: .cfg / .pho / .ext / .int / .cnt / .tie (/.cze) ingest and packing.

Mirrors the reference's ingest so a dataset folder that runs in MATLAB runs here:

* ``functions/ReadFiles.m:49``  -- whitespace/tab delimited, runs of delimiters joined, leading
  delimiters ignored, ``#`` comments, blank lines skipped; exactly one file per extension
  (``ReadFiles.m:24-47``; the GUI file pickers are not reproduced: ambiguity is an error).
* ``functions/findSetting.m:7-55`` -- ``Key value``; quoted value -> string, else str2double;
  NaN and 0/1 checks.
* ``main.m:112-177`` -- defaults (Output_Filename, Meas_std, Type 'fisheye', Check_Points 0) and
  the mandatory keys.  ``main.m:60-95`` batch mode: the folder's .cfg, else the project's.
* ``main.m:196-264`` -- omega/phi/kappa degrees -> radians (``x*pi/180``), missing distortion
  terms -> 0, ``Estimate_AllGCP`` -> TIE = sorted unique PHO target ids.
* ``main.m:277-384`` -- per image point joins to EXT / INT / CNT / TIE (first match, as the
  reference's linear scans), cam_num = INT pair order, numImg / numCam / n.  The joins are hash
  lookups instead of the reference's O(n_pts * n_rows) string scans.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

import numpy as np

from .capi import PackedProblem, TYPES


class IngestError(RuntimeError):
    pass


def read_table(path):
    rows = []
    with open(path, "r") as fh:
        for line in fh:
            h = line.find("#")
            if h >= 0:
                line = line[:h]
            toks = line.split()
            if toks:
                rows.append(toks)
    return rows


def find_file(folder, ext, required=True):
    hits = sorted(f for f in os.listdir(folder) if f.endswith(ext) and os.path.isfile(os.path.join(folder, f)))
    if len(hits) == 1:
        return os.path.join(folder, hits[0])
    if not required and not hits:
        return None
    raise IngestError(f"expected exactly one {ext} file in {folder}, found {len(hits)}")


def _num(s):
    try:
        return float(s)
    except ValueError:
        return float("nan")


def find_setting(cfg_rows, key, check01=False):
    """findSetting.m: returns (value, ok)."""
    for row in cfg_rows:
        if row[0] == key:
            sval = row[1] if len(row) > 1 else ""
            if len(sval) >= 1 and sval[0] == "'" and sval[-1] == "'":
                value = sval[1:-1]
            else:
                value = _num(sval)
            if isinstance(value, float) and math.isnan(value):
                return value, False
            if check01 and value not in (0.0, 1.0):
                return value, False
            return value, True
    return -1, False


MANDATORY = [  # (data.settings field, .cfg key, must be 0/1) -- main.m:150-171
    ("Iteration_Cap", "Iteration_Cap", False), ("threshold", "Threshold_Value", False),
    ("Inner_Constraints", "Inner_Constraints", True), ("Estimate_Xc", "Estimate_Xc", True),
    ("Estimate_Yc", "Estimate_Yc", True), ("Estimate_Zc", "Estimate_Zc", True),
    ("Estimate_w", "Estimate_Omega", True), ("Estimate_p", "Estimate_Phi", True),
    ("Estimate_k", "Estimate_Kappa", True), ("Estimate_c", "Estimate_c", True),
    ("Estimate_xp", "Estimate_xp", True), ("Estimate_yp", "Estimate_yp", True),
    ("Estimate_radial", "Estimate_Radial_Distortions", True),
    ("Num_Radial_Distortions", "Num_Radial_Distortions", False),
    ("Estimate_decent", "Estimate_Decentering_Distortions", True), ("Estimate_tie", "Estimate_tie", True),
    ("Estimate_AllGCP", "Estimate_AllGCP", True),
]


def parse_settings(cfg_rows, folder):
    s = {}
    v, ok = find_setting(cfg_rows, "Output_Filename")
    s["Output_Filename"] = v if ok else os.path.basename(os.path.abspath(folder)) + ".out"
    v, ok = find_setting(cfg_rows, "Meas_std")
    if ok:
        s["Meas_std"] = float(v)
        vy, oky = find_setting(cfg_rows, "Meas_std_y")
        s["Meas_std_y"] = float(vy) if oky else float(v)  # main.m:397-402
        s["no_std_y"] = 0 if oky else 1                     # main.m:129 (the .out settings list)
    else:
        # main.m:125-127 sets sigma = 1 and no_std_y = 1 without a Meas_std_y field, so the reference then
        # fails in rmfield at main.m:399 (the reference text run on such a .cfg: tests/golden/
        # ref_cam0_nostd.json); load_folder raises that failure once the joins before it are done
        s["Meas_std"] = 1.0
        s["Meas_std_y"] = 1.0
        s["no_std_y"] = 1
        s["_no_meas_std"] = True
    v, ok = find_setting(cfg_rows, "Type")
    s["type"] = v if ok else "fisheye"
    v, ok = find_setting(cfg_rows, "Check_Points", True)
    s["Check_Points"] = int(v) if ok else 0
    missing = []
    for name, key, c01 in MANDATORY:
        v, ok = find_setting(cfg_rows, key, c01)
        if not ok:
            missing.append(key)
        else:
            s[name] = int(v) if c01 else v
    if missing:
        raise IngestError("Error getting settings: " + ", ".join(missing))
    s["Iteration_Cap"] = int(s["Iteration_Cap"])
    s["Num_Radial_Distortions"] = int(s["Num_Radial_Distortions"])
    s["threshold"] = float(s["threshold"])
    return s


@dataclass
class Dataset:
    """The reference's `data` struct (main.m:280-383) in structure-of-arrays form."""
    folder: str
    settings: dict
    pho_target: list
    pho_image: list
    xy: np.ndarray          # (n_pts, 2)
    img: np.ndarray         # ext_index (0-based)
    cam: np.ndarray         # cam_num (0-based INT pair order)
    tie: np.ndarray         # tieIndex (0-based) or -1
    xyz_fixed: np.ndarray   # (n_pts, 3) CNT coordinates
    EXT: list               # rows [imageID, cameraID, Xc, Yc, Zc, w, p, k] (radians)
    INT: list               # per camera (id, ydir, xmin, ymin, xmax, ymax, [xp yp c K.. P1 P2])
    TIE: list
    CNT: dict               # targetID -> (X, Y, Z) (first occurrence)
    numImg: int
    numCam: int
    numGCP: int
    CZE: list = field(default_factory=list)

    @property
    def n_pts(self):
        return len(self.img)

    @property
    def n(self):
        return 2 * len(self.img)

    @property
    def numtie(self):
        return len(self.TIE)

    def pack(self) -> PackedProblem:
        nk = max(int(self.settings["Num_Radial_Distortions"]), 1)
        eop0 = np.array([r[2:8] for r in self.EXT[: self.numImg]], dtype=np.float64).reshape(-1, 6)
        iop0 = np.array([c[6][: 5 + nk] + [0.0] * max(0, 5 + nk - len(c[6])) for c in self.INT[: self.numCam]],
                        dtype=np.float64).reshape(-1, 5 + nk)
        cam_info = np.array([c[1:6] for c in self.INT[: self.numCam]], dtype=np.float64).reshape(-1, 5)
        tie0 = np.array([self.CNT[t] for t in self.TIE], dtype=np.float64).reshape(-1, 3)
        return PackedProblem(self.xy, self.img, self.cam, self.tie, self.xyz_fixed, eop0, iop0, cam_info, tie0,
                             self.numImg, self.numCam, len(self.TIE))


def load_folder(folder, project_dir=None):
    """main.m:60-384.  `project_dir` is the batch-mode fallback location of the .cfg (main.m:77-80)."""
    cfg_path = find_file(folder, ".cfg", required=project_dir is None)
    if cfg_path is None:
        cfg_path = find_file(project_dir, ".cfg")
    cfg = read_table(cfg_path)
    s = parse_settings(cfg, folder)
    if s["type"] not in TYPES:
        raise IngestError("BuildAwG, invalid type in data.settings.type")
    nK = s["Num_Radial_Distortions"]
    pho = read_table(find_file(folder, ".pho"))
    ext = read_table(find_file(folder, ".ext"))
    cnt = read_table(find_file(folder, ".cnt"))
    intr = read_table(find_file(folder, ".int"))
    TIE = []
    if s["Estimate_tie"] == 1 and s["Estimate_AllGCP"] == 0:  # main.m:180-188
        TIE = [r[0] for r in read_table(find_file(folder, ".tie"))]
    EXT = [[r[0], r[1], _num(r[2]), _num(r[3]), _num(r[4]), _num(r[5]) * math.pi / 180,
            _num(r[6]) * math.pi / 180, _num(r[7]) * math.pi / 180] for r in ext]
    INT = []
    if len(intr) % 2:
        raise IngestError(".int must hold two rows per camera")
    for i in range(0, len(intr), 2):
        r1, r2 = intr[i], intr[i + 1]
        vals = [_num(r2[j]) for j in range(3)]
        for j in range(3, 5 + nK):  # main.m:244-254
            vals.append(_num(r2[j]) if j < len(r2) else 0.0)
        INT.append((r1[0], _num(r1[1]), _num(r1[2]), _num(r1[3]), _num(r1[4]), _num(r1[5]), vals))
    CNT = {}
    for r in cnt:
        if r[0] not in CNT:
            CNT[r[0]] = (_num(r[1]), _num(r[2]), _num(r[3]))
    if s["Estimate_AllGCP"] == 1:  # main.m:261-264
        TIE = sorted(set(r[0] for r in pho))
        s["Estimate_tie"] = 1
    CZE = []
    if s["Check_Points"]:
        CZE = read_table(find_file(folder, ".cze"))

    ext_pos, int_pos, tie_pos = {}, {}, {}
    for j, r in enumerate(EXT):
        ext_pos.setdefault(r[0], j)
    for j, r in enumerate(INT):
        int_pos.setdefault(r[0], j)
    for j, t in enumerate(TIE):
        tie_pos.setdefault(t, j)
    n = len(pho)
    xy = np.empty((n, 2))
    img = np.empty(n, np.int32)
    cam = np.empty(n, np.int32)
    tie = np.empty(n, np.int32)
    xyz = np.empty((n, 3))
    cams_used, cnt_used = set(), set()
    for i, r in enumerate(pho):
        xy[i, 0] = _num(r[2])
        xy[i, 1] = _num(r[3])
        e = ext_pos.get(r[1])
        if e is None:
            raise IngestError(f"Could not find image {r[1]} from .pho in .ext")
        img[i] = e
        k = int_pos.get(EXT[e][1])
        if k is None:
            raise IngestError(f"Could not find camera {EXT[e][1]} from .ext in .int")
        if INT[k][1] not in (1.0, -1.0):
            raise IngestError("y_dir should be +-1 only")
        cam[i] = k
        cams_used.add(EXT[e][1])
        c3 = CNT.get(r[0])
        if c3 is None:
            raise IngestError(f"Could not find target {r[0]} from .pho in .cnt")
        cnt_used.add(r[0])
        xyz[i] = c3
        tie[i] = tie_pos.get(r[0], -1)
    for t in TIE:
        if t not in CNT:
            raise IngestError(f"Error Buildxhat(): can't find {t} from .tie in .cnt")
    numImg = len(set(r[1] for r in pho))
    numCam = len(cams_used)
    if n and (img.max() >= numImg):
        raise IngestError("EXT must list exactly the images measured in .pho, in unknown order (Buildxhat.m:22)")
    if n and (cam.max() >= numCam):
        raise IngestError("INT must list exactly the cameras used, in order (Buildxhat.m:65)")
    if s.pop("_no_meas_std", False):
        # main.m:397-399: no_std_y is set but the Meas_std_y field was never created -> rmfield fails
        raise IngestError("no Meas_std in the .cfg: the reference fails at main.m:399 "
                          "(rmfield of the absent Meas_std_y field)")
    return Dataset(folder=folder, settings=s, pho_target=[r[0] for r in pho], pho_image=[r[1] for r in pho],
                   xy=xy, img=img, cam=cam, tie=tie, xyz_fixed=xyz, EXT=EXT, INT=INT, TIE=TIE, CNT=CNT,
                   numImg=numImg, numCam=numCam, numGCP=len(cnt_used), CZE=CZE)


def xhat_names(ds: Dataset):
    """Buildxhat.m:34-132 unknown names."""
    s = ds.settings
    names = []
    for i in range(ds.numImg):
        r = ds.EXT[i]
        for nm, flag in zip(("Xc", "Yc", "Zc", "w", "p", "k"),
                            ("Estimate_Xc", "Estimate_Yc", "Estimate_Zc", "Estimate_w", "Estimate_p", "Estimate_k")):
            if s[flag]:
                names.append(f"{nm}_{r[0]}_{r[1]}")
    for i in range(ds.numCam):
        cid = ds.INT[i][0]
        for nm, flag in (("xp", "Estimate_xp"), ("yp", "Estimate_yp"), ("c", "Estimate_c")):
            if s[flag]:
                names.append(f"{nm}_{cid}")
        if s["Estimate_radial"]:
            names.extend(f"k{j + 1}_{cid}" for j in range(s["Num_Radial_Distortions"]))
        if s["Estimate_decent"]:
            names.extend(f"p{j + 1}_{cid}" for j in range(2))
    for t in ds.TIE:
        names.extend([f"X_{t}", f"Y_{t}", f"Z_{t}"])
    return names
