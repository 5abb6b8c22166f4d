"""Write tests/golden/cam0_<variant>.npz: the oracle's run of each cam0 .cfg variant.

These pin the restatement (oracle/fba_oracle.py) against regressions; the restatement itself is
pinned to the reference by tests/golden/jac_golden.json (expression text of BuildAwG.m).
    python tests/golden/make_cam0_golden.py
"""
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))

import fba_oracle as oracle  # noqa: E402
from conftest import CAM0_VARIANTS, variant_folder  # noqa: E402


def main():
    root = tempfile.mkdtemp()
    for name, edits in CAM0_VARIANTS.items():
        d = oracle.load_folder(variant_folder(root, name, edits))
        r = oracle.adjust(d)
        A0, w0, G0, ds0 = oracle.build_awg(d, r.xhat_hist[0])
        rows, cols = np.nonzero(A0)
        np.savez_compressed(
            os.path.join(HERE, f"cam0_{name}.npz"), iterations=r.iterations, xhat=r.xhat,
            names=np.array(r.names), deltasum=np.array(r.deltasum), xhat_hist=np.array(r.xhat_hist),
            sigma02=r.sigma02, rms=np.array(r.rms), v=r.v, rsd=r.rsd, dist_scaling=r.dist_scaling,
            A0_rows=rows.astype(np.int32), A0_cols=cols.astype(np.int32), A0_vals=A0[rows, cols], w0=w0,
            G0=G0 if G0 is not None else np.zeros((0, 7)), A0_shape=np.array(A0.shape))
        print(name, r.iterations, r.sigma02)


if __name__ == "__main__":
    main()
