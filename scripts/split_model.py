"""The subtree split's cut for a bench scene, on the CPU: the scene's observation structure (synth,
the bench's own generator) written for tests/sched_check.cpp's stats mode, which builds the schedule
for worlds 2, 4 and 8 with the verbose cut report (every candidate cut and its modelled cost,
fba_order.cpp build_schedule).  Measurement aid for DESIGN.md section 7.

    python scripts/split_model.py CONFIG
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    config = int(sys.argv[1])
    import fba_import
    fba_import.load()
    from fba_amd import synth
    n_img, n_tie = synth.CONFIGS[config]
    sc = synth.generate(n_img, n_tie, seed=1000 + config)
    exe = "/tmp/fba_sched_check"
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "sched_check.cpp"),
                    os.path.join(ROOT, "fish-eye_bundle_adjustment_amd", "csrc", "fba_order.cpp"), "-o", exe], check=True)
    path = f"/tmp/fba_obs_c{config}.bin"
    eop = np.concatenate([sc["C0"], sc["ang0"]], 1).astype(np.float64)
    with open(path, "wb") as f:
        f.write(np.int64(len(sc["img"])).tobytes())
        f.write(sc["img"].astype(np.int32).tobytes())
        f.write(sc["pid"].astype(np.int32).tobytes())
        f.write(eop.tobytes())
    r = subprocess.run([exe, str(n_img), "1", path], capture_output=True, text=True)
    for line in (r.stdout + r.stderr).splitlines():
        if "split" in line or line.startswith("ok"):
            print(line)


if __name__ == "__main__":
    main()
