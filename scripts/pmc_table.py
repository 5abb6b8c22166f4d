"""DESIGN.md's per-kernel table from committed PMC summaries (scripts/pmc_summary.py output):
    python scripts/pmc_table.py profiles/r06_v1_pmc_config4.json profiles/r06_v7_pmc_config5.json ..."""
import json
import sys

KEYS = ["k_chol_flow", "k_lin_reduce", "k_bwd_flow", "k_red_blocks", "k_backsub", "k_params", "k_red_cam",
        "k_border_rhs", "k_update", "k_sum_parts"]


def main(paths):
    docs = [json.load(open(p)) for p in paths]
    print("| kernel | " + " | ".join(f"config {d['config']}{'' if d.get('network', 'grid') == 'grid' else ' ' + d['network']}"
                                     " µs · MB · GB/s · MFMA" for d in docs) + " |")
    print("|---|" + "---|" * len(docs))
    for k in KEYS:
        cells = []
        for d in docs:
            e = d["kernels"].get(k)
            if not e:
                cells.append("-")
                continue
            mb = e["hbm_bytes_per_launch"] / 1e6
            us = e.get("avg_launch_us")
            gbs = e.get("hbm_GBs")
            mf = e.get("mfma_busy_frac")
            cells.append(f"{us:.1f} · {mb:.0f} · {gbs:.0f} · {mf:.3f}" if us and mf is not None else f"- · {mb:.0f}")
        print(f"| `{k}` | " + " | ".join(cells) + " |")
    print("\nbuild ids: " + ", ".join(f"{p}: {d.get('build_id')}" for p, d in zip(paths, docs)))


if __name__ == "__main__":
    main(sys.argv[1:])
