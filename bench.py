#!/usr/bin/env python3
"""Benchmark: Gauss-Newton iterations/s of the device-resident bundle-adjustment loop.

Workload (BASELINE.json configs[3] = the north-star target scene): synthetic single-camera
fish-eye, 1000 images x 50,000 tie points (500,000 image points, 10 per tie point), inner
constraints, free network, all EOP + IOP + 5 radial + 2 decentering terms, fp64.  A step is one
full Gauss-Newton iteration (BuildAwG linearisation + normal equations + Schur reduction +
bordered Cholesky solve + back-substitution + de-scaling + xhat update + sumabs), inputs resident
in HBM.  With --gpus N (torchrun, one process per GPU) the observations are sharded by tie point
and the reduced system is all-reduced over RCCL (strong scaling of the same scene).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3|4|5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6     # MI355X fp64 matrix (AMD public spec; survey section 8(d))


def scene_folder(config, rank, world, network="grid"):
    from fba_amd import synth
    tag = f"c{config}" + ("" if network == "grid" else f"_{network}")
    folder = os.path.join(os.environ.get("FBA_BENCH_DIR", "/tmp/fba_bench"), tag)
    marker = os.path.join(folder, ".done")
    if rank == 0 and not os.path.exists(marker):
        synth.make_config(config, folder, network=network)
        open(marker, "w").close()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    return folder


def phase_roofline(ds, ms_phase, n_steps):
    """Per-phase algorithmic work ('Measurement') -> roofline numbers."""
    n_pts, nI, nT = ds.n_pts, ds.numImg, ds.numtie
    nk = ds.settings["Num_Radial_Distortions"]
    cw = 5 + nk
    u_c = 6 * nI + cw * ds.numCam
    t = {k: v / n_steps for k, v in ms_phase.items()}
    # Cholesky of the u_c x u_c bordered reduced system + forward solve of its 8 right-hand sides
    chol_flops = u_c ** 3 / 3.0 + 8.0 * u_c ** 2
    lin_bytes = (176 * n_pts + 336 * nT + 744 * nI)
    return t, chol_flops, lin_bytes


def build_id():
    """The identity of the library build this tree runs: a hash of libfba's sources (the HIP kernels, the
    host C++, the public header and the Makefile).  scripts/pmc_summary.py stamps it into every PMC
    summary, so the bench line takes counter data only from a summary of the very build it measured."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(ROOT, "fish-eye_bundle_adjustment_amd", "csrc")
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.cpp")) +
                   glob.glob(os.path.join(csrc, "*.h")) + [os.path.join(csrc, "Makefile"),
                                                           os.path.join(ROOT, "include", "fba.h")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def pmc_summary(config, kernel, network="grid"):
    """The committed rocprofv3 PMC summary of this workload AND this build (profiles/*pmc_config<N>.json
    written by scripts/pmc_summary.py, whose build_id equals build_id()): (file name, the kernel's entry),
    or (None, None) when no summary of this build exists -- then the line carries no counter data rather
    than an older build's."""
    import glob
    tag = f"{config}" + ("" if network == "grid" else f"_{network}")
    bid = build_id()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*pmc_config{tag}.json"))):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("build_id") != bid or d.get("network", "grid") != network:
            continue
        k = d.get("kernels", {}).get(kernel)
        if k:
            return os.path.relpath(f, ROOT), k
    return None, None


def cpu_baseline(folder, seconds):
    """The oracle (test infrastructure) timed on the host: a bounded sample of the same workload.  The
    baseline proper factors the reduced system on the GPU's own block pattern (block-sparse, the same
    nested-dissection order: the ratio compares kernels, not orderings); a shorter sample of the dense
    factorisation follows as a second, labelled number."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import fba_cpu  # C restatement (oracle/fba_cpu.c): OpenMP + OpenBLAS per block / LAPACK
        r = fba_cpu.time_iterations(folder, 0.75 * seconds, solver="sparse")
        rd = fba_cpu.time_iterations(folder, 0.25 * seconds, solver="chol")
    except Exception as e:  # noqa: BLE001
        return {"value": None, "unit": "iter/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}, None
    ph, sm, pat = r["phase_ms"], r["solve_ms"], r["pattern"]
    base = {"value": r["value"], "unit": "iter/s", "cores": r["cores"], "kind": "port",
            "cpu_model": r["cpu_model"], "phase_ms": ph, "solve_ms": sm, "pattern": pat,
            "sample": f"{r['iterations']} full Gauss-Newton iterations of the same scene ({r['n_pts']} image points, "
                      f"u_c={r['u_c']}) in {r['seconds']:.1f} s on {r['cores']} threads of {r['cpu_model']}: "
                      f"oracle/fba_cpu.c -- OpenMP linearise + per-point Schur straight into the 128x128 blocks of "
                      f"the reduced system in the device factorisation's nested-dissection order "
                      f"({ph['linearize_reduce']:.0f} ms/iter), the local inner-constraint border and a "
                      f"level-by-level block Cholesky on the GPU's block pattern ({pat['blocks']} blocks, "
                      f"{pat['levels']} levels; dpotrf / dtrsm / dsyrk / dgemm per block from OpenMP threads, "
                      f"OpenBLAS single-threaded per call; {sm['factor']:.1f} ms factor + "
                      f"{sm['triangular_solves']:.1f} ms solves of 15 right-hand sides, {ph['solve']:.0f} ms/iter "
                      f"with the border) + back-substitution/update ({ph['update']:.0f} ms/iter)"}
    phd = rd["phase_ms"]
    dense = {"value": rd["value"], "unit": "iter/s", "cores": rd["cores"], "kind": "port",
             "phase_ms": phd,
             "sample": f"{rd['iterations']} iterations in {rd['seconds']:.1f} s, the same restatement with the "
                       f"DENSE Cholesky of the bordered reduced system (LAPACK dpotrf/dpotrs, u_c^3/3 flop, "
                       f"{phd['solve']:.0f} ms/iter): no use of the block sparsity"}
    return base, dense


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=4)
    # "convergent": the same counts as a convergent (close-range) network, dense reduced system
    # (synth.generate_convergent) -- a measurement scene, not the headline workload
    ap.add_argument("--network", default="grid", choices=("grid", "convergent"))
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    # N > 1: "replicated" = observations sharded, the summed reduced system factored on every rank (the
    # north star's all-reduce of A'PA / A'Pw); "subtree" = the elimination tree's subtrees factored by the
    # ranks that own their tie points, only the top blocks all-reduced (fba_options.split)
    ap.add_argument("--solve", default=os.environ.get("FBA_BENCH_SOLVE", "replicated"), choices=("replicated", "subtree"))
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    import torch
    # FBA_BENCH_BACKEND=gloo rehearses the multi-rank path with every rank on the one GPU of a test box
    # (device = local rank modulo the visible GPUs); the real runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("FBA_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    import fba_import
    fba = fba_import.load()

    folder = scene_folder(args.config, rank, world, args.network)
    ds = fba.load_folder(folder)
    if world > 1:  # a dedicated stream (capturable: the iteration replays as HIP graphs), RCCL on it too
        torch.cuda.set_stream(torch.cuda.Stream(dev))
    stream = torch.cuda.current_stream(dev).cuda_stream if world > 1 else None
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), device=local, rank=rank, world=world,
                           stream=stream, verbose=args.verbose, split=args.solve == "subtree")
    if world > 1:
        from fba_amd.parallel import ShardedStep
        step = ShardedStep(ctx, device=dev)
    else:
        step = ctx.step

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    dsum = []
    for _ in range(args.steps):
        dsum.append(step())
    torch.cuda.synchronize(dev)
    barrier()
    dt = time.perf_counter() - t0

    # per-phase breakdown, outside the timed region: the same steps with HIP events between the phases
    # (eager launches: the timed loop above replays the captured iteration graphs)
    ctx.set_timing(True)
    phases = np.zeros(8)
    n_phase = max(1, min(args.steps, 3))
    for _ in range(n_phase):
        step()
        phases += ctx.timings()
    ctx.set_timing(False)
    if world > 1:
        import torch.distributed as dist
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())

    names = ["linearize", "point", "accumulate", "border", "cholesky", "backward", "update", "total"]
    ms = {n: float(v) for n, v in zip(names, phases)}
    t, _, lin_bytes = phase_roofline(ds, ms, n_phase)

    # rooflines, outside the timed region: one more step per probed kernel, HIP events around each of
    # its launches on the stream it runs on.  k_chol_flow (the whole block factorisation and forward
    # solve as one persistent dataflow launch) has the largest share of GPU time, so it is `roofline`
    # (FBA_CHOL_FLOW=0: k_panel, one launch per elimination-tree level).
    def probe(kind, name, note):
        ctx.set_probe(kind)
        step()
        pr = ctx.probe_stats()
        ctx.set_probe(0)
        avg_s = pr["ms"] * 1e-3 / max(pr["launches"], 1)
        flops_launch = pr["flops"] / max(pr["launches"], 1)
        # the committed PMC summaries are single-context launches of one build: a subtree-split launch
        # (flow A / B, a fraction of the records) or a build without a summary gets none
        src, pm = (None, None) if ctx.split else pmc_summary(args.config, name, args.network)
        r = {"bound": "mfma", "kernel": f"{name} ({note})",
             "achieved": flops_launch / avg_s / 1e12 if avg_s > 0 else None, "peak": FP64_PEAK_TFLOPS,
             "unit": "TFLOP/s", "launches": pr["launches"], "avg_launch_us": avg_s * 1e6,
             "flops_per_launch": flops_launch,
             "traffic": pm["hbm_bytes_per_launch"] if pm else None,
             "mfma_busy": pm.get("mfma_busy_frac") if pm else None,
             "pmc_summary": src, "build_id": build_id()}
        if pm and pm.get("avg_launch_us"):
            r["traffic_GBs"] = pm["hbm_bytes_per_launch"] / (pm["avg_launch_us"] * 1e-6) / 1e9
        r["frac"] = r["achieved"] / r["peak"] if r["achieved"] else None
        return r
    flow = os.environ.get("FBA_CHOL_FLOW", "1") != "0"
    roof = probe(2, "k_chol_flow", "the whole block Cholesky + forward solve in one persistent dataflow launch: "
                                   "128x128 f64 diagonal-block potrfs, 64-row panel-half solves, 64x64 trailing-"
                                   "update quarters (128x128 whole-block updates when the schedule is throughput-"
                                   "bound), diagonal-block inverses; flops = their algorithmic sum; a "
                                   "latency-bound chain over the elimination-tree levels") if flow else \
        probe(2, "k_panel", "one elimination-tree level: the 128x128 f64 diagonal-block potrf, the panel "
                            "solves and the previous level's trailing updates as in-launch dataflow; a latency-"
                            "bound chain, one launch per level")
    # k_syrk_multi runs only on the per-level path (FBA_CHOL_FLOW=0), for the levels whose updates do not
    # fit into the next level's k_panel launch (and the last level's)
    roof_bulk = probe(1, "k_syrk_multi", "Cholesky trailing update of a level not merged into the next k_panel, "
                                         "64x64 f64 MFMA tiles, K = 128 per source column")
    if not roof_bulk["launches"]:
        roof_bulk = None
    # (no dense-equivalent Cholesky rate: u_c^3/3 over the block-sparse factor's time measures the
    # ordering's sparsity, not the kernel, and exceeds the hardware peak)
    phase_roof = {"linearize_accumulate_GBs": lin_bytes / ((t["linearize"] + t["accumulate"]) * 1e-3) / 1e9}
    value = args.steps / dt
    out = {
        "metric": "Gauss-Newton iter/sec (BuildAwG+solve) and image-point obs/sec",
        "value": value, "unit": "iter/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * dt / args.steps, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"synthetic fish-eye config {args.config}"
                               f"{'' if args.network == 'grid' else ' (' + args.network + ' network)'}: {ds.numImg} "
                               f"images x {ds.numtie} tie points, {ds.n_pts} image points, inner constraints, nK=5",
                   "n_pts": ds.n_pts, "n_img": ds.numImg, "n_tie": ds.numtie, "u": int(ctx.u),
                   "parallelism": f"{'subtree-split' if ctx.split else 'obs-shard'}{world}"},
        "obs_per_s": ds.n_pts * value,
        "phase_ms": {k: t[k] for k in names},
        "deltasum_last": dsum[-1] if dsum else None,
        "roofline": roof,
        **({"roofline_bulk_update": roof_bulk} if roof_bulk else {}),
        "phase_roofline": phase_roof,
    }
    ctx.close()
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"], dense = cpu_baseline(folder, args.cpu_seconds)
        if dense:
            out["cpu_baseline_dense"] = dense
        cb = out["cpu_baseline"]
        if cb.get("value"):
            # how to read the GPU/CPU ratio: per phase, like for like (the CPU's linearise + per-point
            # Schur costs ~cores x its ms per point; the factorisations run on the same block pattern)
            lin_gpu = t["linearize"] + t["point"] + t["accumulate"]
            lin_cpu = cb["phase_ms"]["linearize_reduce"]
            out["gpu_vs_cpu"] = {
                "iteration": value / cb["value"],
                "linearise_reduce": lin_cpu / lin_gpu if lin_gpu > 0 else None,
                "factor": cb["solve_ms"]["factor"] / t["cholesky"] if t["cholesky"] > 0 else None,
                "cpu_linearise_reduce_us_per_point_per_core": 1e3 * lin_cpu * cb["cores"] / ds.n_pts,
                "gpu_linearise_reduce_ns_per_point": 1e6 * lin_gpu / ds.n_pts}
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
