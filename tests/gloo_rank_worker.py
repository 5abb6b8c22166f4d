"""One rank of tests/test_gpu_multiprocess.py, started by torch.distributed.run (the launch bench.py
--gpus N uses): every rank on the one GPU of the test box, gloo instead of RCCL.  The rank drives
libfba through fba_amd.parallel.ShardedStep -- fba_accumulate, the all-reduce of the reduce buffer
(device memory, aliased as a torch tensor), fba_solve_update_async, the in-place all-reduce of the
deltasum share, fba_solve_finish -- and writes its deltasums and owned xhat entries.

    python -m torch.distributed.run --nproc-per-node 2 ... tests/gloo_rank_worker.py <folder> <out> <steps> <split>
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(folder, out, steps, split):
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    import fba_import
    fba = fba_import.load()
    from fba_amd.parallel import ShardedStep
    ds = fba.load_folder(folder)
    torch.cuda.set_stream(torch.cuda.Stream(dev))  # as bench.py: the context runs on torch's stream
    stream = torch.cuda.current_stream(dev).cuda_stream
    ctx = fba.capi.Context(ds.pack(), fba.capi.make_settings(ds.settings), device=0, rank=rank, world=world,
                           stream=stream, split=split)
    try:
        step = ShardedStep(ctx, device=dev)
        d = [step() for _ in range(steps)]
        np.savez(os.path.join(out, f"rank{rank}.npz"), d=np.array(d), xhat=ctx.get_xhat(owned_only=True),
                 split=int(ctx.split))
    finally:
        ctx.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4] == "1")
