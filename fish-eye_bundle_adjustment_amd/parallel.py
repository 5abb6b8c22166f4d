"""Multi-GPU Gauss-Newton step: one process per GPU, observations sharded by tie point
(fba_partition), per-rank normal equations summed by an RCCL all-reduce over xGMI.

    rank r:  fba_accumulate      linearise + point-reduce its own observations (no communication)
             all_reduce(S, r)    the only data-path collective: the reduced camera system
             fba_solve_update_async  replicated factor/solve (identical on every rank), back-substitution
                                 of the rank's own tie points, xhat update (enqueued, no host wait)
             all_reduce(share)   this rank's share of sumabs(delta), in place on the device
             fba_solve_finish    the one host synchronisation: the reference's deltasum

torch.distributed is plumbing here (backend "nccl" = RCCL on ROCm, "gloo" on CPU); the compute is
libfba.so.  The context runs on torch's current stream so the collective is ordered after the
accumulation kernels without a host synchronisation.
"""
from __future__ import annotations

import ctypes

import numpy as np


class _CudaArray:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": "<f8", "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def device_view(ptr, n, device):
    """A torch float64 tensor aliasing n doubles of device memory owned by libfba.so."""
    import torch
    return torch.as_tensor(_CudaArray(ptr, n), device=device)


class ShardedStep:
    """One Gauss-Newton iteration across ranks.  ``ctx`` provides accumulate() / solve_update() (a
    capi.Context); the reduce buffer is the context's device buffer unless ``buffer`` (a float64
    tensor aliasing the same storage) is given."""

    def __init__(self, ctx, group=None, device=None, buffer=None):
        import torch
        self.ctx = ctx
        self.group = group
        if buffer is None:
            self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
            ptr, n = ctx.reduce_buffer()
            self.buf = device_view(ptr, n, self.device)
        else:
            self.buf = buffer
            self.device = buffer.device
        # a device context: this rank's deltasum share is all-reduced in place on the device right after
        # the solve, so an iteration has one host round trip (fba_solve_finish); an engine without
        # device memory (the C oracle in tests/test_multirank.py) hands its share over on the host
        self.on_device = hasattr(ctx, "deltasum_device")
        if self.on_device:
            self.share = device_view(ctx.deltasum_device(), 1, self.device)
        else:
            self.share = torch.zeros(1, dtype=torch.float64, device=self.device)

    def __call__(self):
        import torch.distributed as dist
        self.ctx.accumulate()
        dist.all_reduce(self.buf, group=self.group)
        if self.on_device:
            self.ctx.solve_update_async()
            dist.all_reduce(self.share, group=self.group)
            return self.ctx.solve_finish()
        self.share.fill_(self.ctx.solve_update())
        dist.all_reduce(self.share, group=self.group)
        return float(self.share.item())


def reduce_partials(partials):
    """Host-side reference of the collective: elementwise sum in rank order."""
    out = np.zeros_like(partials[0])
    for p in partials:
        out += p
    return out


def hip_memcpy():
    """Raw hipMemcpy for tests that emulate ranks on one GPU."""
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    return lib.hipMemcpy
