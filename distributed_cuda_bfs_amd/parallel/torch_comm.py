"""Communicator implemented with ``torch.distributed`` (gloo on CPU).

Lets the native engine run multi-process on the CPU backend with the standard
PyTorch process-group machinery (used by the CPU test-suite).  The engine calls
back into Python with raw host addresses; they are wrapped zero-copy with
``torch.frombuffer``.  GPU runs use the native RCCL communicator instead (see
``runtime.init_runtime``) so that collectives are enqueued on the engine's HIP
stream without a host round-trip.
"""
from __future__ import annotations

import ctypes

from .._native import N


def _view(addr: int, nbytes: int, dtype=None):
    import torch

    if nbytes == 0:
        return torch.empty(0, dtype=dtype or torch.uint8)
    buf = (ctypes.c_uint8 * nbytes).from_address(addr)
    t = torch.frombuffer(buf, dtype=torch.uint8)
    return t.view(dtype) if dtype is not None else t


class TorchComm(N.PyComm):
    def __init__(self, group=None):
        super().__init__()
        import torch.distributed as dist

        if not dist.is_initialized():
            raise RuntimeError("TorchComm needs torch.distributed.init_process_group() first")
        self._dist = dist
        self._group = group
        self._rank = dist.get_rank(group)
        self._size = dist.get_world_size(group)

    def get_rank(self) -> int:
        return self._rank

    def get_size(self) -> int:
        return self._size

    def get_name(self) -> str:
        return "torch." + str(self._dist.get_backend(self._group))

    def py_alltoall(self, send: int, recv: int, nbytes: int) -> None:
        out = _view(recv, nbytes * self._size)
        inp = _view(send, nbytes * self._size).clone()
        self._dist.all_to_all_single(out, inp, group=self._group)

    def py_allgather(self, send: int, recv: int, nbytes: int) -> None:
        inp = _view(send, nbytes).clone()
        out = _view(recv, nbytes * self._size)
        chunks = list(out.chunk(self._size)) if nbytes else [out] * self._size
        self._dist.all_gather(chunks, inp, group=self._group)

    def py_allreduce_sum_i64(self, buf: int, count: int) -> None:
        import torch

        t = _view(buf, 8 * count, torch.int64)
        self._dist.all_reduce(t, group=self._group)

    def py_alltoallv(self, send, sc, sd, recv, rc, rd, eb) -> None:
        import torch

        pieces = [_view(send + sd[i] * eb, sc[i] * eb) for i in range(self._size)]
        inp = torch.cat(pieces) if pieces else torch.empty(0, dtype=torch.uint8)
        out = torch.empty(sum(rc) * eb, dtype=torch.uint8)
        self._dist.all_to_all_single(out, inp, output_split_sizes=[c * eb for c in rc],
                                     input_split_sizes=[c * eb for c in sc], group=self._group)
        off = 0
        for i in range(self._size):
            n = rc[i] * eb
            if n:
                _view(recv + rd[i] * eb, n).copy_(out[off:off + n])
            off += n

    def py_barrier(self) -> None:
        self._dist.barrier(group=self._group)
