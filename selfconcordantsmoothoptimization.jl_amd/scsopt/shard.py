"""Row sharding of A across ranks (one process per GPU).

The path shards by samples: rank r holds rows ``row_range(N, world, r)`` of
A (and of y), generated or uploaded in place; x and every length-m vector are
replicated.  The only exchange of an iteration is one in-place fp64 sum
(SURVEY.md §8e): [packed lower-triangular Gram tiles ‖ Aᵀv] for
ProxGGNSCORE / ProxNSCORE, the length-m gradient for ProxLQNSCORE, and one
scalar per objective evaluation.  On GPUs (``native=True``, the default with the
"nccl" backend) libscsopt runs the sum itself: an RCCL communicator of its own
(scs_set_comm_rccl; torch.distributed only carries the 128-byte unique id) calls
ncclAllReduce on the context stream, in place, over xGMI.  Otherwise libscsopt
calls back into ``Comm`` at those points and the sum is
``torch.distributed.all_reduce`` (gloo on CPU).  ``force=True`` runs the exchange
path at one rank too, so a one-GPU host exercises the communicator.
"""
from __future__ import annotations

import ctypes as C


def row_range(N, world, rank):
    """Contiguous, balanced [r0, r1) row block of `rank` (first N % world ranks get one more row)."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad rank {rank} / world {world}")
    base, rem = divmod(int(N), int(world))
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


def allreduce_inplace(t, group=None):
    """Sum `t` over the process group in place (the whole exchange step)."""
    import torch.distributed as dist
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t


class Comm:
    """Binds a libscsopt context to a torch.distributed process group."""

    def __init__(self, rank=None, world=None, group=None, device=None, native=None, force=False):
        from . import _lib
        _lib.require_torch_runtime("scsopt.shard.Comm")
        import torch.distributed as dist
        self.rank = dist.get_rank(group) if rank is None else int(rank)
        self.world = dist.get_world_size(group) if world is None else int(world)
        self.group = group
        self.device = device
        if native is None:
            native = dist.get_backend(group) == "nccl"
        self.native = bool(native)
        # a backend that stages device tensors through host memory (gloo) lands the sum from its own
        # stream: the callback then waits for the device before handing back to libscsopt
        self.host_staged = dist.get_backend(group) != "nccl"
        self.force = bool(force)
        self.buf = None
        self._buf_ctx = None   # the context handle the buffer is bound to
        self._cb = None
        self._ctx = None

    @property
    def active(self):
        return self.world > 1 or self.force

    def attach(self, ctx):
        from . import _lib
        self._ctx = ctx
        if self.native:
            import torch.distributed as dist
            uid = C.create_string_buffer(128)
            if self.rank == 0:
                rc = _lib.lib.scs_rccl_unique_id(uid)
                if rc != _lib.SCS_OK:
                    raise _lib.ScsError(rc, "scs_rccl_unique_id failed")
            box = [uid.raw if self.rank == 0 else None]
            dist.broadcast_object_list(box, src=0, group=self.group)
            uid = C.create_string_buffer(box[0], 128)
            ctx._keep.append(uid)
            ctx.check(_lib.lib.scs_set_comm_rccl(ctx.h, self.rank, self.world, uid))
        else:
            self._cb = _lib.ALLREDUCE_FN(self._callback)
            ctx._keep.append(self._cb)
            ctx.check(_lib.lib.scs_set_comm(ctx.h, self.rank, self.world, self._cb, None))
        if self.force:
            ctx.check(_lib.lib.scs_set_comm_force(ctx.h, 1))

    def broadcast_object(self, obj):
        """rank 0's `obj` on every rank (e.g. the shuffled minibatch list: one permutation for all)."""
        import torch.distributed as dist
        box = [obj if self.rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=self.group)
        return box[0]

    def bind_buffer(self, ctx):
        """Allocate the all-reduce payload buffer (torch-owned device memory) once the dims are known;
        the native RCCL path lets libscsopt own it."""
        if self.native:
            return
        import torch
        from . import _lib
        n = C.c_int64()
        ctx.check(_lib.lib.scs_reduce_buffer_size(ctx.h, C.byref(n)))
        fits = self.buf is not None and self.buf.numel() >= int(n.value)
        if fits and self._buf_ctx == ctx.h.value:
            return   # this context already sums in it (a new batch list may need more: set_batches re-binds)
        if not fits:
            dev = torch.device("cuda", ctx.device) if self.device is None else self.device
            self.buf = torch.zeros(int(n.value), dtype=torch.float64, device=dev)
        # a Comm reused for a second Problem (a new context) binds the same buffer to it too
        ctx._keep.append(self.buf)
        ctx.check(_lib.lib.scs_set_reduce_buffer(ctx.h, C.c_void_p(self.buf.data_ptr()), int(self.buf.numel())))
        self._buf_ctx = ctx.h.value

    def _callback(self, dev_ptr, count, stream, user):
        try:
            import torch
            assert self.buf is not None and dev_ptr == self.buf.data_ptr()
            ext = torch.cuda.ExternalStream(stream, device=self.buf.device)
            with torch.cuda.stream(ext):
                allreduce_inplace(self.buf[: int(count)], self.group)
            # the library reads the sum on its stream right after this returns; a process group
            # that copies device tensors through host memory (gloo) lands the result from its own
            # stream, so wait for the device here (measured: without it, back-to-back row
            # all-gathers of the sharded sample-space branch read a partly landed sum).  NCCL
            # (RCCL) enqueues on the external stream itself: no wait.
            if self.host_staged:
                torch.cuda.synchronize(self.buf.device)
            return 0
        except Exception as e:  # surfaced by libscsopt as SCS_ERR_COMM
            import sys
            print(f"[scsopt] all-reduce failed: {e!r}", file=sys.stderr)
            return 1
