"""Multi-GPU plumbing for the extraction path.

Extraction shards images across ranks with no data-path collective; the only
collective is making every rank hold rank 0's weights.  All float tensors of
the given state dicts are flattened into ONE buffer and sent with a single
broadcast (RCCL over xGMI on the GPU box, gloo in CPU tests) -- one large
message instead of the reference DDP's per-parameter broadcast at wrap time
and its per-forward buffer broadcasts (PoSFeat_model.py:48-55).
"""
import ctypes

import torch
import torch.distributed as dist


def dist_backend():
    """The process-group backend a rank initialises: RCCL ("nccl") on the GPU
    box.  POSFEAT_DIST_BACKEND=gloo (tests) selects gloo, so several ranks can
    share one device -- RCCL refuses two ranks on the same GPU; the SyncBN
    statistics then take SyncBNGroup's host transport."""
    import os
    return os.environ.get("POSFEAT_DIST_BACKEND", "nccl")


def broadcast_weights(state_dicts, device, src=0):
    """In-place broadcast of every tensor in ``state_dicts`` from ``src``."""
    # gloo broadcasts host tensors (the RCCL path keeps the buffer on the device)
    if dist.get_backend() != "nccl":
        device = "cpu"
    floats, ints = [], []
    for sd in state_dicts:
        for k, v in sd.items():
            (floats if v.is_floating_point() else ints).append(v)
    for group, dtype in ((floats, torch.float32), (ints, torch.int64)):
        if not group:
            continue
        flat = torch.cat([t.detach().reshape(-1).to(dtype) for t in group]).to(device)
        dist.broadcast(flat, src=src)
        off = 0
        for t in group:
            n = t.numel()
            t.data.copy_(flat[off:off + n].view(t.shape).to(t.device, t.dtype))
            off += n


def allreduce_head_grad(grad, group=None):
    """Keypoint-head training (configs/train_kp.yaml under DDP): ONE all-reduce
    (sum) of the flat packed head gradient (2.5 MB; RCCL over xGMI on the GPU
    box, gloo in CPU tests) replaces DDP's bucketed per-parameter all-reduce
    (trainer.py:331, PoSFeat_model.py:53-55).  Returns the factor the SGD step
    applies (1/world: DDP averages gradients over ranks)."""
    if not (dist.is_available() and dist.is_initialized()):
        return 1.0
    world = dist.get_world_size(group)
    if world > 1:
        dist.all_reduce(grad, group=group)
    return 1.0 / world


class SyncBNGroup:
    """SyncBatchNorm group of the train-mode backbone (group.hip): the
    reference converts the backbone to torch.nn.SyncBatchNorm under DDP
    (networks/PoSFeat_model.py:49).  Rank 0 draws an RCCL unique id, the id
    travels by one ``dist.broadcast`` of 128 bytes over the process group
    already initialised (nccl = RCCL on the GPU box, gloo in CPU tests), and
    every rank creates its communicator; the BatchNorm statistics are then
    summed in-stream by ncclAllReduce inside the backbone's forward/backward.
    ``lib`` is injectable for the host-side test of the bootstrap.

    Per BatchNorm the in-stream exchange sums 2 C + 1 doubles -- this rank's
    Σy and Σy² (backward: Σg, Σg·x̂) and its pixel count -- so every rank
    normalises by the group's total count, as torch.nn.SyncBatchNorm does with
    its all-gathered per-rank counts.  Ranks may hold different batches (the
    reference Trainer's loader has no drop_last and my_collate drops None
    samples, managers/trainer.py:132-134).  ``shape`` is accepted for the
    callers that pass it and no longer checked.

    Ordering with torch's own communicator: the SyncBN communicator's
    all-reduces are enqueued on the trainer's stream inside the backbone
    forward/backward, the gradient all-reduce on torch's process group after
    the backward; every rank issues the same sequence (same program, no
    data-dependent collectives), and ProcessGroupNCCL's stream waits for the
    trainer's stream, so the two communicators' collectives never interleave
    differently across ranks (the condition under which two RCCL
    communicators can deadlock)."""

    _HostFn = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_int,
                               ctypes.c_void_p)

    def __init__(self, group=None, lib=None, shape=None, transport=None):
        from . import _lib
        self._lib = lib or _lib.lib()
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.group = group
        self.shape = None if shape is None else tuple(int(v) for v in shape)
        backend = dist.get_backend(group)
        # RCCL in-stream for an RCCL process group; over any other backend
        # (gloo: e.g. ranks that share one device) the host transport
        self.transport = transport or ("rccl" if backend == "nccl" else "host")
        if self.transport == "host":
            self._cb = self._HostFn(self._host_allreduce)   # kept alive with the group
            h = ctypes.c_void_p()
            _lib.check(self._lib.posfeat_group_create_host(
                self.world, self.rank, ctypes.cast(self._cb, ctypes.c_void_p), None,
                ctypes.byref(h)))
            self.handle = h
            return
        id_host = torch.zeros(128, dtype=torch.uint8)
        if self.rank == 0:
            buf = (ctypes.c_ubyte * 128)()
            _lib.check(self._lib.posfeat_group_unique_id(ctypes.addressof(buf)))
            id_host.copy_(torch.frombuffer(bytearray(buf), dtype=torch.uint8))
        dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else "cpu"
        t = id_host.to(dev)
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0,
                       group=group)
        self.id = bytes(t.cpu().numpy().tobytes())
        raw = (ctypes.c_ubyte * 128).from_buffer_copy(self.id)
        h = ctypes.c_void_p()
        _lib.check(self._lib.posfeat_group_create_rccl(self.world, self.rank,
                                                        ctypes.addressof(raw), ctypes.byref(h)))
        self.handle = h

    def _host_allreduce(self, buf, n, user):
        """host transport: sum n doubles in place over the group's ranks"""
        try:
            import numpy as np
            t = torch.from_numpy(np.ctypeslib.as_array(buf, shape=(n,)))
            dist.all_reduce(t, group=self.group)
            return 0
        except Exception:  # noqa: BLE001 - reported to the C side as a failed exchange
            return -1

    def close(self):
        if getattr(self, "handle", None) is not None and self.handle.value:
            self._lib.posfeat_group_destroy(self.handle)
        self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter shutdown
            pass
