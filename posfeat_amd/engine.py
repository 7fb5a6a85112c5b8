"""Python handle over the C++/HIP whole-model engine (posfeat_model_* in the C ABI).

``ExtractionEngine`` owns the packed, BN-folded weight blob on the device
(built once from the reference-layout state dicts, or received by RCCL
broadcast) and one engine instance per input shape.  ``run`` issues the whole
ResUNet + KeypointDet forward on the current stream with a single C call
(~70 kernel launches, no host synchronisation).

Real datasets (HPatches, Aachen) come in many image sizes.  The instances are
kept in a least-recently-used map of at most ``POSFEAT_ENGINE_MAX_SHAPES``
(default 8) shapes, and the inference instances share ONE grow-only workspace
(the workspace is pure per-run scratch; runs are ordered on the caller's
stream), so device memory is bounded by the largest shape seen, not by the
number of shapes.  ``train=True`` instances keep their own workspace: it holds
the head's intermediates between ``run`` and ``head_backward``.  Conv tile
choices are cached process-wide by conv descriptor (engine.hip: tile_cache),
so a new shape times only the convs it has not met.
"""
import ctypes
import os
import time
from collections import OrderedDict

import numpy as np
import torch

from . import _lib, weights
from ._lib import check, lib, ptr, stream_ptr


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TILE_DB = os.path.join(ROOT, "records", "tile_db.txt")
_tile_db_loaded = False


def tile_db_export(path):
    """Write the process-wide conv tile choices (posfeat_tile_cache_export)."""
    need = ctypes.c_size_t()
    check(lib().posfeat_tile_cache_export(None, 0, ctypes.byref(need)))
    buf = ctypes.create_string_buffer(need.value)
    check(lib().posfeat_tile_cache_export(buf, need.value, ctypes.byref(need)))
    with open(path, "w") as f:
        f.write(buf.value.decode())
    return buf.value.decode().count("\n")


def tile_db_import(path):
    """Add a tile database's entries to the process-wide choices; returns how many."""
    with open(path) as f:
        return int(lib().posfeat_tile_cache_import(f.read().encode()))


def _load_tile_db():
    """Once per process: the tuning database shipped in records/ (made by
    tools/tile_db.py on an MI355X; POSFEAT_TILE_DB = another file, or 0 for
    none).  An extraction conv's tiles never change its results, only which
    candidate runs; the training step (BackboneTrainer) uses only the exact
    entries for its convs, so every rank and run picks the same tiles."""
    global _tile_db_loaded
    if _tile_db_loaded:
        return
    _tile_db_loaded = True
    path = os.environ.get("POSFEAT_TILE_DB", TILE_DB)
    if path != "0" and os.path.exists(path):
        tile_db_import(path)


class ExtractionEngine:
    """``train=True`` builds instances that keep the head's intermediates for
    ``head_backward`` (keypoint-head training, configs/train_kp.yaml)."""

    def __init__(self, backbone_sd=None, head_sd=None, device="cuda", blob=None, train=False):
        _lib.require_device()
        _load_tile_db()
        self.train = bool(train)
        self.device = torch.device(device)
        self.specs = _lib.model_specs()
        nfl = lib().posfeat_model_weight_floats()
        if blob is None:
            host = weights.pack_for_device(backbone_sd, head_sd, self.specs)
            blob = torch.from_numpy(np.ascontiguousarray(host))
        if blob.numel() > nfl:
            raise ValueError("weight blob larger than the engine layout")
        self.wdev = torch.zeros(nfl, dtype=torch.float32, device=self.device)
        self.wdev[:blob.numel()].copy_(blob.reshape(-1).to(self.device))
        self._inst = OrderedDict()   # (b, h, w) -> (handle, workspace bytes)
        self._own_ws = {}            # train=True: (b, h, w) -> own workspace
        self._shared_ws = None       # train=False: one grow-only workspace
        self.max_shapes = max(1, int(os.environ.get("POSFEAT_ENGINE_MAX_SHAPES", "8")))
        self.stats = {"instances_created": 0, "create_s": 0.0, "workspace_grows": 0}
        # torch's version counter of the blob: an in-place torch write to wdev
        # (or a view of it, e.g. head_weights()) rebuilds the derived weights
        # before the next forward
        self._wver = self.wdev._version

    # ------------------------------------------------------------------
    def _instance(self, b, h, w):
        key = (b, h, w)
        if self._wver != self.wdev._version:   # wdev written in place by a torch op
            self._wver = self.wdev._version
            self.weights_changed()
        inst = self._inst.get(key)
        if inst is None:
            handle = ctypes.c_void_p()
            t0 = time.perf_counter()
            if self.train:
                check(lib().posfeat_model_create_train(b, h, w, ptr(self.wdev),
                                                       ctypes.byref(handle)))
            else:
                # extraction instances share one derived-weight store (bf16
                # planes, Winograd U): built once per engine, not per shape
                share = next(iter(self._inst.values()))[0] if self._inst else None
                check(lib().posfeat_model_create_shared(b, h, w, ptr(self.wdev), share,
                                                        ctypes.byref(handle)))
            inst = (handle, int(lib().posfeat_model_workspace(handle)))
            self.stats["instances_created"] += 1
            self.stats["create_s"] += time.perf_counter() - t0
            # the least recently used instances leave after the new one holds
            # the shared store
            while len(self._inst) >= self.max_shapes:
                old, (oh, _) = self._inst.popitem(last=False)
                lib().posfeat_model_destroy(oh)
                self._own_ws.pop(old, None)
            self._inst[key] = inst
        else:
            self._inst.move_to_end(key)
        handle, nbytes = inst
        if self.train:
            ws = self._own_ws.get(key)
            if ws is None:
                ws = self._own_ws[key] = torch.empty(nbytes + 256, dtype=torch.uint8,
                                                     device=self.device)
        else:
            ws = self._shared_ws
            if ws is None or ws.numel() < nbytes + 256:
                self.stats["workspace_grows"] += 1
                self._shared_ws = None
                ws = self._shared_ws = torch.empty(nbytes + 256, dtype=torch.uint8,
                                                   device=self.device)
        return handle, ws, (-ws.data_ptr()) % 256

    def reserve(self, shapes):
        """Grow the shared workspace once to the largest need over ``shapes``
        ((b, h, w) tuples) instead of once per larger shape met: a workspace
        grow is a device allocation (tens of GB at Aachen / HPatches sizes)
        taken while the pipeline waits.  Planning a shape is host work only
        (posfeat_model_create allocates nothing)."""
        if self.train:
            return
        need = self._shared_ws.numel() if self._shared_ws is not None else 0
        for b, h, w in set(shapes):
            if (b, h, w) in self._inst:
                need = max(need, self._inst[(b, h, w)][1] + 256)
                continue
            handle = ctypes.c_void_p()
            check(lib().posfeat_model_create(b, h, w, ptr(self.wdev), ctypes.byref(handle)))
            need = max(need, int(lib().posfeat_model_workspace(handle)) + 256)
            lib().posfeat_model_destroy(handle)
        if self._shared_ws is None or self._shared_ws.numel() < need:
            self.stats["workspace_grows"] += 1
            self._shared_ws = None
            self._shared_ws = torch.empty(need, dtype=torch.uint8, device=self.device)

    def weights_changed(self):
        """Call after rewriting ``wdev`` in place: every extraction instance
        rebuilds its derived weights (bf16 planes, Winograd-domain weights) at
        its next forward (posfeat_model_weights_changed)."""
        for handle, _ in self._inst.values():
            check(lib().posfeat_model_weights_changed(handle))

    @property
    def cached_shapes(self):
        return list(self._inst.keys())

    @property
    def workspace_bytes(self):
        """device bytes held in engine workspaces"""
        n = sum(t.numel() for t in self._own_ws.values())
        return n + (self._shared_ws.numel() if self._shared_ws is not None else 0)

    def set_timing(self, b, h, w, enable=True):
        handle, _, _ = self._instance(b, h, w)
        check(lib().posfeat_model_set_timing(handle, 1 if enable else 0))

    def timing(self, b, h, w, prefix):
        """(ms, flops, launches) summed over launches whose label starts with prefix
        in the last timed run (host-synchronises)."""
        handle, _, _ = self._instance(b, h, w)
        ms, fl, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        check(lib().posfeat_model_timing(handle, prefix.encode(), ctypes.byref(ms),
                                         ctypes.byref(fl), ctypes.byref(n)))
        return ms.value, fl.value, n.value

    def timing_events(self, b, h, w, arith=False):
        """[(label, ms, flops)] of every timed launch of the last run
        (host-synchronises); ``arith=True`` appends the arithmetic mask of the
        label's MFMA launches (1 fp32 MFMA, 2 bf16x6, 3 both, 0 none)."""
        handle, _, _ = self._instance(b, h, w)
        out, i = [], 0
        lab, ms, fl = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_double()
        while lib().posfeat_model_timing_event(handle, i, ctypes.byref(lab), ctypes.byref(ms),
                                               ctypes.byref(fl)) == 0:
            ev = (lab.value.decode(), ms.value, fl.value)
            if arith:
                ev += (int(lib().posfeat_model_timing_event_arith(handle, i)),)
            out.append(ev)
            i += 1
        return out

    def run(self, img, outputs=("local_map", "global_map", "global_feat", "local_map_small")):
        """img: [b,3,h,w] fp32 on the device (h, w multiples of 16).

        Returns a dict of NCHW tensors plus ``_local_map_nhwc`` -- a view into
        the engine workspace (valid until the next ``run`` of this engine).
        """
        if img.dtype != torch.float32 or img.dim() != 4 or img.shape[1] != 3:
            raise ValueError("img must be float32 [b,3,h,w]")
        img = img.contiguous()
        _lib.require_device(img)
        b, _, h, w = img.shape
        if h % 16 or w % 16:
            raise ValueError("image height/width must be multiples of 16 (datasets crop to /16)")
        handle, ws, off = self._instance(b, h, w)
        dev = img.device
        res = {"local_point": torch.empty(b, 1, h, w, device=dev)}
        if "local_map" in outputs:
            res["local_map"] = torch.empty(b, 128, h // 4, w // 4, device=dev)
        if "global_map" in outputs:
            res["global_map"] = torch.empty(b, 128, h // 16, w // 16, device=dev)
        if "global_feat" in outputs:
            res["global_feat"] = torch.empty(b, 128, device=dev)
        if "local_map_small" in outputs:
            res["local_map_small"] = torch.empty(b, 64, h // 4, w // 4, device=dev)
        o = _lib.ExtractOut()
        for k in ("local_map", "global_map", "global_feat", "local_point", "local_map_small"):
            setattr(o, k, res[k].data_ptr() if k in res else None)
        check(lib().posfeat_model_extract(handle, ptr(img), ctypes.byref(o),
                                          ctypes.c_void_p(ws.data_ptr() + off),
                                          ws.numel() - off, stream_ptr()))
        base = o.local_map_nhwc - ws.data_ptr()
        cs = o.local_map_cstride
        nfl = b * (h // 4) * (w // 4) * cs
        res["_local_map_nhwc"] = ws[base:base + nfl * 4].view(torch.float32).view(
            b, h // 4, w // 4, cs)
        return res

    def run_backbone(self, img, outputs=("local_map", "global_map", "local_map_small")):
        """ResUNet.forward alone (DescNet.py:64-84): NCHW maps of img [b,3,h,w]."""
        img, (handle, ws, off), b, h, w = self._prep(img)
        dev = img.device
        res = {}
        if "local_map" in outputs:
            res["local_map"] = torch.empty(b, 128, h // 4, w // 4, device=dev)
        if "global_map" in outputs:
            res["global_map"] = torch.empty(b, 128, h // 16, w // 16, device=dev)
        if "global_feat" in outputs:
            res["global_feat"] = torch.empty(b, 128, device=dev)
        if "local_map_small" in outputs:
            res["local_map_small"] = torch.empty(b, 64, h // 4, w // 4, device=dev)
        o = _lib.ExtractOut()
        for k in ("local_map", "global_map", "global_feat", "local_map_small"):
            setattr(o, k, res[k].data_ptr() if k in res else None)
        check(lib().posfeat_model_backbone(handle, ptr(img), ctypes.byref(o),
                                           ctypes.c_void_p(ws.data_ptr() + off),
                                           ws.numel() - off, stream_ptr()))
        return res

    def run_keypointdet(self, x, img):
        """KeypointDet.forward([x, img]) alone (DeteNet.py:102-121): x =
        cat[local_map, local_map_small] [b,192,h/4,w/4], img [b,3,h,w] ->
        local_point [b,1,h,w]."""
        img, (handle, ws, off), b, h, w = self._prep(img)
        x = x.float().contiguous()
        _lib.require_device(x)
        if tuple(x.shape) != (b, 192, h // 4, w // 4):
            raise ValueError("x must be [b,192,h/4,w/4] = cat[local_map, local_map_small]")
        lp = torch.empty(b, 1, h, w, device=img.device)
        check(lib().posfeat_model_keypointdet(handle, ptr(x), ptr(img), ptr(lp),
                                              ctypes.c_void_p(ws.data_ptr() + off),
                                              ws.numel() - off, stream_ptr()))
        return lp

    def _prep(self, img):
        if img.dtype != torch.float32 or img.dim() != 4 or img.shape[1] != 3:
            raise ValueError("img must be float32 [b,3,h,w]")
        img = img.contiguous()
        _lib.require_device(img)
        b, _, h, w = img.shape
        if h % 16 or w % 16:
            raise ValueError("image height/width must be multiples of 16 (datasets crop to /16)")
        return img, self._instance(b, h, w), b, h, w

    # ------------------------------------------------------------ training
    @property
    def head_offset(self):
        return int(lib().posfeat_model_head_offset())

    @property
    def head_floats(self):
        return int(lib().posfeat_model_head_floats())

    def head_weights(self):
        """View of the trainable KeypointDet region of the device blob."""
        return self.wdev[self.head_offset:self.head_offset + self.head_floats]

    def head_backward(self, dlocal_point, grad=None):
        """dL/d(head params) (packed like ``head_weights()``) from dL/d local_point
        [b,1,h,w] of the last ``run`` of that shape.  Needs ``train=True``."""
        if not self.train:
            raise RuntimeError("head_backward needs an engine built with train=True")
        b, _, h, w = dlocal_point.shape
        handle, ws, off = self._instance(b, h, w)
        if grad is None:
            grad = torch.empty(self.head_floats, dtype=torch.float32, device=self.device)
        dl = dlocal_point.float().contiguous()
        _lib.require_device(dl)
        check(lib().posfeat_model_head_backward(handle, ptr(dl), ptr(grad),
                                                ctypes.c_void_p(ws.data_ptr() + off),
                                                ws.numel() - off, stream_ptr()))
        return grad

    def sgd_step(self, grad, lr):
        """torch.optim.SGD (no momentum) on the head region: w -= lr * grad."""
        check(lib().posfeat_sgd(ptr(self.head_weights()), ptr(grad), self.head_floats,
                                float(lr), stream_ptr()))
        self.weights_changed()   # written by a kernel: torch's version counter does not see it

    def close(self):
        for handle, _ in self._inst.values():
            lib().posfeat_model_destroy(handle)
        self._inst.clear()
        self._own_ws.clear()
        self._shared_ws = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _module_key(module, device):
    return (id(module), tuple(p._version for p in module.state_dict(keep_vars=True).values()),
            str(device))


class _ModuleEngines:
    """One ExtractionEngine per (module, parameter versions, device): rebuilt
    (weights re-packed) only when the module's parameters change."""

    def __init__(self):
        self._c = {}

    def get(self, module, device, make):
        key = _module_key(module, device)
        eng = self._c.get(key)
        if eng is None:
            for k in [k for k in self._c if k[0] == id(module)]:
                self._c.pop(k).close()
            eng = make()
            self._c[key] = eng
        return eng


_BB = _ModuleEngines()
_KD = _ModuleEngines()


def backbone_forward(module, x):
    """ResUNet.forward through the engine's backbone-only mode (DescNet.py:64-84
    outputs); KeypointDet is not run."""
    if module.training:
        raise NotImplementedError(
            "train-mode (batch-statistics BN) ResUNet.forward runs in training.BackboneTrainer; "
            "call .eval() for the eval-mode forward")
    eng = _BB.get(module, x.device, lambda: ExtractionEngine(
        module.state_dict(), {k: torch.zeros(s) for k, s in weights.head_param_shapes()},
        device=x.device))
    return eng.run_backbone(x.float())


def keypointdet_forward(module, x, img):
    """KeypointDet.forward([x, img]) through the engine's head-only mode."""
    eng = _KD.get(module, img.device, lambda: ExtractionEngine(
        {k: torch.zeros(s) for k, s in weights.backbone_param_shapes()}, module.state_dict(),
        device=img.device))
    return eng.run_keypointdet(x, img.float())
