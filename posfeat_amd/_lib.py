"""ctypes binding of libposfeat_hip.so (the C ABI in include/posfeat_hip.h).

The library is loaded lazily on first use and NEVER silently replaced: if the
.so is missing, or no gfx950 device is visible when a GPU op is called, the op
raises.  There is no CPU fallback in the product path.

``torch`` is imported before the library so that the HIP runtime torch bundles
(SONAME libamdhip64.so.7) is the one our library binds to -- one runtime per
process, so torch's caching-allocator pointers and streams are valid here.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("POSFEAT_HIP_LIB", os.path.join(_HERE, "libposfeat_hip.so"))

_lib = None

c_int, c_float, c_void_p, c_size_t = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
c_ll = ctypes.c_longlong
P_int = ctypes.POINTER(ctypes.c_int)


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("n", "h", "w", "cin", "x_cstride", "cout", "kh", "kw",
                                     "stride", "pad", "y_cstride", "res_cstride", "act")]


class ExtractOut(ctypes.Structure):
    _fields_ = [("local_map", c_void_p), ("global_map", c_void_p), ("global_feat", c_void_p),
                ("local_point", c_void_p), ("local_map_small", c_void_p),
                ("local_map_nhwc", c_void_p), ("local_map_cstride", c_int)]


class L2WOut(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("coord1", "coord2", "g1", "g2", "g1_std", "g2_std",
                                        "l1_exp_n", "l2_exp_n", "l1_org_n", "l2_org_n", "valid1",
                                        "valid2", "w1", "w2", "w1_std", "w2_std")]


# name -> (restype, argtypes); mirrors include/posfeat_hip.h
SIGNATURES = {
    "posfeat_strerror": (ctypes.c_char_p, [c_int]),
    "posfeat_abi_version": (c_int, []),
    "posfeat_device_ok": (c_int, []),
    "posfeat_conv_packed_k": (c_int, [c_int, c_int, c_int]),
    "posfeat_set_conv_precision": (c_int, [c_int]),
    "posfeat_conv2d_nhwc": (c_int, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]),
    "posfeat_conv2d_workspace": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "posfeat_conv2d_nhwc_ws": (c_int, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p,
                                       c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "posfeat_conv2d_nhwc_planes": (c_int, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p,
                                           ctypes.c_longlong, c_void_p, c_void_p, c_void_p,
                                           c_void_p, c_size_t, c_int, c_void_p]),
    "posfeat_conv1x1_dual": (c_int, [c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int,
                                     c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                     c_void_p, c_int, c_void_p]),
    "posfeat_conv2d_stats_workspace": (c_size_t, [ctypes.POINTER(ConvDesc)]),
    "posfeat_conv2d_nhwc_stats": (c_int, [ctypes.POINTER(ConvDesc), c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_void_p, c_size_t, c_void_p, c_void_p,
                                          c_float, c_void_p]),
    "posfeat_conv2_up4_weights_floats": (c_size_t, []),
    "posfeat_conv2_up4_workspace": (c_size_t, [c_int, c_int, c_int]),
    "posfeat_conv2_up4_weights": (c_int, [c_void_p, c_void_p, c_void_p]),
    "posfeat_conv2_up4": (c_int, [c_int, c_int, c_int, c_void_p, c_int, c_void_p, c_int, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_size_t,
                                  c_void_p, c_void_p, c_float, c_void_p]),
    "posfeat_detect_workspace": (c_int, [c_int, c_int, c_int, c_int, ctypes.POINTER(c_size_t)]),
    "posfeat_detect": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float, c_int,
                               c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                               c_size_t, c_void_p]),
    "posfeat_ab_build": (c_int, []),
    "posfeat_model_weights_changed": (c_int, [c_void_p]),
    "posfeat_detect_each": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_float,
                                    c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_size_t, c_void_p]),
    "posfeat_sample_desc_each": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                         c_int, c_void_p, c_int, c_void_p, c_void_p]),
    "posfeat_nms_mask": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "posfeat_sample_desc": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int,
                                    c_void_p, c_int, c_void_p, c_void_p]),
    "posfeat_nchw_to_nhwc": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                     c_void_p]),
    "posfeat_nhwc_to_nchw": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                     c_void_p]),
    "posfeat_normalize_rgb8": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p,
                                       c_void_p]),
    "posfeat_line2window_workspace": (c_size_t, [c_int] * 6),
    "posfeat_line2window": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int,
                                    c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_float, c_int, c_float, c_int,
                                    ctypes.POINTER(L2WOut), c_void_p, c_size_t, c_void_p]),
    "posfeat_epipolar_loss": (c_int, [c_int, c_int] + [c_void_p] * 14 + [c_float] * 5 +
                              [c_void_p, c_void_p]),
    "posfeat_disk_loss_workspace": (c_size_t, [c_int, c_int, c_int]),
    "posfeat_disk_loss": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                  c_int, c_int] + [c_void_p] * 8 + [c_float] * 5 +
                          [c_void_p, c_void_p, c_size_t, c_void_p]),
    "posfeat_disk_loss_grad_workspace": (c_size_t, [c_int, c_int, c_int]),
    "posfeat_disk_loss_grad": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int, c_int,
                                       c_int, c_int] + [c_void_p] * 8 + [c_float] * 5 +
                               [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "posfeat_conv_wgrad_workspace": (c_size_t, [c_int] * 7),
    "posfeat_conv_wgrad": (c_int, [c_void_p, c_int, c_void_p, c_int] + [c_int] * 7 +
                           [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "posfeat_sgd": (c_int, [c_void_p, c_void_p, c_ll, c_float, c_void_p]),
    "posfeat_model_create_train": (c_int, [c_int, c_int, c_int, c_void_p,
                                           ctypes.POINTER(c_void_p)]),
    "posfeat_model_head_offset": (c_ll, []),
    "posfeat_model_head_floats": (c_ll, []),
    "posfeat_model_head_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                            c_void_p]),
    "posfeat_wino_workspace": (c_size_t, [c_int] * 5),
    "posfeat_wino_weights": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "posfeat_conv3x3_wino": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                     c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_size_t,
                                     c_void_p]),
    "posfeat_wino6_workspace": (c_size_t, [c_int] * 5),
    "posfeat_wino6_weights": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p]),
    "posfeat_wino6_weights_floats": (c_size_t, [c_int, c_int, c_int]),
    "posfeat_wino6_weights_planes": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "posfeat_conv3x3_wino6_ex": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                         c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int,
                                         c_void_p, c_size_t, c_void_p]),
    "posfeat_wino6_wgrad_workspace": (c_size_t, [c_int] * 5),
    "posfeat_conv3x3_wino6_wgrad": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                            c_int, c_int, c_void_p, c_void_p, c_void_p, c_size_t,
                                            c_void_p]),
    "posfeat_conv3x3_wino6": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p,
                                      c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_size_t,
                                      c_void_p]),
    "posfeat_wino_wgrad_workspace": (c_size_t, [c_int] * 5),
    "posfeat_conv3x3_wino_wgrad": (c_int, [c_void_p, c_int, c_void_p, c_int] + [c_int] * 5 +
                                   [c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    "posfeat_bbtrain_num_layers": (c_int, []),
    "posfeat_bbtrain_layer": (c_int, [c_int, ctypes.POINTER(ctypes.c_char_p), P_int, P_int, P_int,
                                      P_int, P_int, ctypes.POINTER(c_ll)]),
    "posfeat_bbtrain_param_floats": (c_ll, []),
    "posfeat_bbtrain_stat_floats": (c_ll, []),
    "posfeat_bbtrain_create": (c_int, [c_int, c_int, c_int, ctypes.POINTER(c_void_p)]),
    "posfeat_bbtrain_act_bytes": (c_size_t, [c_void_p]),
    "posfeat_bbtrain_scratch_bytes": (c_size_t, [c_void_p]),
    "posfeat_bbtrain_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p,
                                        c_void_p, ctypes.POINTER(c_void_p), c_void_p]),
    "posfeat_bbtrain_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                         c_int, c_void_p, c_void_p]),
    "posfeat_bbtrain_set_timing": (c_int, [c_void_p, c_int]),
    "posfeat_bbtrain_timing_event": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_char_p),
                                             ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]),
    "posfeat_bbtrain_timing_event_arith": (c_int, [c_void_p, c_int]),
    "posfeat_bbtrain_timing": (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double), P_int]),
    "posfeat_bbtrain_destroy": (None, [c_void_p]),
    "posfeat_bbtrain_set_group": (c_int, [c_void_p, c_void_p]),
    "posfeat_group_unique_id": (c_int, [c_void_p]),
    "posfeat_group_create_rccl": (c_int, [c_int, c_int, c_void_p, ctypes.POINTER(c_void_p)]),
    "posfeat_local_group_create": (c_int, [c_int, c_int, ctypes.POINTER(c_void_p)]),
    "posfeat_group_create_local": (c_int, [c_void_p, c_int, ctypes.POINTER(c_void_p)]),
    "posfeat_group_create_host": (c_int, [c_int, c_int, c_void_p, c_void_p,
                                          ctypes.POINTER(c_void_p)]),
    "posfeat_group_destroy": (None, [c_void_p]),
    "posfeat_local_group_destroy": (None, [c_void_p]),
    "posfeat_adam": (c_int, [c_void_p] * 4 + [c_ll] + [c_float] * 5 + [c_ll, c_float, c_void_p]),
    "posfeat_line2window_backward_workspace": (c_size_t, [c_int] * 6),
    "posfeat_line2window_backward": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_int,
                                             c_int, c_int, c_void_p, c_void_p,
                                             ctypes.POINTER(L2WOut), c_void_p, c_float, c_int] +
                                     [c_float] * 6 + [c_void_p, c_int, c_void_p, c_int, c_void_p,
                                                      c_size_t, c_void_p]),
    "posfeat_model_num_specs": (c_int, []),
    "posfeat_model_conv_spec": (c_int, [c_int, ctypes.POINTER(ctypes.c_char_p), P_int, P_int,
                                        P_int, P_int, ctypes.POINTER(c_ll),
                                        ctypes.POINTER(c_ll)]),
    "posfeat_model_weight_floats": (c_ll, []),
    "posfeat_model_create": (c_int, [c_int, c_int, c_int, c_void_p, ctypes.POINTER(c_void_p)]),
    "posfeat_tile_cache_export": (c_int, [ctypes.c_char_p, c_size_t, ctypes.POINTER(c_size_t)]),
    "posfeat_tile_cache_import": (c_int, [ctypes.c_char_p]),
    "posfeat_model_create_shared": (c_int, [c_int, c_int, c_int, c_void_p, c_void_p,
                                            ctypes.POINTER(c_void_p)]),
    "posfeat_model_workspace": (c_size_t, [c_void_p]),
    "posfeat_model_extract": (c_int, [c_void_p, c_void_p, ctypes.POINTER(ExtractOut), c_void_p,
                                      c_size_t, c_void_p]),
    "posfeat_model_backbone": (c_int, [c_void_p, c_void_p, ctypes.POINTER(ExtractOut), c_void_p,
                                       c_size_t, c_void_p]),
    "posfeat_model_keypointdet": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_size_t, c_void_p]),
    "posfeat_model_set_timing": (c_int, [c_void_p, c_int]),
    "posfeat_model_timing": (c_int, [c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), P_int]),
    "posfeat_model_timing_event_arith": (c_int, [c_void_p, c_int]),
    "posfeat_model_timing_event": (c_int, [c_void_p, c_int, ctypes.POINTER(ctypes.c_char_p),
                                           ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]),
    "posfeat_model_destroy": (None, [c_void_p]),
    "posfeat_match_workspace": (c_size_t, [c_int, c_int]),
    "posfeat_disk_flash_lse_workspace": (c_size_t, [c_int, c_int]),
    "posfeat_disk_flash_lse": (c_int, [c_void_p, c_void_p, c_int, c_int, ctypes.c_float, c_void_p,
                                       c_void_p, c_size_t, c_void_p]),
    "posfeat_match": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, ctypes.c_float,
                              c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
}


def lib():
    """Load (once) and return the ctypes library; raise if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                "libposfeat_hip.so not found at %s -- build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C "
                "posfeat_amd/csrc). There is no CPU fallback." % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        _warn_ab_switches(L)
    return _lib


# path switches only the A/B build reads (common.h pf_ab_getenv); the shipped
# library ignores them -- say so instead of silently running the default path
# (POSFEAT_BF6=0 used to select fp32-MFMA convs)
AB_ONLY_SWITCHES = (
    "POSFEAT_BF6", "POSFEAT_BF6B", "POSFEAT_BF6D", "POSFEAT_BF6X", "POSFEAT_BF6X_RB4",
    "POSFEAT_BF6_HALO", "POSFEAT_BF6_STEM", "POSFEAT_CONV_KERNEL", "POSFEAT_CONV_MAXSPLIT",
    "POSFEAT_DISK_FLASH", "POSFEAT_GEMM_B256", "POSFEAT_GFUSE", "POSFEAT_GFUSE_BLOCKS",
    "POSFEAT_GC_ORDER", "POSFEAT_TRAIN_WINO_BF6X", "POSFEAT_WG_TARGET", "POSFEAT_WG_MINCH", "POSFEAT_WINO_WG_TARGET", "POSFEAT_GFUSE_K80", "POSFEAT_HEADFUSE", "POSFEAT_HEAD_UP4", "POSFEAT_IMGSTATS",
    "POSFEAT_S2PHASE", "POSFEAT_SIDE", "POSFEAT_SIDE_AT", "POSFEAT_TRAINTAP",
    "POSFEAT_TRAIN_BN_EPI", "POSFEAT_TRAIN_HALO_BF6", "POSFEAT_TRAIN_TUNE", "POSFEAT_TRAIN_WINO6", "POSFEAT_TRAIN_WINO6_WGRAD",
    "POSFEAT_TUNE_SIMILAR", "POSFEAT_UP2FUSE", "POSFEAT_UP4TAP", "POSFEAT_UP4WINO",
    "POSFEAT_WGRAD_BF6", "POSFEAT_WGRAD_BF6_ALL", "POSFEAT_WINO", "POSFEAT_WINO6",
    "POSFEAT_WINO6_ENC", "POSFEAT_WINO_ENC", "POSFEAT_WINPATCH")


def _warn_ab_switches(L):
    if L.posfeat_ab_build() == 1:
        return
    on = [k for k in AB_ONLY_SWITCHES if k in os.environ]
    if on:
        import warnings
        warnings.warn("%s set but %s is the shipped build, which ignores these A/B path "
                      "switches (build `make -C posfeat_amd/csrc ab` and set POSFEAT_HIP_LIB; "
                      "the conv precision is posfeat_set_conv_precision)"
                      % (", ".join(on), os.path.basename(LIB_PATH)), RuntimeWarning, stacklevel=3)


def check(code):
    if code != 0:
        raise RuntimeError(lib().posfeat_strerror(code).decode())


_DEV_OK = {}


def require_device(t=None):
    """Raise unless a gfx950 GPU is visible (and ``t`` lives on it)."""
    if t is not None and not t.is_cuda:
        raise RuntimeError("posfeat_amd: tensor must be on the GPU (got %s)" % t.device)
    if not torch.cuda.is_available():
        raise RuntimeError("posfeat_amd: no GPU visible; the HIP path has no CPU fallback")
    dev = torch.cuda.current_device()
    ok = _DEV_OK.get(dev)
    if ok is None:
        ok = _DEV_OK[dev] = bool(lib().posfeat_device_ok())
    if not ok:
        raise RuntimeError("posfeat_amd: current device is not gfx950 (MI355X)")


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def bbtrain_table():
    """Train-mode backbone layer table: ([(name, cin, cout, k, stride, has_bias,
    (w_off, b_off, g_off, be_off, rm_off, rv_off))], param_floats, stat_floats)."""
    L = lib()
    layers = []
    for i in range(L.posfeat_bbtrain_num_layers()):
        name = ctypes.c_char_p()
        ci, co, k, s, hb = c_int(), c_int(), c_int(), c_int(), c_int()
        offs = (c_ll * 6)()
        check(L.posfeat_bbtrain_layer(i, ctypes.byref(name), ctypes.byref(ci), ctypes.byref(co),
                                      ctypes.byref(k), ctypes.byref(s), ctypes.byref(hb), offs))
        layers.append((name.value.decode(), ci.value, co.value, k.value, s.value, bool(hb.value),
                       tuple(int(o) for o in offs)))
    return layers, int(L.posfeat_bbtrain_param_floats()), int(L.posfeat_bbtrain_stat_floats())


def model_specs():
    """[(name, cout, cin, kh, kw, w_off, b_off)] from the engine's layer table."""
    L = lib()
    out = []
    for i in range(L.posfeat_model_num_specs()):
        name = ctypes.c_char_p()
        co, ci, kh, kw = c_int(), c_int(), c_int(), c_int()
        wo, bo = c_ll(), c_ll()
        check(L.posfeat_model_conv_spec(i, ctypes.byref(name), ctypes.byref(co), ctypes.byref(ci),
                                        ctypes.byref(kh), ctypes.byref(kw), ctypes.byref(wo),
                                        ctypes.byref(bo)))
        out.append((name.value.decode(), co.value, ci.value, kh.value, kw.value, wo.value,
                    bo.value))
    return out
