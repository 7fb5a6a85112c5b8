"""Drive the host-side logic of the C ABI through the AddressSanitizer build
(build/asan/libposfeat_hip_asan.so, `make -C posfeat_amd/csrc asan`: host code
only, compiled with -fsanitize=address).  Run under the clang ASan runtime:

  LD_PRELOAD=<libclang_rt.asan-x86_64.so> ASAN_OPTIONS=detect_leaks=0 \
      python tools/asan_host.py build/asan/libposfeat_hip_asan.so

Covers what runs on the host before any device work: argument validation of
every entry point that takes sizes (invalid descriptors, null pointers,
negative / zero / odd sizes), conv planning and workspace sizing over the
model's layer table and ragged shapes, the model's layer-spec table, the
engine's and the descriptor trainer's instance planning (posfeat_model_create /
_create_train / posfeat_bbtrain_create: a dry pass over every layer that sizes
the workspace), and the string tables.  No torch import (the ASan runtime
must own malloc before any other library loads); no kernel is launched (the
host-only build has no device code).  Prints one line per section and exits
non-zero on a failed check; ASan aborts the process on any memory error."""
import ctypes
import sys

c_int, c_size_t, c_void_p, c_ll = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_longlong


class ConvDesc(ctypes.Structure):  # include/posfeat_hip.h posfeat_conv_desc
    _fields_ = [(n, c_int) for n in ("n", "h", "w", "cin", "x_cstride", "cout", "kh", "kw",
                                     "stride", "pad", "y_cstride", "res_cstride", "act")]


def check(cond, what):
    if not cond:
        print("FAIL:", what)
        sys.exit(1)


def main():
    L = ctypes.CDLL(sys.argv[1])
    L.posfeat_strerror.restype = ctypes.c_char_p
    for f in ("posfeat_conv2d_workspace", "posfeat_conv2d_stats_workspace",
              "posfeat_conv2_up4_workspace", "posfeat_line2window_workspace",
              "posfeat_line2window_backward_workspace", "posfeat_disk_loss_workspace",
              "posfeat_disk_loss_grad_workspace", "posfeat_disk_flash_lse_workspace",
              "posfeat_match_workspace", "posfeat_conv_wgrad_workspace",
              "posfeat_wino_wgrad_workspace", "posfeat_wino_workspace",
              "posfeat_model_workspace", "posfeat_bbtrain_act_bytes",
              "posfeat_bbtrain_scratch_bytes"):
        getattr(L, f).restype = c_size_t
    for f in ("posfeat_model_head_offset", "posfeat_model_head_floats",
              "posfeat_model_weight_floats", "posfeat_bbtrain_param_floats",
              "posfeat_bbtrain_stat_floats"):
        getattr(L, f).restype = c_ll

    # string table and constants
    for code in range(-12, 2):
        check(L.posfeat_strerror(code) is not None, "strerror %d" % code)
    check(L.posfeat_abi_version() == 1, "abi")
    check(L.posfeat_conv_packed_k(3, 7, 7) == 224, "packed_k")
    print("strings/constants ok")

    # the layer table
    n = L.posfeat_model_num_specs()
    check(n > 50, "num specs")
    name = ctypes.c_char_p()
    vals = [c_int() for _ in range(4)]
    offs = [c_ll() for _ in range(2)]

    def spec(i):
        return L.posfeat_model_conv_spec(i, ctypes.byref(name), *[ctypes.byref(v) for v in vals],
                                         *[ctypes.byref(o) for o in offs])
    for i in range(n):
        check(spec(i) == 0 and name.value, "spec %d" % i)
    check(spec(n) != 0 and spec(-1) != 0, "spec out of range")
    check(L.posfeat_model_conv_spec(0, None, None, None, None, None, None, None) == 0,
          "spec with null outputs")
    check(L.posfeat_model_weight_floats() > 0 and L.posfeat_model_head_floats() > 0, "floats")
    nb = L.posfeat_bbtrain_num_layers()
    for i in range(nb):
        v5 = [c_int() for _ in range(5)]
        o6 = (c_ll * 6)()
        check(L.posfeat_bbtrain_layer(i, ctypes.byref(name), *[ctypes.byref(v) for v in v5],
                                      o6) == 0, "bbtrain layer %d" % i)
    v5 = [c_int() for _ in range(5)]
    check(L.posfeat_bbtrain_layer(nb, ctypes.byref(name), *[ctypes.byref(v) for v in v5],
                                  (c_ll * 6)()) != 0, "bbtrain layer out of range")
    print("layer tables ok (%d model convs, %d train layers)" % (n, nb))

    # conv planning and workspace sizing over many shapes (incl. ragged / tiny)
    cnt = 0
    for (cin, cout, k, s) in ((4, 64, 7, 2), (64, 64, 3, 1), (256, 64, 1, 1), (64, 256, 1, 1),
                              (512, 1024, 1, 2), (1024, 256, 1, 1), (192, 1152, 1, 1),
                              (512, 256, 3, 1), (256, 128, 3, 1), (3, 64, 3, 1), (1152, 192, 1, 1)):
        for (nn, h, w) in ((1, 7, 9), (2, 31, 41), (32, 120, 160), (1, 1, 1), (3, 480, 640)):
            d = ConvDesc(n=nn, h=h, w=w, cin=cin, x_cstride=(cin + 3) // 4 * 4, cout=cout, kh=k,
                         kw=k, stride=s, pad=(k - 1) // 2, y_cstride=cout, res_cstride=0, act=1)
            L.posfeat_conv2d_workspace(ctypes.byref(d))
            L.posfeat_conv2d_stats_workspace(ctypes.byref(d))
            cnt += 1
    bad = ConvDesc(n=1, h=8, w=8, cin=3, x_cstride=3, cout=8, kh=3, kw=3, stride=1, pad=1,
                   y_cstride=8, res_cstride=0, act=0)
    check(L.posfeat_conv2d_nhwc(ctypes.byref(bad), c_void_p(16), c_void_p(16), None, None,
                                c_void_p(16), None) != 0, "bad x_cstride")
    for field, v in (("n", 0), ("h", -1), ("cout", 0), ("stride", 0), ("kh", 0), ("act", 9)):
        d = ConvDesc(n=1, h=8, w=8, cin=32, x_cstride=32, cout=8, kh=3, kw=3, stride=1, pad=1,
                     y_cstride=8, res_cstride=0, act=0)
        setattr(d, field, v)
        check(L.posfeat_conv2d_nhwc(ctypes.byref(d), c_void_p(16), c_void_p(16), None, None,
                                    c_void_p(16), None) != 0, "bad %s" % field)
        L.posfeat_conv2d_workspace(ctypes.byref(d))
    check(L.posfeat_conv2d_nhwc(None, None, None, None, None, None, None) != 0, "null desc")
    print("conv planning ok (%d shapes)" % cnt)

    # other sizing / validation entry points
    nbytes = c_size_t()
    check(L.posfeat_detect_workspace(1, 480, 640, 2048, ctypes.byref(nbytes)) == 0, "detect ws")
    check(L.posfeat_detect_workspace(0, 480, 640, 2048, ctypes.byref(nbytes)) != 0, "detect b=0")
    check(L.posfeat_detect_workspace(1, 2, 640, 2048, ctypes.byref(nbytes)) != 0, "detect h=2")
    for args in ((1, 480, 640), (32, 480, 640), (1, 96, 208), (0, 480, 640), (1, 17, 640)):
        L.posfeat_conv2_up4_workspace(*args)
    for args in ((8, 480, 640, 480, 640, 16), (1, 64, 64, 64, 64, 16), (0, 64, 64, 64, 64, 16)):
        L.posfeat_line2window_workspace(*args)
        L.posfeat_line2window_backward_workspace(*args)
    for args in ((8, 480, 640), (1, 16, 16), (0, 16, 16)):
        L.posfeat_disk_loss_workspace(*args)
        L.posfeat_disk_loss_grad_workspace(*args)
    for args in ((8, 4800), (1, 1), (0, 0)):
        L.posfeat_disk_flash_lse_workspace(*args)
    for args in ((8192, 8192), (0, 5), (1, 1), (20480, 7000)):
        L.posfeat_match_workspace(*args)
    for args in ((8, 120, 160, 192, 192, 3, 3, 1), (2, 7, 9, 64, 64, 1, 1, 2), (1, 1, 1, 4, 8, 3, 3, 1)):
        L.posfeat_conv_wgrad_workspace(*args)
    for args in ((8, 120, 160, 512, 256), (1, 4, 4, 32, 32), (1, 3, 5, 32, 32)):
        L.posfeat_wino_wgrad_workspace(*args)
        L.posfeat_wino_workspace(*args)
    print("sizing/validation ok")

    # engine and trainer instance planning (host dry pass over every layer)
    blob = (ctypes.c_float * 16)()
    for (b, h, w) in ((1, 64, 96), (32, 480, 640), (2, 96, 208), (1, 16, 16), (3, 768, 1024)):
        m = c_void_p()
        r = L.posfeat_model_create(b, h, w, blob, ctypes.byref(m))
        check(r == 0 and m.value, "model_create %s" % ((b, h, w),))
        check(L.posfeat_model_workspace(m) > 0, "model workspace")
        L.posfeat_model_destroy(m)
        m = c_void_p()
        check(L.posfeat_model_create_train(b, h, w, blob, ctypes.byref(m)) == 0, "create_train")
        L.posfeat_model_destroy(m)
    for bad_shape in ((0, 64, 96), (1, 17, 96), (1, 64, 95), (-1, 64, 64)):
        m = c_void_p()
        check(L.posfeat_model_create(*bad_shape, blob, ctypes.byref(m)) != 0, "bad model shape")
    check(L.posfeat_model_create(1, 64, 96, None, None) != 0, "null out")
    for (b, h, w) in ((8, 480, 640), (2, 128, 160), (1, 64, 64)):
        t = c_void_p()
        check(L.posfeat_bbtrain_create(b, h, w, ctypes.byref(t)) == 0 and t.value, "bbtrain_create")
        check(L.posfeat_bbtrain_act_bytes(t) > 0 and L.posfeat_bbtrain_scratch_bytes(t) > 0,
              "bbtrain bytes")
        L.posfeat_bbtrain_destroy(t)
    t = c_void_p()
    check(L.posfeat_bbtrain_create(0, 64, 64, ctypes.byref(t)) != 0, "bbtrain bad batch")
    print("instance planning ok")
    print("ASAN HOST RUN CLEAN")


if __name__ == "__main__":
    main()
