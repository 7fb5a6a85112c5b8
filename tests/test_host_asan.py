"""Host-side AddressSanitizer run of the C ABI (SURVEY.md §5 "race detection /
sanitizers"; the reference has none).  `make -C posfeat_amd/csrc asan` builds
every source with -fsanitize=address on the HOST side only (-Xarch_host: GPU
sanitizers are not available on this pool) into
build/asan/libposfeat_hip_asan.so; tools/asan_host.py then drives argument
validation, conv planning / workspace sizing over the model's layer shapes and
ragged ones, the layer tables, and the engine's / trainers' instance planning
(a dry pass over every layer) in a child process under the clang ASan
runtime.  Any heap / stack overflow, use-after-free or arithmetic trap aborts
the child.  (It found posfeat_wino_wgrad_workspace dividing by zero for
Cin < 128, fixed in wino.hip.)  CPU only: no kernel is launched."""
import glob
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _asan_runtime():
    c = sorted(glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so"))
    return c[-1] if c else None


def test_host_abi_under_asan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("clang ASan runtime not found")
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(["make", "-s", "-j", jobs, "-C", os.path.join(ROOT, "posfeat_amd", "csrc"),
                    "asan"], check=True, timeout=900)
    lib = os.path.join(ROOT, "build", "asan", "libposfeat_hip_asan.so")
    env = dict(os.environ, LD_PRELOAD=rt, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "asan_host.py"), lib],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ASAN HOST RUN CLEAN" in r.stdout, (r.stdout[-2000:] +
                                                                      r.stderr[-4000:])
