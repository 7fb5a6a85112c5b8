"""Every legal conv tile (POSFEAT_CONV_TILE, one child process each) on the
stem, 1x1, strided 1x1, 3x3 s1 / s2 and a B=32 layer1-scale 1x1: three
repeated launches must be BIT-equal and within 1e-5 of Sum|x||w| of the fp64
conv (tools/tile_sweep.py).  This is the regression test of the stale-operand
race of round 2 (an inline-asm v_cvt_pk_bf16_f32 whose VGPR write the
compiler's hazard recognizer could not see, so MFMAs read the register's old
value when scheduled right behind it: conv_glds_kernel<128,64,..,BF6> and the
bf16x6 stem variant); tools/isa_check.py checks the ISA for
the hazard itself."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_every_tile_repeatable_and_accurate():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "tile_sweep.py")],
                       capture_output=True, text=True, timeout=900)
    print(r.stdout[-6000:])
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
