"""The bit-sliced `-k <k>ids` start pass (pm_ids.hip) is generated and
compiled for gfx950 on the host (hipRTC, no GPU needed)."""
import pytest

from patmatchdocker_amd import _lib, engine
from patmatchdocker_amd.convert import convert
from patmatchdocker_amd.regex import compile_pattern


@pytest.mark.parametrize("pat,k,types", [("TGCTGASTCAGCANW", 2, "ids"), ("TGCTGASTCAGCANW", 1, "s"),
                                         ("GAATTC", 3, "id"), ("TATAWAWR", 2, "i"), ("ACGTNNNNACGT", 3, "d")])
def test_ids_kernel_compiles(pat, k, types):
    prog = compile_pattern(convert("-n", pat), ignore_case=True)
    assert engine.ids_jit_compile(prog, k, types) > 1000


def test_ids_kernel_shape_bound():
    prog = compile_pattern("A" * 40, ignore_case=True)
    with pytest.raises(_lib.UnsupportedOnGPU):
        engine.ids_jit_compile(prog, 3, "ids")   # 160 state registers
