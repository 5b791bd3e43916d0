"""LDS bank-conflict model (tools/lds_bank_model.py) of the swizzles the kernels use:
the fragment reads / writes of the forward and transposed-read images and the XF 5
(tconv on load) u stores are conflict-free; the model reproduces the 4-way conflict of
the round-4 8-byte u stores it replaced (35 % conflict cycles on the r5 PMC pass)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import lds_bank_model as m  # noqa: E402


def test_fwd_and_transposed_images_conflict_free():
    assert m.check_fwd() == 1
    for bm in (32, 64, 128, 256):
        assert m.check_tr(bm) == (1, 1)


def test_tconv_onload_u_stores():
    old, one_phase, interleaved = m.check_ut_store()
    assert old == 4 and one_phase == 2 and interleaved == 1


def test_epilogue_staging_half_swap():
    assert m.check_epi() == (1, 1)
    assert m.check_epi(half_swap=False) == (2, 1)


def test_generic_wgrad_row_pair_swap():
    for w in (64, 128, 256):
        assert m.check_wgrad_store(w) == 1
        assert m.check_wgrad_store(w, swap=False) == 2


def test_tconv_fwd_staging():
    for w in (8, 16, 32, 64):
        assert m.check_tconv_epi(w) == (1, 1)
    assert m.check_tconv_epi(32, padded=True) == (1, 2)
