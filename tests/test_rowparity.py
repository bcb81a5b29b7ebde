"""The per-row parity bar itself (tests/rowparity.py), on small hand-made BSR values."""
import numpy as np
import pytest

from rowparity import assert_rows_close, row_errors


def test_row_scale_is_per_row():
    # two block rows of 2x2 blocks; row 1 is 1e6 smaller than row 0
    indptr = np.array([0, 2, 3])
    ref = np.zeros((3, 2, 2))
    ref[0] = [[1e8, 2e7], [3e7, 1e8]]
    ref[1] = [[-5e7, 0.0], [0.0, -5e7]]
    ref[2] = [[100.0, 1.0], [1.0, 100.0]]
    got = ref.copy()
    got[2, 0, 0] += 1e-8  # 1e-10 of its own row: fails per row, passes against the global max
    rel, r = row_errors(got, ref, indptr)
    assert r == 1 and rel == pytest.approx(1e-10)
    assert np.abs(got - ref).max() <= 1e-12 * np.abs(ref).max()  # the old global bar would pass
    with pytest.raises(AssertionError):
        assert_rows_close(got, ref, indptr)
    got[2, 0, 0] = ref[2, 0, 0] * (1 + 1e-14)
    assert_rows_close(got, ref, indptr)


def test_zero_rows_must_be_exact():
    indptr = np.array([0, 1])
    ref = np.zeros((1, 2, 2))
    got = ref.copy()
    assert row_errors(got, ref, indptr)[0] == 0.0
    got[0, 1, 1] = 1e-300
    assert row_errors(got, ref, indptr)[0] == float("inf")
