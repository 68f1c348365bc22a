"""codec.packed_positions (CPU): where the packed layout (include/hhuff.h, hhuff_*_batch_packed) puts each string
when the host packed path does not return out_off -- tile t = i // 64 starts at its slot position, its kept strings
follow back to back, failed strings (HHUFF_FAIL_LEN) take no bytes."""
import numpy as np
import pytest

from h2o_amd import codec


def _loop(in_off, out_len, decode):
    pos = np.zeros(len(out_len), np.int64)
    for i, L in enumerate(out_len):
        if i % 64 == 0:
            cur = int(in_off[i]) * 8 // 5 if decode else int(in_off[i])
        pos[i] = cur
        if L != codec.FAIL_LEN:
            cur += int(L)
    return pos


@pytest.mark.parametrize("n", [1, 63, 64, 65, 200, 1000])
@pytest.mark.parametrize("decode", [False, True])
def test_packed_positions_match_the_tile_rule(n, decode):
    rng = np.random.default_rng(n + decode)
    lens = rng.integers(0, 90, n)
    in_off = np.zeros(n + 1, np.uint32)
    in_off[1:] = np.cumsum(lens)
    out_len = np.where(rng.random(n) < 0.1, codec.FAIL_LEN,
                       (lens * (8 if decode else 3) // (5 if decode else 4))).astype(np.uint32)
    np.testing.assert_array_equal(codec.packed_positions(in_off, out_len, decode), _loop(in_off, out_len, decode))
