"""Bit-identity rule for GEMM tile ids (include/pps_abi.h): every tile below
TILE_P16_FIRST (the register-staged kernels and the pipelined ones on
32x32x16 MFMA blocks) gives the same bits; the pipelined tiles on 16x16x32
blocks (ids >= TILE_P16_FIRST) sum each 32-wide K chunk in one MFMA, so they
agree bit for bit with each other (or, for shapes the pipelined kernel
cannot stage, fall back to the first group).  Accuracy is checked
separately for both groups."""
import numpy as np


def check_tile_bits(tiles, outs, p16_first):
    """Tile 0 (the built-in choice) may pick from either group: it must equal
    one of them."""
    base, s16, auto = None, None, None
    for t, o in zip(tiles, outs):
        if t == 0:
            auto = o
        elif t < p16_first:
            if base is None:
                base = o
            np.testing.assert_array_equal(o, base, err_msg='tile %d' % t)
        else:
            if s16 is None:
                s16 = o
            np.testing.assert_array_equal(o, s16, err_msg='tile %d' % t)
    if auto is not None:
        assert any(g is not None and np.array_equal(auto, g) for g in (base, s16)), \
            'tile 0 matches neither rounding group'
