"""Bit-identity rule for GEMM tile ids (include/pps_abi.h): every tile below
TILE_P16_FIRST (the register-staged kernels and the pipelined ones on
32x32x16 MFMA blocks) gives the same bits; the pipelined tiles on 16x16x32
blocks (ids >= TILE_P16_FIRST) sum each 32-wide K chunk in one MFMA, so they
agree bit for bit with each other (or, for shapes the pipelined kernel
cannot stage, fall back to the first group).  The patch-staged 3x3 tiles
(ids 56-59) run K in (channel chunk, tap) order: they agree with each other
where they apply and run tile 38 (the 16x16x32 group) elsewhere.
Accuracy is checked separately for every group."""
import numpy as np


def check_tile_bits(tiles, outs, p16_first, c16_first=56):
    """Tile 0 (the built-in choice) may pick from either group: it must equal
    one of them."""
    base, s16, auto, c16 = None, None, None, []
    for t, o in zip(tiles, outs):
        if t == 0:
            auto = o
        elif t >= c16_first:
            c16.append((t, o))
        elif t < p16_first:
            if base is None:
                base = o
            np.testing.assert_array_equal(o, base, err_msg='tile %d' % t)
        else:
            if s16 is None:
                s16 = o
            np.testing.assert_array_equal(o, s16, err_msg='tile %d' % t)
    patch = None
    for t, o in c16:
        if s16 is not None and np.array_equal(o, s16):
            continue  # shape outside the patch kernel: tile 38
        if patch is None:
            patch = o
        np.testing.assert_array_equal(o, patch, err_msg='tile %d' % t)
    if auto is not None:
        assert any(g is not None and np.array_equal(auto, g) for g in (base, s16)), \
            'tile 0 matches neither rounding group'
