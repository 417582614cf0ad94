"""The C-ABI library builds for gfx950, loads without a GPU, and exports every
entry point that include/pps_abi.h declares (no compute calls here)."""
import os
import re

from tests.conftest import ROOT


def _declared():
    with open(os.path.join(ROOT, 'include', 'pps_abi.h')) as f:
        src = f.read()
    return sorted(set(re.findall(r'^(?:int64_t|int|const char\*)\s+(pps_\w+)\s*\(', src, re.M)))


def test_header_declares_entry_points():
    names = _declared()
    assert 'pps_distmat' in names and 'pps_conv2d_bn_act' in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    from pps_amd import _lib
    L = _lib.lib()
    for name in _declared():
        assert hasattr(L, name), name
    assert set(_declared()) == set(_lib.exported_symbols())


def test_library_metadata_calls():
    from pps_amd import _lib
    L = _lib.lib()
    assert L.pps_abi_version() == 1
    ops = L.pps_registered_ops().decode().split(';')
    assert 'PairWiseDistance' in ops


def test_code_object_targets_gfx950():
    lib = os.path.join(ROOT, 'pps_amd', 'libpps_hip.so')
    with open(lib, 'rb') as f:
        blob = f.read()
    assert b'amdgcn-amd-amdhsa--gfx950' in blob


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    from pps_amd import _lib
    monkeypatch.setattr(_lib, '_LIB', None)
    monkeypatch.setattr(_lib, 'LIB_PATH', str(tmp_path / 'nope.so'))
    import pytest
    with pytest.raises(RuntimeError, match='no CPU fallback|There is no CPU fallback'):
        _lib.lib()


def test_pipelined_tile_shapes():
    """pps_x3p_tile_shape (host-only) mirrors the pipelined tile table
    (pps_internal.hpp): the ids the fused part pooling may use are exactly
    the 192-row tiles with <= 256 columns (192x256: f32 activations only)."""
    from pps_amd import ops
    want = {29: (128, 128), 30: (192, 128), 31: (128, 64), 32: (192, 64), 33: (256, 128),
            34: (128, 256), 35: (192, 256), 36: (128, 128), 37: (192, 128), 38: (128, 128),
            39: (192, 128), 40: (128, 64), 41: (192, 64), 42: (256, 128), 43: (128, 256),
            44: (128, 256), 45: (128, 128), 46: (192, 128), 47: (192, 128), 48: (192, 64),
            49: (96, 128), 50: (96, 128), 51: (128, 128), 52: (192, 128), 53: (96, 128),
            55: (64, 128)}
    assert ops.num_tiles() == 60
    for t, shape in want.items():
        assert ops.tile_shape(t) == shape, t
    assert ops.tile_shape(28) == (0, 0) and ops.tile_shape(54) == (0, 0)  # 54: gemm_ws
    # plane activations: only the 192x256 8-wave tile falls back (to 128 rows:
    # two stages of it would not fit the LDS); the 192-row 8-wave and 96-row
    # tiles take the planes natively (uneven DMA pieces per wave)
    assert ops.tile_shape(35, True) == (128, 256) and ops.tile_shape(37, True)[0] == 192
    assert ops.tile_shape(47, True)[0] == 192 and ops.tile_shape(49, True)[0] == 96
    assert ops.tile_shape(50, True) == (96, 128)
    pps_f32 = [t for t in want if ops.tile_shape(t)[0] == 192 and ops.tile_shape(t)[1] <= 256]
    pps_pl = [t for t in want if ops.tile_shape(t, True)[0] == 192 and
              ops.tile_shape(t, True)[1] <= 256]
    assert pps_f32 == [30, 32, 35, 37, 39, 41, 46, 47, 48, 52]
    assert pps_pl == [30, 32, 37, 39, 41, 46, 47, 48, 52]


def _defines():
    with open(os.path.join(ROOT, 'include', 'pps_abi.h')) as f:
        src = f.read()
    return {k: int(v, 0) for k, v in re.findall(r'^#define\s+(PPS_\w+)\s+(0x[0-9a-fA-F]+|\d+)\b',
                                                 src, re.M)}


def test_python_flag_constants_match_the_header():
    """The or-ed tile flags, the autotune flags and the slot size the Python
    side passes across the ABI are the header's values (a drift would run a
    different launch without an error)."""
    from pps_amd import native, ops
    d = _defines()
    pairs = {'PPS_TILE_B_TILED': ops.TILE_B_TILED, 'PPS_TILE_COL_ORDER': ops.TILE_COL_ORDER,
             'PPS_TILE_SEAM': ops.TILE_SEAM, 'PPS_TILE_H2': ops.TILE_H2,
             'PPS_TILE_H2P': ops.TILE_H2P, 'PPS_TILE_H2E': ops.TILE_H2E,
             'PPS_AMAX_SLOT_FLOATS': ops.AMAX_SLOT_FLOATS,
             'PPS_AUTOTUNE_NO_PLANES': native.AUTOTUNE_NO_PLANES,
             'PPS_AUTOTUNE_SPLITK': native.AUTOTUNE_SPLITK,
             'PPS_AUTOTUNE_NO_SEAM': native.AUTOTUNE_NO_SEAM,
             'PPS_AUTOTUNE_NO_H2': native.AUTOTUNE_NO_H2,
             'PPS_AUTOTUNE_NO_H2E': native.AUTOTUNE_NO_H2E,
             'PPS_AUTOTUNE_NO_GROUPS': native.AUTOTUNE_NO_GROUPS}
    for name, value in pairs.items():
        assert d[name] == value, (name, d.get(name), value)
    flags = [v for k, v in d.items() if k.startswith('PPS_TILE_') and k in pairs]
    assert ops.TILE_FLAGS == sum(flags)
