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
