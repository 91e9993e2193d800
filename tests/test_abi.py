"""CPU-side checks of the C-ABI boundary: the library loads and exports every symbol include/scd.h declares."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'scd.h')


def declared_symbols():
    text = open(HEADER).read()
    return sorted(set(re.findall(r'^\s*(?:const\s+)?\w+\s*\*?\s*(scd_\w+)\s*\(', text, flags=re.M)))


@pytest.fixture(scope='module')
def lib():
    from multimodal_siamese_cd_amd import build, hip
    build.build_lib()
    return hip.load_library()


def test_header_declares_core_entry_points():
    syms = declared_symbols()
    for s in ('scd_conv_igemm', 'scd_conv_wgrad', 'scd_bn_train_stats', 'scd_bn_relu_backward', 'scd_maxpool2_fwd',
              'scd_pjaccard_fwd', 'scd_pjaccard_bwd', 'scd_last_error', 'scd_device_check'):
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_python_binding_covers_header(lib):
    from multimodal_siamese_cd_amd import hip
    assert sorted(hip.EXPORTED_SYMBOLS) == declared_symbols()


def test_version_and_error_without_gpu(lib):
    from multimodal_siamese_cd_amd import hip
    assert 'gfx950' in hip.version()
    # argument validation runs on the host and reports through scd_last_error (no GPU touched)
    rc = lib.scd_pack_conv3x3(None, 0, 0, 0, 0, None, None)
    assert rc == -1
    assert b'pack_conv3x3' in lib.scd_last_error()


def test_struct_layout_matches_header(lib):
    from multimodal_siamese_cd_amd import hip
    # offsets as a C compiler lays them out (x86-64 SysV): pointers 8-aligned
    assert ctypes.sizeof(hip.NHWC) == 32
    assert hip.IGEMM.wpk.offset == 72 and hip.IGEMM.dst.offset == 96
    assert hip.WGRAD.src.offset == 32 and hip.WGRAD.dx.offset == 81


def test_product_path_refuses_cpu_tensors(lib):
    import torch
    from multimodal_siamese_cd_amd import engine
    x = torch.zeros(1, 5, 16, 16)
    with pytest.raises(RuntimeError, match='MI355X'):
        engine.pack_pair(x, x)
