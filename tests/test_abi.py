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


def test_struct_layout_matches_c_compiler(tmp_path):
    """Compile include/scd.h with the host C compiler and compare every descriptor offset with ctypes."""
    import shutil
    import subprocess
    from multimodal_siamese_cd_amd import hip
    cc = shutil.which('gcc') or shutil.which('cc')
    if cc is None:
        pytest.skip('no host C compiler')
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fields = {'scd_nhwc_t': (hip.NHWC, ['data', 'n', 'h', 'w', 'c', 'ldc', 'dtype']),
              'scd_igemm_t': (hip.IGEMM, [f[0] for f in hip.IGEMM._fields_]),
              'scd_wgrad_t': (hip.WGRAD, [f[0] for f in hip.WGRAD._fields_])}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "scd.h"', 'int main(void) {']
    for ctype, (_, names) in fields.items():
        lines.append(f'printf("{ctype} size %zu\\n", sizeof({ctype}));')
        for nm in names:
            lines.append(f'printf("{ctype} {nm} %zu\\n", offsetof({ctype}, {nm}));')
    lines += ['return 0;', '}']
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    subprocess.run([cc, '-I', os.path.join(root, 'include'), str(src), '-o', str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split('\n')
    got = {(a, b): int(c) for a, b, c in (ln.split() for ln in out if ln)}
    for ctype, (cls, names) in fields.items():
        assert got[(ctype, 'size')] == ctypes.sizeof(cls), ctype
        for nm in names:
            assert got[(ctype, nm)] == getattr(cls, nm).offset, (ctype, nm)


def test_product_path_refuses_cpu_tensors(lib):
    import torch
    from multimodal_siamese_cd_amd import engine
    x = torch.zeros(1, 5, 16, 16)
    with pytest.raises(RuntimeError, match='MI355X'):
        engine.pack_pair(x, x)
