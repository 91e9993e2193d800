"""Build libscd.so in-tree with hipcc for gfx950 (no JIT cache: the .so travels with the repo snapshot)."""
from __future__ import annotations

import glob
import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, 'csrc')
OUT = os.path.join(PKG, '_lib', 'libscd.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
FLAGS = ['-O3', '-std=c++17', '--offload-arch=gfx950', '-fPIC', '-shared', '-Wall']


def sources():
    return sorted(glob.glob(os.path.join(CSRC, '*.hip')))


def deps():
    return sources() + sorted(glob.glob(os.path.join(CSRC, '*.h'))) + [
        os.path.join(os.path.dirname(PKG), 'include', 'scd.h')]


def up_to_date() -> bool:
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(d) <= t for d in deps())


def build_lib(force: bool = False, verbose: bool = True) -> str:
    if not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    tmp = OUT + '.tmp'
    cmd = [HIPCC, *FLAGS, '-o', tmp, *sources()]
    if verbose:
        print(' '.join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)
    return OUT


if __name__ == '__main__':
    build_lib(force=True)
