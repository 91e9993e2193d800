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


def build_lib(force: bool = False, verbose: bool = True, jobs: int | None = None, out: str | None = None,
              defines: tuple = ()) -> str:
    """One object per translation unit, compiled in parallel (the units share no device code), then linked.
    `out` / `defines` (e.g. ('SCD_WGRAD_ROW_WALK=1',)): an A/B variant library elsewhere (SCD_LIB selects it)."""
    OUT_ = out or OUT
    if out is None and not force and up_to_date():
        return OUT
    os.makedirs(os.path.dirname(OUT_), exist_ok=True)
    objdir = os.path.join(os.path.dirname(OUT_), 'obj')
    os.makedirs(objdir, exist_ok=True)
    cflags = [f for f in FLAGS if f != '-shared'] + [f'-D{d}' for d in defines]
    procs, objs = [], []
    jobs = jobs or min(8, os.cpu_count() or 1)
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src) + '.o')
        objs.append(obj)
        cmd = [HIPCC, *cflags, '-c', '-o', obj, src]
        if verbose:
            print(' '.join(cmd), flush=True)
        procs.append(subprocess.Popen(cmd))
        while sum(p.poll() is None for p in procs) >= jobs:
            procs[[p.poll() is None for p in procs].index(True)].wait()
    if any(p.wait() != 0 for p in procs):
        raise RuntimeError('hipcc failed (see the compiler output above)')
    tmp = OUT_ + '.tmp'
    subprocess.run([HIPCC, *FLAGS, '-o', tmp, *objs], check=True)
    os.replace(tmp, OUT_)
    return OUT_


if __name__ == '__main__':
    import sys
    if len(sys.argv) > 1:  # python -m multimodal_siamese_cd_amd.build <out.so> [DEFINE=VALUE ...]
        build_lib(out=os.path.abspath(sys.argv[1]), defines=tuple(sys.argv[2:]))
    else:
        build_lib(force=True)
