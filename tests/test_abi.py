"""CPU: libsad.so builds for gfx950, loads, and exports exactly the C ABI that
include/sad.h declares (no compute calls: there is no GPU here)."""
import os
import re
import subprocess

import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, 'include', 'sad.h')


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(sad_[a-z0-9_]+)\s*\(', src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for must in ('sad_frontend_run', 'sad_backbone_run', 'sad_heads_merge_run', 'sad_last_error', 'sad_conv2d_run'):
        assert must in syms


def test_library_exports_every_declared_symbol():
    from sad import _lib
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), f'{s} missing from libsad.so'
    out = subprocess.run(['nm', '-D', '--defined-only', _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r'\bT (sad_[a-z0-9_]+)', out))
    assert set(declared_symbols()) <= exported
    # ctypes prototypes cover the whole ABI
    assert set(_lib.SIGNATURES) == set(declared_symbols())


def test_library_is_gfx950_code_object():
    from sad import _lib
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objdump', '--offloading', _lib.LIB_PATH],
                         capture_output=True, text=True)
    txt = out.stdout + out.stderr
    if 'gfx' not in txt:  # older objdump: look for the target id string in the bundle
        txt = open(_lib.LIB_PATH, 'rb').read().decode('latin1')
    assert 'gfx950' in txt


def test_version_and_error_strings():
    from sad import _lib
    lib = _lib.load()
    assert b'gfx950' in lib.sad_version()
    assert isinstance(lib.sad_last_error(), bytes)


def test_argument_errors_are_reported_without_gpu():
    """Bad arguments are rejected before any device work, with a message."""
    from sad import _lib
    lib = _lib.load()
    rc = lib.sad_frontend_plan_create(None, None)
    assert rc == -1 and b'null' in lib.sad_last_error()
    with pytest.raises(RuntimeError, match='libsad'):
        _lib.check(rc, 'sad_frontend_plan_create')


def test_product_refuses_cpu_device():
    from sad.engine import FrontEnd
    with pytest.raises(RuntimeError, match='no CPU path'):
        FrontEnd('cpu')
