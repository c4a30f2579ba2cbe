"""The C-ABI boundary: libmep_hip.so loads, exports every entry point include/mep.h declares,
and the ctypes mirrors of the descriptor structs match the C layout (gcc probe).  CPU only: no
compute call is made."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

import mep_amd  # noqa: F401  (registered by conftest)
from mep_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'mep.h')


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\bint\s+(mep_[a-z0-9_]+)\s*\(', src)))


def test_library_loads_and_version():
    L = _lib.lib()
    assert L.mep_abi_version() == _lib.ABI_VERSION == 7


def test_every_declared_symbol_is_exported():
    L = _lib.lib()
    names = declared_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.SIGNATURES, 'no ctypes signature for %s' % n


def test_last_error_roundtrip():
    assert isinstance(_lib.last_error(), str)
    # an invalid head descriptor is rejected on the host, before any launch
    d = _lib.HeadDesc(NC=99, B=4)
    rc = _lib.lib().mep_head_fwd_bwd(ctypes.byref(d), None)
    assert rc == -1000
    assert 'invalid descriptor' in _lib.last_error()


def test_head_partial_stride():
    NC = 7
    assert _lib.lib().mep_head_partial_stride(NC) == 2 * NC * NC + NC ** 3 + 5 * NC


@pytest.mark.skipif(subprocess.call(['which', 'gcc'], stdout=subprocess.DEVNULL) != 0, reason='no gcc')
def test_struct_layout_matches_c():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mep.h"', 'int main(void){']
    for cname, st in _lib.STRUCTS.items():
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for fname, _ in st._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, fname, cname, fname))
    lines.append('return 0;}')
    with tempfile.TemporaryDirectory() as td:
        c = os.path.join(td, 'probe.c')
        exe = os.path.join(td, 'probe')
        open(c, 'w').write('\n'.join(lines))
        subprocess.check_call(['gcc', '-I', os.path.dirname(HEADER), c, '-o', exe])
        out = subprocess.check_output([exe]).decode().split('\n')
    got = dict(line.split() for line in out if line.strip())
    for cname, st in _lib.STRUCTS.items():
        assert int(got[cname]) == ctypes.sizeof(st), cname
        for fname, _ in st._fields_:
            assert int(got[cname + '.' + fname]) == getattr(st, fname).offset, (cname, fname)
