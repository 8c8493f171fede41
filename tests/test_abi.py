"""The C-ABI boundary (CPU only: no compute calls).

* libpafb2p.so loads and exports every function include/b2p.h declares;
* the ctypes prototypes in paf_b2p/_lib.py cover exactly that set;
* the struct layouts agree with the header (sizes / offsets via a tiny C
  probe compiled with gcc against include/b2p.h);
* the device-free helpers (geometry checks, sizes, error strings) behave.
"""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import REPO

import paf_b2p
from paf_b2p import _lib as L

HDR = os.path.join(REPO, "include", "b2p.h")


def declared_functions(path):
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(b2p_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(L.LIB_PATH)
    names = declared_functions(HDR)
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_prototypes_match_header():
    assert sorted(L.PROTOTYPES) == declared_functions(HDR)


def test_nm_shows_plain_c_symbols():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (b2p_\w+)", out))
    assert set(declared_functions(HDR)) <= exported  # extern "C": unmangled


def test_struct_layout_matches_header(tmp_path):
    probe = tmp_path / "probe.c"
    probe.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "b2p.h"
int main(void) {
  printf("%zu %zu %zu %zu %zu %zu\n", sizeof(b2p_geom_t), offsetof(b2p_geom_t, nsamp_int),
         offsetof(b2p_geom_t, mean), sizeof(b2p_info_t), sizeof(b2p_stats_t),
         offsetof(b2p_stats_t, kernel_ms));
  return 0;
}''')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(probe), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(L.Geom), L.Geom.nsamp_int.offset, L.Geom.mean.offset, C.sizeof(L.Info),
            C.sizeof(L.Stats), L.Stats.kernel_ms.offset]
    assert got == want


def test_bmf_defaults_and_sizes():
    g = L.Geom()
    assert L.lib().b2p_geom_bmf(C.byref(g)) == 0
    assert (g.nbit, g.big_endian, g.nchunk, g.nsamp_df, g.nchan_chunk) == (16, 1, 48, 128, 7)
    assert g.nsamp_int == 1 << 20
    assert L.lib().b2p_frame_bytes(C.byref(g)) == 48 * 7168
    assert L.lib().b2p_block_bytes(C.byref(g)) == 2818572288
    assert L.lib().b2p_geom_check(C.byref(g)) == 0


@pytest.mark.parametrize("bad", [
    dict(nbit=4), dict(nbit=8, big_endian=1), dict(npol=1), dict(ndim=1), dict(npol_out=3),
    dict(nchunk=0), dict(nsamp_int=3, nsamp_df=2), dict(nchan_chunk=3),  # 12-B chunk
    dict(nchan_chunk=8193), dict(nchan_chunk=4096, npol_out=2, nchunk=3),
])
def test_geometry_rejected(bad):
    g = paf_b2p.make_geom(**{**dict(nchan_chunk=256), **bad})
    assert L.lib().b2p_geom_check(C.byref(g)) == L.B2P_EINVAL


def test_geometry_accepted():
    for g in (paf_b2p.generic_geom(256), paf_b2p.generic_geom(1024), paf_b2p.bmf_geom(),
              paf_b2p.generic_geom(336, nbit=16), paf_b2p.generic_geom(3),
              paf_b2p.bmf_geom(npol_out=2, mean=1)):
        assert L.lib().b2p_geom_check(C.byref(g)) == 0, g.as_dict()


def test_strerror_covers_codes():
    for code in range(0, -10, -1):
        s = L.lib().b2p_strerror(code).decode()
        assert s and s != "unknown error"
    assert L.lib().b2p_strerror(-99).decode() == "unknown error"


def test_open_without_gpu_fails_cleanly(have_gpu):
    if have_gpu:
        pytest.skip("a GPU is visible")
    with pytest.raises(paf_b2p.B2PError) as e:
        paf_b2p.Integrator(paf_b2p.generic_geom(256), device=0)
    assert e.value.code == L.B2P_ENODEV
    with pytest.raises(paf_b2p.B2PError):
        paf_b2p.Integrator(paf_b2p.generic_geom(256), device=-1)


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    # no CPU fallback: without libpafb2p.so every entry point raises
    monkeypatch.setattr(L, "_lib", None)
    monkeypatch.setattr(L, "LIB_PATH", str(tmp_path / "absent" / "libpafb2p.so"))
    with pytest.raises(ImportError, match="no CPU fallback"):
        paf_b2p.Integrator(paf_b2p.bmf_geom())
    with pytest.raises(ImportError):
        L.lib()
