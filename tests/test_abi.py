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
  printf("%zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(b2p_geom_t), offsetof(b2p_geom_t, nsamp_int),
         offsetof(b2p_geom_t, mean), sizeof(b2p_info_t), sizeof(b2p_stats_t),
         offsetof(b2p_stats_t, kernel_ms), sizeof(b2p_tuning_t), offsetof(b2p_tuning_t, assemble_grid));
  return 0;
}''')
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), str(probe), "-o", str(exe)],
                   check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(L.Geom), L.Geom.nsamp_int.offset, L.Geom.mean.offset, C.sizeof(L.Info),
            C.sizeof(L.Stats), L.Stats.kernel_ms.offset, C.sizeof(L.Tuning),
            L.Tuning.assemble_grid.offset]
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


def test_blocks_per_launch_rule():
    """queued blocks per b2p_integrate_n launch: a launch reads >= 4 GiB,
    1..8 blocks; the Python mirror (bench.py's default) is the same rule"""
    sizes = [0, 1, 1 << 24, 1 << 28, 512 << 20, 1 << 30, (1 << 30) + 1, 2 << 30, 2818572288, 4 << 30, 1 << 40]
    got = [L.lib().b2p_blocks_per_launch(n) for n in sizes]
    assert got == [1, 8, 8, 8, 8, 4, 3, 2, 1, 1, 1]
    assert got == [paf_b2p.blocks_per_launch(n) for n in sizes]


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


def test_release_library_has_no_test_hook():
    """The shipped libpafb2p.so carries no fault-injection entry and reads no
    environment knobs (launch variants go through b2p_open_tuned); the test
    build (lib/hooks/, -DB2P_TEST_HOOKS) is the only one with the hook."""
    lib = C.CDLL(L.LIB_PATH)
    assert not hasattr(lib, "b2p_test_inject_push_fail")
    blob = open(L.LIB_PATH, "rb").read()
    for word in (b"B2P_INJECT", b"B2P_ASM_VARIANT", b"B2P_UNROLL", b"B2P_FUSE", b"B2P_STAGE"):
        assert word not in blob, word
    und = subprocess.run(["nm", "-D", "--undefined-only", L.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert not re.search(r"\bgetenv\b", und)
    assert not hasattr(lib, "b2p_debug_build") and not hasattr(lib, "b2p_test_debug_shrink_bound")
    hooks = os.path.join(os.path.dirname(L.LIB_PATH), "hooks", "libpafb2p.so")
    assert hasattr(C.CDLL(hooks), "b2p_test_inject_push_fail")
    debug = C.CDLL(os.path.join(os.path.dirname(L.LIB_PATH), "debug", "libpafb2p.so"))
    for name in ("b2p_debug_build", "b2p_test_debug_shrink_bound", "b2p_test_inject_push_fail"):
        assert hasattr(debug, name), name
    assert debug.b2p_debug_build() == 1


def test_tuning_defaults_and_refusals():
    """b2p_tuning_init marks every field "default"; out-of-range values are
    refused with B2P_EINVAL before any device is touched (no clamping)"""
    t = L.Tuning.make()
    assert t.size == C.sizeof(L.Tuning)
    assert (t.nontemporal, t.interleave, t.fuse) == (-1, -1, -1)
    assert (t.max_threads, t.unroll, t.replicas, t.stage_mib) == (0, 0, 0, 0)
    g = L.Geom()
    L.lib().b2p_geom_bmf(C.byref(g))
    for bad in ({"unroll": 5}, {"max_threads": 32}, {"threads": 100}, {"wg_per_cu": 33},
                {"replicas": 2000}, {"nontemporal": 2}, {"fuse": -2}, {"stage_mib": 20000},
                {"row_groups": -1}):
        ctx = C.c_void_p()
        tt = L.Tuning.make(**bad)
        assert L.lib().b2p_open_tuned(C.byref(ctx), C.byref(g), 0, C.byref(tt)) == L.B2P_EINVAL, bad
        assert b"tuning" in L.lib().b2p_last_error(None)
    tt = L.Tuning.make()
    tt.size = 4
    ctx = C.c_void_p()
    assert L.lib().b2p_open_tuned(C.byref(ctx), C.byref(g), 0, C.byref(tt)) == L.B2P_EINVAL
    with pytest.raises(KeyError):
        L.Tuning.make(bogus=1)


def test_group_refuses_bad_timeout_and_pci_args():
    grp = C.c_void_p()
    arr = (C.c_void_p * 1)(None)
    assert L.lib().b2p_group_open_timed(C.byref(grp), arr, 1, 0, 0) == L.B2P_EINVAL
    assert L.lib().b2p_device_pci_bus_id(0, None, 32) == L.B2P_EINVAL
    assert L.lib().b2p_strerror(L.B2P_ETIMEDOUT).decode().startswith("collective did not complete")
