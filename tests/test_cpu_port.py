"""The tuned CPU port (oracle/b2p_cpu_port.c) -- bench.py's cpu_baseline --
equals the oracle bit for bit on every ISA this CPU offers, over the bench
layouts, the committed golden fixtures, extreme values and random layouts.
The port is a baseline, never the checker: these tests pin it TO the oracle."""
import numpy as np
import pytest
from hypothesis import given, settings, strategies as st

import b2p_oracle as npo
import oracle_c as co
from conftest import golden_geom, load_golden

SEED = 20181105
ISAS = [i for i in ("scalar", "avx2", "avx512bw", "avx512vnni") if co.port_isa(i) == i]


def same(g, buf, isa, nthreads=1):
    a = co.integrate(g, buf, nthreads=2)
    b = co.port_integrate(g, buf, nthreads=nthreads, isa=isa)
    return np.array_equal(a, b)


def test_isa_dispatch_names():
    assert co.port_isa("scalar") == "scalar"
    assert co.port_isa("auto") in ("scalar", "avx2", "avx512bw", "avx512vnni")
    assert "scalar" in ISAS


@pytest.mark.parametrize("isa", ISAS)
@pytest.mark.parametrize("layout", [
    dict(nbit=8, nchan_chunk=256),                                   # configs[1]
    dict(nbit=8, nchan_chunk=1024),                                  # configs[2..4]
    dict(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7),   # BMF
    dict(nbit=16, nchan_chunk=48),                                   # int16 LE
    dict(nbit=8, nchunk=3, nsamp_df=16, nchan_chunk=12),             # TFTFP int8
    dict(nbit=16, big_endian=1, nchunk=8, nsamp_df=128, nchan_chunk=8),
])
@pytest.mark.parametrize("npol_out", [1, 2])
def test_port_equals_oracle(isa, layout, npol_out):
    g = npo.Geom(**layout, npol_out=npol_out)
    nframes = max(2, (3 << 20) // g.frame_bytes)
    g = npo.Geom(**{**g.asdict(), "nsamp_int": nframes * g.nsamp_df})
    buf = co.fill_synthetic(g, g.block_bytes, SEED, 3, 1)
    assert same(g, buf, isa, nthreads=3)


@pytest.mark.parametrize("isa", ISAS)
@pytest.mark.parametrize("name", ["bmf_small", "int8_256", "int16le_48"])
def test_port_on_golden_fixtures(isa, name):
    d = load_golden(name)
    g = golden_geom(d, npol_out=1, mean=0)
    assert np.array_equal(co.finalize(g, co.port_integrate(g, d["input"], isa=isa)).view(np.uint32),
                          d["power_p1_m0"].view(np.uint32))


@pytest.mark.parametrize("isa", ISAS)
def test_port_extremes_cross_the_int32_flush(isa):
    """every int8 component -128 for 40 000 rows (past the 32 768-add
    flush of the 32-bit lanes), every int16 component -32768 (each pmaddwd
    lane exactly 2^31)"""
    g8 = npo.Geom(nbit=8, nchan_chunk=64, nsamp_int=40000)
    b8 = np.full(g8.block_bytes, 0x80, dtype=np.uint8)
    assert same(g8, b8, isa, nthreads=1)
    assert int(co.port_integrate(g8, b8, isa=isa)[0]) == 40000 * 4 * 128 * 128
    g16 = npo.Geom(nbit=16, big_endian=1, nchunk=2, nsamp_df=16, nchan_chunk=8, nsamp_int=4096)
    b16 = np.tile(np.array([0x80, 0x00], np.uint8), g16.block_bytes // 2)
    assert same(g16, b16, isa)
    assert int(co.port_integrate(g16, b16, isa=isa)[0]) == 4096 * 4 * 2 ** 30


@settings(max_examples=40, deadline=None)
@given(nbit=st.sampled_from([8, 16]), be=st.booleans(), nchunk=st.integers(1, 6),
       nsamp_df=st.integers(1, 40), nchan_chunk=st.integers(1, 40), npol_out=st.sampled_from([1, 2]),
       nframes=st.integers(1, 9), threads=st.integers(1, 4))
def test_port_random_layouts(nbit, be, nchunk, nsamp_df, nchan_chunk, npol_out, nframes, threads):
    g = npo.Geom(nbit=nbit, big_endian=int(be and nbit == 16), nchunk=nchunk, nsamp_df=nsamp_df,
                 nchan_chunk=nchan_chunk, npol_out=npol_out, nsamp_int=nframes * nsamp_df)
    buf = co.fill_synthetic(g, g.block_bytes, SEED, nchunk, nframes)
    for isa in ISAS:
        assert same(g, buf, isa, nthreads=threads), isa


def test_port_rejects_ragged():
    g = npo.Geom(nbit=8, nchan_chunk=256, nsamp_int=16)
    with pytest.raises(ValueError):
        co.port_integrate(g, np.zeros(g.frame_bytes + 4, np.uint8))


def test_cpu_leg_deals_threads_over_every_l3(monkeypatch):
    """bench.py's CPU leg (oracle/cpu_baseline.pick_cpus): one core per L3
    domain before any domain gets a second, idlest core of each first, CPUs
    listed in order so the first threads sit on node 0 (a host of 2 nodes x
    4 CCDs x 4 cores, SMT siblings at +32, stands in for the 9575F)"""
    import cpu_baseline as cb
    l3 = {c: str((c % 32) // 4) for c in range(64)}          # CCD of each logical CPU
    node = {0: set(range(0, 16)) | set(range(32, 48)), 1: set(range(16, 32)) | set(range(48, 64))}
    busy = {c: (0.9 if c in (0, 4) else 0.0) for c in range(64)}  # the first core of CCDs 0, 1 busy
    monkeypatch.setattr(cb, "allowed_cpus", lambda: list(range(64)))
    monkeypatch.setattr(cb, "busy_fraction", lambda cpus, s=0.25: {c: busy[c] for c in cpus})
    monkeypatch.setattr(cb, "l3_domain", lambda c: l3[c])
    monkeypatch.setattr(cb, "numa_nodes", lambda: node)
    topo = {}
    for c in range(64):
        topo[f"/sys/devices/system/cpu/cpu{c}/topology/physical_package_id"] = "0" if c % 32 < 16 else "1"
        topo[f"/sys/devices/system/cpu/cpu{c}/topology/core_id"] = str(c % 32)
    monkeypatch.setattr(cb, "_read", lambda p: topo.get(p))
    p = cb.pick_cpus(8, 0.0)
    assert p["cpus"] == [1, 5, 8, 12, 16, 20, 24, 28]        # one per CCD, busy cores skipped
    assert p["l3_domains"] == 8 and p["l3_domains_allowed"] == 8 and p["nodes"] == [0, 1]
    p = cb.pick_cpus(12, 0.0)
    assert len(p["cpus"]) == 12 and len(set(p["cpus"])) == 12 and all(c < 32 for c in p["cpus"])
    per = {}
    for c in p["cpus"]:
        per[l3[c]] = per.get(l3[c], 0) + 1
    assert sorted(per.values()) == [1, 1, 1, 1, 2, 2, 2, 2]   # dealt: no CCD gets a third first
    p = cb.pick_cpus(40, 0.0)                                 # more threads than cores: SMT siblings
    assert len(set(p["cpus"])) == 40


def test_cpu_leg_reports_other_tenants_load():
    """others_busy: the mean load of the CPUs a leg did not run on"""
    import cpu_baseline as cb
    a = {0: (0, 0), 1: (0, 0), 2: (0, 0)}
    b = {0: (0, 100), 1: (50, 100), 2: (100, 100)}            # (idle ticks, total ticks)
    assert cb.others_busy(a, b, {0}) == 0.25                  # cpu 1 half busy, cpu 2 idle
    assert cb.others_busy(a, b, {0, 1, 2}) is None
