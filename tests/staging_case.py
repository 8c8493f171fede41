"""Host-span staging cases (test infrastructure).

``run_case`` is the body of the host-staging property test: one integration
of a small layout pushed from host memory (registered or pageable) through
two small staging buffers, cut into random pushes, compared with the oracle
bit for bit.  It is shared by

  * tests/test_gpu_random_layouts.py::test_host_spans_through_small_staging
    (release library, in the pytest process), and
  * tests/debug_build_checks.py (the debug library, lib/debug/, in a child
    process: every span load and every staging chunk checked).

Run as a script it is one case in its own process:

  python3 tests/staging_case.py NBIT BE NCHUNK NCC NSAMP_DF NFRAMES STAGE_MIB REGISTER CUTS SEED

CUTS: comma-separated frame indexes (or "-").  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "paf-baseband2power_amd"), os.path.join(REPO, "oracle")]

LAYOUTS = [(8, 0, 1, 1024), (16, 0, 1, 512), (16, 1, 48, 7), (8, 0, 3, 100)]


def case_geom(layout, mib):
    """the Geom of one case: layout (nbit, big_endian, nchunk, nchan_chunk)
    with the smallest whole-vector chunk (BMF: 128 samples), mib MiB long"""
    import b2p_oracle as npo
    nbit, be, nchunk, ncc = layout
    word = 4 * nbit // 8
    nsamp_df = 1
    while (nsamp_df * ncc * word) % 16:
        nsamp_df *= 2
    if (nbit, be, nchunk, ncc) == (16, 1, 48, 7):
        nsamp_df = 128
    frame = nchunk * nsamp_df * ncc * word
    nframes = max(1, (mib << 20) // frame)
    return npo.Geom(nbit=nbit, big_endian=be, nchunk=nchunk, nsamp_df=nsamp_df, nchan_chunk=ncc,
                    nsamp_int=nframes * nsamp_df)


def run_case(layout, stage_mib, mib, cut_fracs, register, seed):
    """one host-span integration through stage_mib-MiB staging; returns the
    case description on success, raises on any mismatch or error"""
    import numpy as np
    import oracle_c as co
    import paf_b2p
    g = case_geom(layout, mib)
    nframes = g.nsamp_int // g.nsamp_df
    buf = co.fill_synthetic(g, g.block_bytes, seed, 2, 8)
    cuts = sorted({int(f * nframes) for f in cut_fracs} - {0, nframes})
    bounds = [0] + [c * g.frame_bytes for c in cuts] + [g.block_bytes]
    with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()), tuning={"stage_mib": stage_mib}) as it:
        if register:
            it.register_host(buf)
        try:
            for a, b in zip(bounds[:-1], bounds[1:]):
                it.push(buf[a:b])
            out = it.finish()
        finally:  # never leave freed memory registered for the next example
            if register:
                it.unregister_host(buf)
    want = co.power(g, buf, nthreads=8)
    assert np.array_equal(out.view(np.uint32), want.view(np.uint32)), (layout, stage_mib, mib, cuts, register)
    return {"layout": layout, "stage_mib": stage_mib, "mib": mib, "cuts": cuts, "register": register}


def main():
    nbit, be, nchunk, ncc, nsamp_df, nframes, stage_mib, register = map(int, sys.argv[1:9])
    cuts = [] if sys.argv[9] == "-" else [int(x) for x in sys.argv[9].split(",")]
    seed = int(sys.argv[10])
    import numpy as np
    import b2p_oracle as npo
    import oracle_c as co
    import paf_b2p
    g = npo.Geom(nbit=nbit, big_endian=be, nchunk=nchunk, nsamp_df=nsamp_df, nchan_chunk=ncc,
                 nsamp_int=nframes * nsamp_df)
    buf = co.fill_synthetic(g, g.block_bytes, seed, 2, 8)
    bounds = [0] + [c * g.frame_bytes for c in cuts] + [g.block_bytes]
    res = {"case": sys.argv[1:], "frame_bytes": g.frame_bytes, "block_bytes": g.block_bytes}
    try:
        with paf_b2p.Integrator(paf_b2p.make_geom(**g.asdict()), tuning={"stage_mib": stage_mib}) as it:
            res["launch"] = {"threads": it.info.threads, "columns": it.info.columns,
                             "row_groups": it.info.row_groups, "row_vectors": it.info.row_vectors}
            if register:
                it.register_host(buf)
            try:
                for a, b in zip(bounds[:-1], bounds[1:]):
                    it.push(buf[a:b])
                out = it.finish()
            finally:
                if register:
                    it.unregister_host(buf)
        res["equal"] = bool(np.array_equal(out.view(np.uint32), co.power(g, buf, nthreads=8).view(np.uint32)))
    except Exception as e:  # noqa: BLE001 -- reported
        res["error"] = str(e)[-300:]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
