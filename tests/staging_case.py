"""One host-staging case in its own process (test infrastructure): a GPU
fault in one case must not poison the next one's HIP context.  Used by
tests/test_gpu_random_layouts.py's diagnosis runs:

  python3 tests/staging_case.py NBIT BE NCHUNK NCC NSAMP_DF NFRAMES STAGE_MIB REGISTER CUTS SEED

CUTS: comma-separated frame indexes (or "-").  Prints one JSON line."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(REPO, "paf-baseband2power_amd"), os.path.join(REPO, "oracle")]


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
            for a, b in zip(bounds[:-1], bounds[1:]):
                it.push(buf[a:b])
            out = it.finish()
            if register:
                it.unregister_host(buf)
        res["equal"] = bool(np.array_equal(out.view(np.uint32), co.power(g, buf, nthreads=8).view(np.uint32)))
    except Exception as e:  # noqa: BLE001 -- reported
        res["error"] = str(e)[-300:]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
