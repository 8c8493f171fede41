#!/usr/bin/env python3
"""bench.py -- baseband Msamples/s integrated + % HBM-read roofline.

One "step" = one full 1024x1024-sample integration (README.md:2) of one
sub-band per GPU: the HBM-resident block is unpacked, detected and
time-integrated by the gfx950 kernel and the fp32 spectrum is emitted
(finalize kernel).  Default workload = BASELINE.json configs[1]: 256 chans
x 2 pols int8 (1 GiB per integration).  Inputs are synthetic (counter-based
generator) and rotate over 4 distinct 1-GiB blocks per GPU so the
256 MiB Infinity Cache cannot serve repeats.

Multi-GPU (torchrun, one process per GPU): sub-band r on GPU r, no data-path
collective; the K spectra of every rank are gathered to rank 0 over RCCL
(torch.distributed "nccl") inside the timed region (configs[3]/[4]).
value = all ranks' samples / max-over-ranks time  (weak scaling).
--split time instead cuts ONE sub-band's integration along time across the
ranks (second mode): each rank integrates its share, emits
exact uint64 partials, and one RCCL reduce (SUM) of the K x nout partials
brings them to rank 0, which rounds once to fp32 (strong scaling; value =
one sub-band's samples / max-over-ranks time).

Prints ONE JSON line on rank 0.  Options beyond the driver contract:
  --config c2|c5|bmf|c3   workload (c3 = pinned host buffer, H2D overlapped;
                          its value is PCIe-bound and is never the default)
  --cpu-seconds S         bounded CPU-baseline sample (0 disables)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))

import torch  # noqa: E402  (first: one HIP runtime per process, see paf_b2p/_lib.py)
import torch.distributed as dist  # noqa: E402

import paf_b2p  # noqa: E402
from paf_b2p import distributed as D  # noqa: E402
from paf_b2p.geometry import CONFIGS, samples_per_block  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
try:  # the metric string exactly as BASELINE.json names it
    METRIC = json.load(open(os.path.join(REPO, "BASELINE.json"), encoding="utf-8"))["metric"]
except (OSError, ValueError, KeyError):
    METRIC = "baseband Msamples/s integrated + % HBM-read roofline, 1024\u00d71024 accum"
SEED = 20181105
NBLOCKS = 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c2", choices=["c2", "c5", "bmf", "c3"])
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on one GPU (spectra gathered on the host)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed even at world size 1 (rehearses the "
                         "RCCL gather path on one GPU)")
    ap.add_argument("--split", default="subband", choices=["subband", "time"],
                    help="time: one integration split across the ranks (strong scaling)")
    ap.add_argument("--no-fuse", action="store_true",
                    help="use b2p_push + b2p_finish_async instead of b2p_integrate")
    return ap.parse_args()


def pmc_traffic(config: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary for this
    config (profiles/pmc_<config>.json, written by tools/pmc_summary.py from
    separate --pmc passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM)."""
    p = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None, None
    try:
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), os.path.relpath(p, REPO)
    except Exception:
        return None, None


def _host_cpu() -> dict:
    """model / logical CPUs / NUMA nodes of the box (SURVEY.md 8d asks for them)"""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        numa = len([d for d in os.listdir("/sys/devices/system/node") if d.startswith("node")])
    except OSError:
        numa = None
    return {"model": model, "logical_cpus": os.cpu_count(), "numa_nodes": numa}


def cpu_baseline(geom, seconds: float, threads: int):
    """The oracle's C restatement (oracle/b2p_oracle.c), OpenMP over host
    threads, on a bounded sample of the same workload held in host RAM;
    a quarter of the budget times it on one thread as well."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import b2p_oracle as npo  # noqa: E402
    import oracle_c as co  # noqa: E402
    g = npo.Geom(**geom.as_dict())
    sample_bytes = min(g.block_bytes, 256 << 20) // g.frame_bytes * g.frame_bytes
    buf = co.fill_synthetic(g, sample_bytes, SEED, 0, 0)
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)

    def timed(nthreads, budget):
        co.integrate(g, buf[: g.frame_bytes * 64], nthreads=nthreads)  # warm
        passes, t0 = 0, time.perf_counter()
        while True:
            co.integrate(g, buf, nthreads=nthreads)
            passes += 1
            el = time.perf_counter() - t0
            if el >= budget or passes >= 100000:
                return passes, el

    passes, el = timed(threads, seconds * 0.75)
    p1, e1 = timed(1, seconds * 0.25)
    per_pass = sample_bytes // g.word_bytes * g.npol
    return {"value": round(passes * per_pass / el / 1e6, 2), "unit": "Msamples/s", "cores": threads,
            "kind": "port",
            "sample": f"{passes} passes over {sample_bytes >> 20} MiB of the same synthetic "
                      f"{g.nchan}-chan int{g.nbit} block ({el:.1f} s, host RAM, no file I/O)",
            "value_1thread": round(p1 * per_pass / e1 / 1e6, 2),
            "host": _host_cpu()}


def main():
    a = parse()
    rank, world, local = D.env_ranks()
    n_gpus = max(world, 1)
    cfg = CONFIGS[a.config]
    geom = cfg["geom"]()
    dist_on = world > 1 or a.force_dist
    rccl = dist_on and a.dist_backend == "nccl"
    if dist_on:
        D.init(a.dist_backend, local)
    split = a.split == "time"
    subband = 0 if split else D.subband_of(rank)
    spb = samples_per_block(geom)  # one sub-band's integration
    elem0 = 0
    if split:  # this rank's share of the integration's frames
        first, nf = D.time_share(rank, world, geom.nsamp_int // geom.nsamp_df)
        full_nsamp = geom.nsamp_int
        geom = paf_b2p.make_geom(**{f: getattr(geom, f) for f, _ in geom._fields_ if f != "reserved"})
        geom.nsamp_int = nf * geom.nsamp_df
        elem0 = first * paf_b2p.geometry.frame_bytes(geom) // (geom.nbit // 8)
    # with one visible GPU every rank maps to it (paf_baseband2power.cu:89-90)
    it = paf_b2p.Integrator(geom, device=D.device_of(local))
    nout, bb = it.nout, it.block_bytes
    if rccl:
        # one stream for the integrator and torch: the collective after the
        # loop is stream-ordered behind the last finalize, with no host wait
        # in between (b2p_set_stream; torch's NCCL work waits on this stream)
        ts = torch.cuda.Stream()
        torch.cuda.set_stream(ts)
        it.set_stream(ts.cuda_stream)

    if split:
        # exact partial sums, K x nout uint64 (as int64 for torch), reduced
        # to rank 0 after the loop; rank 0 then rounds them to fp32
        sums_t = torch.zeros((max(a.steps, 1), nout), dtype=torch.int64, device="cuda")
        spec_t = torch.zeros((max(a.steps, 1), nout), dtype=torch.float32, device="cuda")
        out_ptr = sums_t.data_ptr()
    elif rccl:
        # finalize writes the K spectra straight into torch device memory;
        # the gather follows the last finalize on the shared stream
        out_t = torch.zeros((a.steps, nout), dtype=torch.float32, device="cuda")
        out_ptr = out_t.data_ptr()
    else:
        out_buf = it.alloc(max(a.steps, 1) * nout * 4)
        out_ptr = out_buf.ptr

    host_mode = a.config == "c3"
    blocks = []
    if host_mode:
        import numpy as np
        hb = np.empty(bb, dtype=np.uint8)
        d = it.alloc(bb)
        it.fill_synthetic(d, SEED, subband, 0, elem0=elem0)
        hb[:] = it.download(d)
        d.free()
        it.register_host(hb)
        blocks = [hb]
    else:
        for b in range(NBLOCKS):
            d = it.alloc(bb)
            it.fill_synthetic(d, SEED, subband, b, elem0=elem0)
            blocks.append(d)
    it.sync()

    def step(k, out_row):
        if split:  # this rank's share -> exact partial sums (row out_row)
            it.push(blocks[k % len(blocks)])
            it.finish_partial(out_ptr + (out_row or 0) * nout * 8, True)
            return
        dst = out_ptr + (out_row or 0) * nout * 4
        if a.no_fuse or host_mode:  # the push / finish_async pair
            it.push(blocks[k % len(blocks)])
            it.finish_async(dst, True)
        else:  # b2p_integrate: one integrate launch per integration (its
            # finalize rides on the next launch)
            it.integrate(blocks[k % len(blocks)], dst, True)

    for w in range(a.warmup):
        step(w, None)
    it.sync()
    if dist_on:
        if rccl:
            torch.cuda.synchronize()
        # the first collective of a communicator sets up its channels; run
        # the timed region's collective once here, on same-shaped buffers
        if split:
            D.reduce_sums(sums_t if rccl else sums_t.cpu())
        elif rccl:
            D.gather_spectra(out_t)
        else:
            D.gather_spectra(torch.zeros((a.steps, nout), dtype=torch.float32))
        if rccl:
            torch.cuda.synchronize()
        dist.barrier()

    it.reset_stats()
    # one event pair on the integrator's stream around the K launches (per-
    # launch events would put a few us of event plumbing between kernels)
    it.set_timing(2)
    t0 = time.perf_counter()
    for k in range(a.steps):
        step(a.warmup + k, k)
    it.set_timing(0)  # records the closing event right behind the last launch (no wait)
    if not rccl:
        it.sync()
    if split:
        if dist_on:
            if rccl:
                total = D.reduce_sums(sums_t)  # RCCL reduce (SUM) of K x nout partials
            else:  # gloo rehearsal: partials through host memory
                host_total = D.reduce_sums(sums_t.cpu())
                total = host_total.cuda() if host_total is not None else None
        else:
            total = sums_t
        if rank == 0:
            it.finalize_sums(total.data_ptr(), a.steps, spec_t.data_ptr(), full_nsamp)
            it.sync()
        torch.cuda.synchronize()
    elif rccl:
        gathered = D.gather_spectra(out_t)  # RCCL all-gather of K x nout fp32
        torch.cuda.synchronize()
    elif dist_on:
        host = it.download(out_buf, nbytes=a.steps * nout * 4).view("float32").reshape(a.steps, nout)
        gathered = D.gather_spectra(torch.from_numpy(host.copy()))
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t0
    st = it.stats()

    el_max = D.max_over_ranks(el, "cuda" if rccl else "cpu") if dist_on else el
    if dist_on and rank == 0 and not split:
        assert len(gathered) == world and all(g.shape == (a.steps, nout) for g in gathered)

    kern_avg_s = st["kernel_ms"] / max(st["launches"], 1) / 1e3
    bytes_per_launch = st["bytes"] / max(st["launches"], 1)
    achieved = bytes_per_launch / kern_avg_s / 1e9 if kern_avg_s > 0 else 0.0
    traffic, traffic_src = pmc_traffic(a.config)

    if rank == 0:
        value = D.aggregate_rate(1 if split else n_gpus, a.steps, spb, el_max)
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(el_max / max(a.steps, 1) * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if split else "weak",
            "vs_baseline": None,
            "dtype": f"int{geom.nbit}" + ("-be" if geom.big_endian else ""),
            "data": "synthetic (counter-based SplitMix64 Gaussian, seed 20181105, sub-band = rank)",
            "config": {
                "workload": cfg["what"] + (
                    f"; ONE integration split by time over {world} GPU(s), exact partials reduced"
                    if split else ("" if world == 1 else f"; {world} sub-bands, 1 per GPU")),
                "baseline_config": {"c2": "configs[1]", "c5": "configs[4]", "c3": "configs[2]",
                                    "bmf": "reference-native"}[a.config],
                "nchan": int(geom.nchunk * geom.nchan_chunk),
                "npol": int(geom.npol),
                "nsamp_int": int(geom.nsamp_int),
                "bytes_per_integration": int(bb * (world if split else 1)),
                "input": "pinned host buffer, H2D overlapped (PCIe-inclusive)" if host_mode
                         else f"HBM-resident, {NBLOCKS} rotating blocks",
                "parallelism": (f"time split x{n_gpus}" + (
                    (", RCCL reduce (SUM) of uint64 partials" if rccl else ", gloo reduce (rehearsal)")
                    if dist_on else "")) if split else (f"sub-band sharding x{n_gpus}" + (
                    (", RCCL all-gather of spectra" if rccl else ", gloo gather (rehearsal)")
                    if dist_on else "")),
                "launch": {"threads": it.info.threads, "columns": it.info.columns,
                           "row_groups": it.info.row_groups, "replicas": it.info.replicas,
                           "unroll": it.info.unroll, "nt_loads": bool(it.info.nontemporal)},
            },
            "roofline": {
                "bound": "hbm",
                "kernel": "b2p_integrate_kernel",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "avg_launch_us": round(kern_avg_s * 1e6, 2),
                "timing": "HIP events on the integrator stream bracketing the timed launches "
                          "(region / launches: gaps and finalizes included, an upper bound)",
                "finalizes": ("carried by the next integrate launch; "
                              f"{st['finalizes']} standalone finalize launch(es) inside the region"),
            },
            "cpu_baseline": None,
        }
        if world == 1 and a.cpu_seconds > 0 and not host_mode:
            res["cpu_baseline"] = cpu_baseline(geom, a.cpu_seconds, a.cpu_threads)
        print(json.dumps(res), flush=True)

    for b in blocks:
        if hasattr(b, "free"):
            b.free()
    if host_mode:
        it.unregister_host(blocks[0])
    it.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
