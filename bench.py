#!/usr/bin/env python3
"""bench.py -- baseband Msamples/s integrated + % HBM-read roofline.

One "step" = one full 1024x1024-sample integration (README.md:2) of one
sub-band per GPU: the HBM-resident block is unpacked, detected and
time-integrated by the gfx950 kernel and the fp32 spectrum is emitted.
Default workload = BASELINE.json configs[1]: 256 chans x 2 pols int8 (1 GiB
per integration).  Inputs are synthetic (counter-based generator)
and rotate over 4 distinct blocks per GPU so the 256 MiB Infinity Cache
cannot serve repeats.

Ranks.  `--gpus N` is the number of ranks, one process per GPU:
  * under torch.distributed.run (WORLD_SIZE set) every rank checks that
    WORLD_SIZE == --gpus and exits 2 otherwise;
  * without a launcher and N > 1, this process starts
    `python3 -m torch.distributed.run --nproc-per-node N bench.py ...` as a
    child BEFORE touching the GPU, waits for it and exits with its code (rank
    0 prints the JSON line).  RCCL needs N visible GPUs; `--dist-backend
    gloo` rehearses N ranks sharing fewer GPUs (spectra gathered on the host).
Sub-band r lives on GPU r, no data-path collective; the K spectra of every
rank are gathered to rank 0 (torch.distributed gather; "nccl" = RCCL)
inside each timed region (configs[3]/[4]).  value = all ranks' samples /
max-over-ranks time (weak scaling).  `--split time` instead cuts ONE
sub-band's integration along time across the ranks (second
mode): exact uint64 partials, one reduce (SUM) to rank 0, one fp32 rounding
there (strong scaling).

Timing.  A timed region is EXACTLY --steps integrations bracketed by a
barrier + device synchronize on both sides, its collective included.  The
region is repeated until --min-seconds of timed work has accumulated (a
20-step region of configs[1] is only 3 ms); every rank's region times are
max-reduced per repeat and `value` / `ms_per_step` come from the median
repeat (all repeats' range is reported).

Verification.  After timing, every rank downloads each input block its last
region integrated and checks every spectrum that region emitted bit for bit
against the C oracle (outside the timed region; the oracle is the checker,
never the measured path); rank 0 also checks that the gathered spectra equal
what each rank holds.  `verified` is in the JSON line and a mismatch exits 3.

Launch shape.  The headline integrates bench.py's HBM-resident blocks as the
stage integrates blocks queued in its ring: floor(4 GiB / block) per launch
(b2p_integrate_n), e.g. 4 for configs[1].  A real-time ring never queues, so
the stage then launches one block at a time: that shape is timed in the same
run after the headline (`one_per_launch`, --bpl1-seconds) and verified too.

Roofline.  `roofline.frac` is from HIP events around each region's launches,
`frac_of_value` from the host-timed median region `value` comes from (the two
differ by the region's host bracketing), `frac_kernel_only` from per-launch
packet events.  `traffic` is the committed PMC summary's, marked STALE when
the kernel's sources changed after it was measured (`provenance`).

Secondary layouts.  At one rank with the default configs[1] workload the
line also carries `secondary`: the reference-native BMF layout, configs[4]'s
per-GPU share and configs[2] (pinned host, PCIe-bound), each timed for
--secondary-seconds after the headline, verified against the oracle and
given a roofline of its own; the headline `value` stays configs[1].

Prints ONE JSON line on rank 0.  Options beyond the driver contract:
  --config c2|c5|bmf|c3   workload (c3 = pinned host buffer, H2D overlapped;
                          its value is PCIe-bound and is never the default)
  --cpu-seconds S         bounded CPU-baseline sample (0 disables)
  --blocks N              distinct input blocks per rank (default 4)
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "paf-baseband2power_amd")
ORACLE = os.path.join(REPO, "oracle")

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
try:  # the metric string exactly as BASELINE.json names it
    METRIC = json.load(open(os.path.join(REPO, "BASELINE.json"), encoding="utf-8"))["metric"]
except (OSError, ValueError, KeyError):
    METRIC = "baseband Msamples/s integrated + % HBM-read roofline, 1024×1024 accum"
SEED = 20181105
NBLOCKS = 4
BASELINE_CONFIG = {"c2": "configs[1]", "c5": "configs[4]", "c3": "configs[2]", "bmf": "reference-native"}


def baseline_config(config: str, world: int, split: bool) -> str:
    """which BASELINE.json config this run is: configs[1] is one 256-ch
    sub-band on 1 GPU, configs[3] four of them gathered to rank 0,
    configs[4] eight 1024-ch sub-bands; other world sizes run the same
    per-GPU workload (weak scaling)"""
    if split:
        return f"{BASELINE_CONFIG[config]}, one integration split over {world} GPU(s)"
    if world == 1:
        return BASELINE_CONFIG[config]
    if config == "c2":
        return "configs[3]" if world == 4 else f"configs[1] per GPU x{world} (configs[3] is x4)"
    if config == "c5":
        return "configs[4]" if world == 8 else f"configs[4] per GPU x{world} (configs[4] is x8)"
    return f"{BASELINE_CONFIG[config]} per GPU x{world}"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks, one process per GPU")
    ap.add_argument("--steps", type=int, default=50, help="integrations per timed region")
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--min-seconds", type=float, default=5.0,
                    help="repeat the K-step region until this much timed work has run")
    ap.add_argument("--config", default="c2", choices=["c2", "c5", "bmf", "c3"])
    ap.add_argument("--cpu-seconds", type=float, default=9.0,
                    help="CPU-baseline budget, run after the GPU legs: 60 %% for the tuned port at "
                         "every CPU the job may use (>= 5 s by default), 25 %% at 1 thread, 15 %% "
                         "for the oracle beside it; the every-logical-CPU leg adds 15 %%")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N ranks on fewer GPUs (spectra gathered on the host)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed even at world size 1 (rehearses the "
                         "RCCL gather path on one GPU)")
    ap.add_argument("--split", default="subband", choices=["subband", "time"],
                    help="time: one integration split across the ranks (strong scaling)")
    ap.add_argument("--no-fuse", action="store_true",
                    help="use b2p_push + b2p_finish_async instead of b2p_integrate")
    ap.add_argument("--no-verify", action="store_true", help="skip the post-timing oracle check")
    ap.add_argument("--blocks-per-launch", type=int, default=0, choices=range(0, 9), metavar="0..8",
                    help="integrations per integrate launch (b2p_integrate_n: a consumer draining "
                         "queued HBM-resident blocks); 1 = one b2p_integrate per block; 0 (default) = "
                         "auto, as the stage batches queued blocks: floor(4 GiB / block), 1..8")
    ap.add_argument("--blocks", type=int, default=0,
                    help="distinct HBM-resident input blocks per rank (0 = auto: 4, or the blocks "
                         "per launch if more); fewer than 4 lets the 256 MiB Infinity Cache serve "
                         "repeats of small blocks, so use it only to fit many ranks on one GPU")
    ap.add_argument("--bpl1-seconds", type=float, default=2.0,
                    help="when the headline batches queued blocks, also time this long of regions "
                         "with ONE block per launch (the real-time stage's launch shape) and report "
                         "it beside the headline (0 disables)")
    ap.add_argument("--secondary", default="bmf,c5,c3",
                    help="with the default configs[1] workload at one rank, also time these layouts after the "
                         "headline and report each under `secondary`, verified against the oracle: bmf "
                         "(reference-native int16 BE TFTFP, 2.625 GiB), c5 (configs[4] per GPU, 1024 ch, 4 GiB), "
                         "c3 (configs[2], 4 GiB from pinned host memory, PCIe-bound); '' for none")
    ap.add_argument("--secondary-seconds", type=float, default=2.0,
                    help="timed seconds per secondary layout")
    ap.add_argument("--dist-timeout", type=float, default=300.0,
                    help="seconds one multi-rank phase (rendezvous, first collective, a timed "
                         "region, verification) may take; past it the rank exits 4 naming it")
    a = ap.parse_args(argv)
    bad = [x for x in a.secondary.split(",") if x and x not in SECONDARY_WHAT]
    if bad:
        ap.error(f"--secondary: unknown layout(s) {bad}; choose from {sorted(SECONDARY_WHAT)}")
    if a.gpus < 1 or a.steps < 1 or a.warmup < 0 or a.blocks < 0:
        ap.error("--gpus and --steps must be >= 1, --warmup and --blocks >= 0")
    return a


# --------------------------------------------------------------------------
# launcher: N ranks without an external torch.distributed.run
# --------------------------------------------------------------------------
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launcher_cmd(a, argv: list[str], port: int) -> list[str]:
    """the torch.distributed.run command line that starts a.gpus ranks of
    this script with the same arguments"""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
            f"--nproc-per-node={a.gpus}", "--master-addr", "127.0.0.1", "--master-port", str(port),
            os.path.abspath(__file__), *argv]


def visible_gpus() -> int:
    """device count without initialising HIP (true of torch.cuda.device_count
    on this image)"""
    import torch
    return torch.cuda.device_count()


def launch_ranks(a, argv: list[str]) -> int:
    """Start a.gpus ranks as ONE child process tree and wait for it.  Called
    before anything in this process touches the GPU; this process never
    initialises HIP and never execs."""
    if a.dist_backend == "nccl":
        n = visible_gpus()
        if n < a.gpus:
            print(f"bench.py: --gpus {a.gpus} over RCCL needs {a.gpus} visible GPUs, found {n} "
                  "(RCCL refuses two ranks on one device; --dist-backend gloo rehearses)",
                  file=sys.stderr)
            return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["BENCH_LAUNCHED_RANKS"] = str(a.gpus)
    return subprocess.run(launcher_cmd(a, argv, _free_port()), env=env).returncode


def check_world(a, world: int) -> str | None:
    """None if the launched world matches --gpus, else the reason to refuse"""
    if world != a.gpus:
        return (f"bench.py: WORLD_SIZE={world} but --gpus {a.gpus}; refusing to report "
                f"{world} rank(s) as {a.gpus} GPU(s)")
    return None


# --------------------------------------------------------------------------
# labels
# --------------------------------------------------------------------------
def workload_label(config: str, geom_desc: str, world: int, split: bool, host_mode: bool,
                   ndev: int | None = None) -> str:
    """what ran, on how many GPUs: ndev (the GPUs the ranks map to) below
    world means ranks sharing GPUs, a gloo rehearsal of the plumbing"""
    ndev = world if ndev is None else ndev
    where = "pinned host buffer, H2D overlapped" if host_mode else "HBM-resident"
    over = (f"{world} MI355X" if ndev >= world
            else f"{world} ranks sharing {ndev} MI355X (rehearsal, not a scaling run)")
    if split:
        return (f"1 sub-band, {geom_desc}, {where}; one integration split by time over "
                f"{over}, exact partials reduced to rank 0")
    return (f"{world} sub-band(s), {geom_desc} each, {where}, "
            + (f"1 per MI355X over {over}" if ndev >= world else f"over {over}")
            + (", spectra gathered to rank 0" if world > 1 else ""))


def parallelism_label(world: int, split: bool, dist_on: bool, rccl: bool) -> str:
    if split:
        s = f"time split x{world}"
        if dist_on:
            s += ", RCCL reduce (SUM) of uint64 partials" if rccl else ", gloo reduce (rehearsal)"
        return s
    s = f"sub-band sharding x{world}"
    if dist_on:
        s += ", RCCL gather of spectra to rank 0" if rccl else ", gloo gather to rank 0 (rehearsal)"
    return s


# the sources that decide what the integrate kernel reads (its code and its
# launch planner): a PMC summary measured on other sources is stale
KERNEL_SOURCES = ("paf-baseband2power_amd/csrc/b2p_kernels.hip", "paf-baseband2power_amd/csrc/b2p_ctx.hip",
                  "paf-baseband2power_amd/csrc/b2p_internal.h", "paf-baseband2power_amd/csrc/b2p_plan.h")


def kernel_sources_sha() -> str:
    """sha256 over KERNEL_SOURCES' bytes, in order (no git needed: the GPU
    box's snapshot has no .git); tools/pmc_summary.py stamps it into
    profiles/pmc_<config>.json"""
    import hashlib
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        with open(os.path.join(REPO, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    return h.hexdigest()


def device_code_sha(lib: str | None = None) -> str | None:
    """sha256 of the gfx950 code objects the library carries (its ELF
    section .hip_fatbin): what the GPU runs.  A change to the host half of
    KERNEL_SOURCES (b2p_ctx.hip) changes kernel_sources_sha but not this;
    None if the library has no such section"""
    import hashlib
    import struct
    if lib is None:
        sys.path.insert(0, PKG)
        from paf_b2p import _lib
        lib = _lib.LIB_PATH
    try:
        data = open(lib, "rb").read()
    except OSError:
        return None
    if data[:4] != b"\x7fELF" or data[4] != 2:  # ELF64 only
        return None
    shoff = struct.unpack_from("<Q", data, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)

    def section(i):  # sh_name, sh_type, sh_flags, sh_addr, sh_offset, sh_size, ...
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    names = section(shstrndx)[4]
    for i in range(shnum):
        sh = section(i)
        name = data[names + sh[0]: data.index(b"\0", names + sh[0])]
        if name == b".hip_fatbin":
            return hashlib.sha256(data[sh[4]: sh[4] + sh[5]]).hexdigest()
    return None


def pmc_traffic(config: str, bytes_per_launch: float):
    """HBM bytes per launch from the committed rocprofv3 PMC summary for this
    config (profiles/pmc_<config>.json, written by tools/pmc_summary.py from
    separate --pmc passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM).
    Measured on launches of another size (blocks per launch), it is scaled
    by this run's algorithmic bytes per launch, and the source says so.
    Returns (bytes, source, provenance): provenance names the commit the
    summary was measured on and whether the kernel sources changed since
    (`stale`: then the traffic belongs to other code)."""
    p = os.path.join(REPO, "profiles", f"pmc_{config}.json")
    if not os.path.exists(p):
        return None, None, None
    try:
        d = json.load(open(p))
        hbm, alg = d.get("hbm_bytes_per_launch"), d.get("algorithmic_bytes_per_launch")
        src = os.path.relpath(p, REPO)
        sha = d.get("kernel_sources_sha256")
        prov = {"measured_commit": d.get("commit"), "kernel_sources_commit": d.get("kernel_sources_commit"),
                "stale": sha != kernel_sources_sha() if sha else None}
        if d.get("device_code_sha256"):  # the code objects measured vs the ones this run loads
            prov["device_code_match"] = d["device_code_sha256"] == device_code_sha()
        if prov["stale"] is None:
            prov["note"] = "summary predates source stamping: freshness unknown"
        if prov["stale"]:
            src += " (STALE: the kernel sources changed after it was measured)"
        if hbm and alg and bytes_per_launch and int(alg) != int(bytes_per_launch):
            return (int(round(hbm / alg * bytes_per_launch)),
                    f"{src} (measured on {alg}-B launches, scaled to {int(bytes_per_launch)} B)", prov)
        return hbm, src, prov
    except (OSError, ValueError):
        return None, None, None


# --------------------------------------------------------------------------
# CPU baseline and verification (the oracle's only uses; outside any timing)
# --------------------------------------------------------------------------
def cpu_threads() -> int:
    sys.path.insert(0, ORACLE)
    import cpu_baseline as cb
    return cb.effective_cpus()


def cpu_baseline(geom_dict: dict, seconds: float) -> dict | None:
    """The tuned CPU port (oracle/b2p_cpu_port.c) timed in a child process
    (its own OpenMP binding), at the job's CPU quota less one thread
    (cpu_baseline.baseline_threads: threads that fill the quota exactly get
    throttled) with libgomp's default wait policy, and at 1 thread, with the scalar
    oracle beside it, on one full block.  The line reports the share of
    throttled cgroup periods and the interquartile range beside `value`."""
    sys.path.insert(0, ORACLE)
    import cpu_baseline as cb
    threads = cb.baseline_threads()
    picked = cb.pick_cpus(threads)

    def child(env, budget, *extra):
        r = subprocess.run([sys.executable, os.path.join(ORACLE, "cpu_baseline.py"),
                            json.dumps(geom_dict), str(budget), str(SEED), *extra], env=env,
                           capture_output=True, text=True, timeout=max(120, budget * 10))
        if r.returncode != 0:
            print(f"bench.py: cpu baseline failed ({r.returncode}): {r.stderr[-500:]}", file=sys.stderr)
            return None
        return json.loads(r.stdout.strip().splitlines()[-1])

    res = child(cb.child_env(threads, cpus=picked["cpus"], wait="default"), seconds)
    if res is not None:
        res["cpus_picked"] = {**picked, "rule": "the cgroup quota less one thread, one logical CPU per "
                                                "physical core, dealt round-robin over every L3 domain (CCD) "
                                                "of every NUMA node, the idlest allowed core of each over the "
                                                "sample before the legs; CPU order, so each thread's "
                                                "first-touched tile is on its own node; libgomp's default wait "
                                                "policy (OMP_WAIT_POLICY unset)"}
    return res


def oracle_spectrum(geom_dict: dict, read_chunk, nbytes: int, threads: int):
    """oracle fp32 spectrum of a block, fed in whole-frame chunks (exact
    uint64 sums accumulate across chunks)"""
    sys.path.insert(0, ORACLE)
    import numpy as np

    import b2p_oracle as npo
    import oracle_c as co
    g = npo.Geom(**geom_dict)
    step = max(1, (256 << 20) // g.frame_bytes) * g.frame_bytes
    acc = np.zeros(g.nout, dtype=np.uint64)
    for off in range(0, nbytes, step):
        n = min(step, nbytes - off)
        co.integrate(g, read_chunk(off, n), nthreads=threads, acc=acc)
    return co.finalize(g, acc)


def synthetic_reader(geom_dict: dict, subband: int, block: int, threads: int):
    """chunks of a synthetic block regenerated on the host by the oracle's
    C generator (the same counter-based stream as b2p_fill_synthetic)"""
    sys.path.insert(0, ORACLE)
    import b2p_oracle as npo
    import oracle_c as co
    g = npo.Geom(**geom_dict)
    esz = g.nbit // 8

    def rd(off, n):
        return co.fill_synthetic(g, n, SEED, subband, block, elem0=off // esz)
    return rd


SECONDARY_WHAT = {
    "bmf": ("reference-native", "BMF: 336 ch x 2 pol int16 BE TFTFP (48 chunks x 7 ch, 128 samples per frame)"),
    "c5": ("configs[4] per GPU", "1024 ch x 2 pol int8 (one of configs[4]'s eight sub-bands)"),
    "c3": ("configs[2]", "1024 ch x 2 pol int8 from a pinned host buffer, H2D overlapped"),
}


def secondary_leg(name: str, dev: int, seconds: float, vthreads: int, verify: bool) -> dict:
    """One of the other BASELINE layouts beside the headline, in the same
    run: "bmf" the reference-native layout the drop-in serves
    (capture.h:20,28; paf-baseband2power.conf:2-9), "c5" one GPU's share of
    configs[4], both HBM-resident over NBLOCKS rotating blocks, one block per
    integrate launch (floor(4 GiB / block) = 1, the stage's rule); "c3"
    configs[2], one block in a registered host buffer pushed through the
    staging pair (PCIe-bound; its ceiling, a bare H2D of the same block, is
    measured right after).  A region is the leg's integrations bracketed by
    device syncs; regions repeat for `seconds`; the last region's spectra
    are checked against the C oracle bit for bit.  Algorithmic bytes: 2 B
    per complex sample (int8), 4 B (int16); the block per launch."""
    import numpy as np

    import paf_b2p
    from paf_b2p.geometry import CONFIGS, samples_per_block
    geom = CONFIGS[name]["geom"]()
    gd = {f: int(getattr(geom, f)) for f, _ in geom._fields_ if f != "reserved"}
    host = name == "c3"
    it = paf_b2p.Integrator(geom, device=dev)
    nout, bb = it.nout, it.block_bytes
    K = 1 if host else NBLOCKS
    blocks = []
    try:
        if host:  # the block in pinned host memory, generated on the GPU and copied home once
            hb = np.empty(bb, dtype=np.uint8)
            d = it.alloc(bb)
            it.fill_synthetic(d, SEED, 0, 0)
            hb[:] = it.download(d)
            d.free()
            it.register_host(hb)
            blocks = [hb]
        else:
            for b in range(K):
                d = it.alloc(bb)
                it.fill_synthetic(d, SEED, 0, b)
                blocks.append(d)
        out = it.alloc(K * nout * 4)
        it.sync()

        def region():
            it.sync()
            t0 = time.perf_counter()
            it.set_timing(2)
            for k in range(K):
                if host:
                    it.push(blocks[k])
                    it.finish_async(out.ptr + k * nout * 4, True)
                else:
                    it.integrate(blocks[k], out.ptr + k * nout * 4, True)
            it.set_timing(0)
            it.sync()
            return time.perf_counter() - t0

        region()  # warm-up region
        it.reset_stats()
        els = [region()]
        while sum(els) < seconds and len(els) < 100000:
            els.append(region())
        st = it.stats()
        h2d = None
        if host:  # the leg's ceiling: a bare pinned H2D of the same block, same process
            dst = it.alloc(bb)
            it.upload_into(dst, blocks[0])
            rates, t_all = [], time.perf_counter()
            while len(rates) < 3 or (time.perf_counter() - t_all < 1.0 and len(rates) < 50):
                t0 = time.perf_counter()
                it.upload_into(dst, blocks[0])
                rates.append(bb / (time.perf_counter() - t0) / 1e9)
            dst.free()
            h2d = {"gbs": round(statistics.median(rates), 2), "copies": len(rates),
                   "range": [round(min(rates), 2), round(max(rates), 2)],
                   "what": f"hipMemcpy of the same {bb >> 20} MiB registered host block into HBM, no kernel"}
        ok = None
        if verify:
            spec = it.download(out, nbytes=K * nout * 4).view(np.float32).reshape(K, nout)
            ok = True
            for k in range(K):
                if host:
                    def rd(off, n, blk=blocks[k]):
                        return blk[off:off + n]
                else:
                    def rd(off, n, blk=blocks[k]):
                        return it.download(blk, nbytes=n, offset=off)
                ref = oracle_spectrum(gd, rd, bb, vthreads)
                ok &= bool(np.array_equal(spec[k].view(np.uint32), ref.view(np.uint32)))
        el = statistics.median(els)
        kern_s = st["kernel_ms"] / max(st["launches"], 1) / 1e3
        per_launch = st["bytes"] / max(st["launches"], 1)
        achieved = per_launch / kern_s / 1e9 if kern_s > 0 else 0.0
        traffic, src, prov = pmc_traffic(name, per_launch)
        baseline, what = SECONDARY_WHAT[name]
        res = {
            "baseline_config": baseline,
            "workload": (f"{what}, {bb} B per integration, "
                         + ("one block in a registered host buffer" if host else
                            f"{K} rotating HBM-resident blocks, 1 block per integrate launch")),
            "value": round(samples_per_block(geom) / (el / K) / 1e6, 1),
            "unit": "Msamples/s",
            "ms_per_step": round(el / K * 1e3, 4),
            "timed_regions": len(els),
            "timed_seconds": round(sum(els), 4),
            "verified": ok,
            "verification": f"every spectrum of the last region ({K}) against the C oracle of its block, bit for bit",
            "roofline": {
                "bound": "hbm", "kernel": "b2p_integrate_kernel<..., MULTI=false>",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "frac_of_value": round(bb / (el / K) / 1e9 / HBM_PEAK_GBS, 4),
                "algorithmic_bytes_per_launch": int(per_launch),
                "bytes_per_sample": int(geom.nbit // 8 * 2),
                "avg_launch_us": round(kern_s * 1e6, 2),
                "launches_timed": int(st["launches"]),
                "traffic": traffic, "traffic_source": src, "traffic_provenance": prov,
                "timing": ("frac: HIP events bracketing each region's launches (finalizes included); "
                           "frac_of_value: the host-timed median region"),
            },
        }
        if host:
            pcie = bb / (el / K) / 1e9
            hbm = dict(res["roofline"])
            res["roofline"] = {
                "bound": "pcie", "achieved": round(pcie, 2), "peak": h2d["gbs"], "unit": "GB/s",
                "frac": round(pcie / h2d["gbs"], 4), "peak_source": h2d,
                "algorithmic_bytes_per_launch": hbm["algorithmic_bytes_per_launch"],
                "hbm": {k: hbm[k] for k in ("achieved", "frac", "avg_launch_us", "launches_timed")},
                "timing": ("achieved: the block's bytes per ms_per_step (staging copies overlapped with the "
                           "integrate launches); peak: peak_source, the bare H2D stream of the same bytes"),
            }
        return res
    finally:
        if host and blocks:
            it.unregister_host(blocks[0])
        for d in blocks:
            if hasattr(d, "free"):
                d.free()
        it.close()


# --------------------------------------------------------------------------
def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return launch_ranks(a, argv)

    sys.path.insert(0, PKG)
    from paf_b2p import distributed as D
    rank, world, local = D.env_ranks()
    bad = check_world(a, world)
    if bad:
        print(bad, file=sys.stderr)
        return 2

    import numpy as np
    import torch  # first: one HIP runtime per process, see paf_b2p/_lib.py
    import torch.distributed as dist

    import paf_b2p
    from paf_b2p.geometry import CONFIGS, samples_per_block

    cfg = CONFIGS[a.config]
    geom = cfg["geom"]()
    dist_on = world > 1 or a.force_dist
    rccl = dist_on and a.dist_backend == "nccl"
    wd = D.Watchdog(rank, a.dist_timeout)
    if dist_on:
        with wd.phase(f"rendezvous ({a.dist_backend} init_process_group, {world} ranks)"):
            D.init(a.dist_backend, local, a.dist_timeout)
    split = a.split == "time"
    host_mode = a.config == "c3"
    subband = 0 if split else D.subband_of(rank)
    spb = samples_per_block(geom)  # one sub-band's integration
    full_geom = {f: int(getattr(geom, f)) for f, _ in geom._fields_ if f != "reserved"}
    elem0 = 0
    if split:  # this rank's share of the integration's frames
        first, nf = D.time_share(rank, world, geom.nsamp_int // geom.nsamp_df)
        full_nsamp = geom.nsamp_int
        geom = paf_b2p.make_geom(**full_geom)
        geom.nsamp_int = nf * geom.nsamp_df
        elem0 = first * paf_b2p.geometry.frame_bytes(geom) // (geom.nbit // 8)
    my_geom = {f: int(getattr(geom, f)) for f, _ in geom._fields_ if f != "reserved"}
    K = a.steps
    # rank r on GPU r; with one visible GPU every rank maps to it
    # (paf_baseband2power.cu:89-90).  torch's current device follows, so
    # its tensors (spectra, partials) live where the integrator runs
    dev = D.device_of(local)
    torch.cuda.set_device(dev)
    it = paf_b2p.Integrator(geom, device=dev)
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
        # to rank 0 after each region; rank 0 then rounds them to fp32
        sums_t = torch.zeros((K, nout), dtype=torch.int64, device="cuda")
        spec_t = torch.zeros((K, nout), dtype=torch.float32, device="cuda")
        out_ptr = sums_t.data_ptr()
    elif rccl:
        # finalize writes the K spectra straight into torch device memory;
        # the gather follows the last finalize on the shared stream
        out_t = torch.zeros((K, nout), dtype=torch.float32, device="cuda")
        out_ptr = out_t.data_ptr()
    else:
        out_buf = it.alloc(K * nout * 4)
        out_ptr = out_buf.ptr

    # several queued blocks per integrate launch (b2p_integrate_n), for the
    # HBM-resident fused path only; every integration still gets its spectrum
    bpl_auto = paf_b2p.blocks_per_launch(bb)
    bpl = a.blocks_per_launch or bpl_auto
    if not a.blocks_per_launch:  # auto: every launch the same size (a divisor of K)
        bpl = max(n for n in range(1, bpl + 1) if K % n == 0)
    if split or host_mode or a.no_fuse:
        bpl = 1
    nblocks = a.blocks or max(NBLOCKS, a.blocks_per_launch or bpl_auto)

    blocks = []
    if host_mode:
        hb = np.empty(bb, dtype=np.uint8)
        d = it.alloc(bb)
        it.fill_synthetic(d, SEED, subband, 0, elem0=elem0)
        hb[:] = it.download(d)
        d.free()
        it.register_host(hb)
        blocks = [hb]
    else:
        for b in range(nblocks):  # distinct blocks (within a launch too, when they suffice)
            d = it.alloc(bb)
            it.fill_synthetic(d, SEED, subband, b, elem0=elem0)
            blocks.append(d)
    it.sync()

    def step(k, out_row):
        blk = blocks[k % len(blocks)]
        if split:  # this rank's share -> exact partial sums (row out_row)
            it.push(blk)
            it.finish_partial(out_ptr + out_row * nout * 8, True)
            return
        dst = out_ptr + out_row * nout * 4
        if a.no_fuse or host_mode:  # the push / finish_async pair
            it.push(blk)
            it.finish_async(dst, True)
        else:  # b2p_integrate: one integrate launch per integration (its
            # finalize rides on the next launch)
            it.integrate(blk, dst, True)

    cur = {"bpl": bpl}  # the launch shape of the regions being timed
    # integrate launches per bench phase, in issue order (roofline.launch_phases:
    # tools/trace_legs.py cuts a rocprofv3 kernel trace of this run by them)
    phases, nl = [], {"n": 0, "mark": 0}

    def phase(name):
        phases.append([name, nl["n"] - nl["mark"]])
        nl["mark"] = nl["n"]

    def steps(k0, row0, n):
        """integrations k0 .. k0+n-1 into output rows row0 .."""
        j = 0
        while j < n:
            m = min(cur["bpl"], n - j)
            nl["n"] += 1
            if m == 1:
                step(k0 + j, row0 + j)
            else:
                it.integrate_n([blocks[(k0 + j + i) % len(blocks)] for i in range(m)],
                               out_ptr + (row0 + j) * nout * 4, True)
            j += m

    coll = {"op": "gather"}

    def collective():
        """the region's exchange: spectra gathered (or partials reduced) to
        rank 0; returns what rank 0 holds"""
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
                it.finalize_sums(total.data_ptr(), K, spec_t.data_ptr(), full_nsamp)
                it.sync()
            return None
        if rccl:
            if coll["op"] == "gather":
                return D.gather_spectra(out_t)  # RCCL gather of K x nout fp32 to rank 0
            return D.all_gather_spectra(out_t)
        if dist_on:
            host = it.download(out_buf, nbytes=K * nout * 4).view("float32").reshape(K, nout)
            return D.gather_spectra(torch.from_numpy(host.copy()))
        return None

    def fence():
        it.sync()
        if rccl or split:
            torch.cuda.synchronize()
        if dist_on:
            dist.barrier()

    kk = 0
    for _ in range(a.warmup):
        steps(kk, 0, 1 if bpl == 1 else min(bpl, K))
        kk += 1 if bpl == 1 else min(bpl, K)
    it.sync()
    phase("warmup")
    if dist_on:  # a communicator's first collective sets up its channels
        wd.arm(f"first {a.dist_backend} collective (communicator set-up)")
        try:
            collective()
        except RuntimeError as e:  # a backend without gather: every rank gets the spectra
            if split:
                raise
            print(f"bench.py: rank {rank}: gather failed ({e}); using all_gather", file=sys.stderr)
            coll["op"] = "all_gather"
            collective()
    fence()
    # who actually ran: the live group read back, and every rank's GPU
    world_seen = D.observed_world()
    ident = {"rank": rank, "local_rank": local, "host": socket.gethostname(),
             "device": int(it.info.device), "pci_bus_id": paf_b2p.pci_bus_id(int(it.info.device)),
             "name": torch.cuda.get_device_name(int(it.info.device)),
             "visible_devices": os.environ.get("HIP_VISIBLE_DEVICES")
             or os.environ.get("ROCR_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}
    idents = D.gather_identities(ident)
    ngpu_seen = D.distinct_gpus(idents)
    wd.disarm()

    def region():
        nonlocal kk
        if dist_on:
            wd.arm("a timed region (its collective included)")
        fence()
        t0 = time.perf_counter()
        it.set_timing(2)  # one event pair on the integrator's stream around the K launches
        steps(kk, 0, K)
        kk += K
        it.set_timing(0)  # records the closing event right behind the last launch (no wait)
        if not rccl:  # host-side exchange (gloo) reads what the integrator's stream wrote
            it.sync()
        got = collective()
        fence()
        wd.disarm()
        return time.perf_counter() - t0, got

    def timed_leg(min_seconds):
        """repeat the K-step region until min_seconds of timed work: every
        repeat's time max-reduced over the ranks; returns those times, this
        rank's per-step median, what rank 0 gathered last, the first step of
        the last region, and the integrator's event stats of the leg"""
        it.reset_stats()
        el0, got = region()
        el0_max = D.max_over_ranks(el0, "cuda" if rccl else "cpu") if dist_on else el0
        repeats = max(1, min(100000, math.ceil(min_seconds / max(el0_max, 1e-9))))
        els = [el0]
        for _ in range(repeats - 1):
            el, got = region()
            els.append(el)
        if dist_on:
            t = torch.tensor(els, dtype=torch.float64, device="cuda" if rccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            els_max = t.cpu().tolist()
        else:
            els_max = els
        return els_max, els, got, kk - K, it.stats()

    els_max, els, gathered, last_k0, st = timed_leg(a.min_seconds)
    phase("headline")
    if dist_on:
        mine = torch.tensor([statistics.median(els)], dtype=torch.float64,
                            device="cuda" if rccl else "cpu")
        per_rank = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(per_rank, mine)
        per_rank_ms = [round(float(x.item()) / K * 1e3, 4) for x in per_rank]
    else:
        per_rank_ms = [round(statistics.median(els) / K * 1e3, 4)]
    el_med = statistics.median(els_max)

    # ---- verification (outside timing) ------------------------------------
    def verify(k0, gathered):
        """every spectrum of the region that started at step k0 against the C
        oracle of its input block, bit for bit; rank 0 also checks the
        gathered spectra.  Returns (ok on every rank, info)"""
        vinfo = {}
        vthreads = max(1, cpu_threads() // world)
        rows_ok = True
        blocks_of_rows = {}
        for j in range(K):
            blocks_of_rows.setdefault((k0 + j) % len(blocks), []).append(j)
        if split:
            if rank == 0:
                spec = spec_t.cpu().numpy()
                for b, rows in blocks_of_rows.items():
                    ref = oracle_spectrum(full_geom, synthetic_reader(full_geom, 0, b, vthreads),
                                          paf_b2p.geometry.block_bytes(paf_b2p.make_geom(**full_geom)),
                                          vthreads)
                    rows_ok &= all(np.array_equal(spec[j].view(np.uint32), ref.view(np.uint32))
                                   for j in rows)
        else:
            if rccl:
                local_spec = out_t.cpu().numpy()
            else:
                local_spec = it.download(out_buf, nbytes=K * nout * 4).view(np.float32).reshape(K, nout)
            for b, rows in blocks_of_rows.items():
                blk = blocks[b]
                if host_mode:
                    def rd(off, n, blk=blk):
                        return blk[off:off + n]
                else:
                    def rd(off, n, blk=blk):
                        return it.download(blk, nbytes=n, offset=off)
                ref = oracle_spectrum(my_geom, rd, bb, vthreads)
                rows_ok &= all(np.array_equal(local_spec[j].view(np.uint32), ref.view(np.uint32))
                               for j in rows)
            if dist_on:  # rank 0 holds exactly what every rank emitted
                csum = torch.tensor([int(np.sum(local_spec.view(np.uint32), dtype=np.uint64))],
                                    dtype=torch.int64, device="cuda" if rccl else "cpu")
                sums = [torch.zeros_like(csum) for _ in range(world)]
                dist.all_gather(sums, csum)
                if rank == 0:
                    g_ok = len(gathered) == world and all(
                        tuple(gt.shape) == (K, nout) and
                        int(np.sum(gt.cpu().numpy().view(np.uint32), dtype=np.uint64)) == int(s.item())
                        for gt, s in zip(gathered, sums))
                    rows_ok &= g_ok
                    vinfo["gather"] = "rank 0 holds every rank's K spectra" if g_ok else "MISMATCH"
        ok_t = torch.tensor([1 if rows_ok else 0], dtype=torch.int64, device="cuda" if rccl else "cpu")
        if dist_on:
            dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        vinfo.update(what=(f"every spectrum of the last timed region ({K}) against the C oracle of "
                           f"its input block ({len(blocks_of_rows)} distinct block(s)"
                           + (", regenerated on the host" if split else ", downloaded from HBM")
                           + f"), bit for bit, {'rank 0' if split else 'every rank'}"),
                     threads=vthreads)
        return bool(ok_t.item()), vinfo

    verified = None
    vinfo = {}
    if dist_on:
        wd.arm("verification against the oracle", max(a.dist_timeout, 900.0))
    if not a.no_verify:
        verified, vinfo = verify(last_k0, gathered)
    wd.disarm()

    # the real-time launch shape beside the batched headline: the stage
    # launches one block at a time unless blocks are queued in its ring
    # (paf_baseband2power.c, run_device_pipelined), so time that too
    one = None
    if bpl > 1 and a.bpl1_seconds > 0:
        cur["bpl"] = 1
        steps(kk, 0, 1)  # warm the one-block launch shape
        kk += 1
        phase("one_per_launch_warmup")
        els1_max, _, gathered1, last1_k0, st1 = timed_leg(a.bpl1_seconds)
        phase("one_per_launch")
        el1 = statistics.median(els1_max)
        if dist_on:
            wd.arm("verification against the oracle (one block per launch)", max(a.dist_timeout, 900.0))
        ok1 = None if a.no_verify else verify(last1_k0, gathered1)[0]
        wd.disarm()
        if ok1 is False:
            verified = False
        k1 = st1["kernel_ms"] / max(st1["launches"], 1) / 1e3
        one = {"blocks_per_launch": 1, "ms_per_step": round(el1 / K * 1e3, 4),
               "value": round(D.aggregate_rate(world, K, spb, el1), 1),
               "frac_of_value": round(bb / (el1 / K) / 1e9 / HBM_PEAK_GBS, 4),
               "frac_events": round(st1["bytes"] / max(st1["launches"], 1) / k1 / 1e9 / HBM_PEAK_GBS, 4)
               if k1 > 0 else None,
               "timed_regions": len(els1_max), "timed_seconds": round(sum(els1_max), 4),
               "verified": ok1}
        cur["bpl"] = bpl

    # cross-check, outside every timed region: the integrate kernel alone,
    # timed by start/stop events on each launch's own dispatch packet (no
    # inter-launch gap, no finalize) -- the quantity rocprofv3 --kernel-trace
    # reports as the kernel's duration; at least 16 launches of the headline
    # shape, after one untimed launch (the GPU sat idle during verification)
    calib_us = None
    if not split and not host_mode and not a.no_fuse:
        n_c = (K // bpl) * bpl or K  # whole launches of the headline shape, rows < K
        steps(0, 0, n_c)
        it.sync()
        phase("calibration_warmup")
        it.reset_stats()
        it.set_timing(1)
        while it.stats()["launches"] < 16:
            steps(0, 0, n_c)
        it.set_timing(0)
        it.sync()
        phase("calibration")
        cs = it.stats()
        if cs["launches"]:
            calib_us = cs["kernel_ms"] / cs["launches"] * 1e3

    # configs[2]'s own ceiling: a bare pinned H2D stream of the same block,
    # measured in this run after the headline (hipMemcpy from the same
    # registered buffer into HBM, no kernel), so the line's PCIe fraction
    # has its denominator beside it ("vs PCIe H2D ceiling and
    # vs HBM")
    h2d = None
    if host_mode:
        dst = it.alloc(bb)
        it.upload_into(dst, blocks[0])  # untimed: first touch of the destination
        rates = []
        t_all = time.perf_counter()
        while len(rates) < 3 or time.perf_counter() - t_all < 2.0:
            t0 = time.perf_counter()
            it.upload_into(dst, blocks[0])
            rates.append(bb / (time.perf_counter() - t0) / 1e9)
            if len(rates) >= 50:
                break
        dst.free()
        h2d = {"gbs": round(statistics.median(rates), 2), "copies": len(rates),
               "range": [round(min(rates), 2), round(max(rates), 2)],
               "what": (f"hipMemcpy of the same {bb >> 20} MiB registered host block into HBM, no kernel, "
                        "median of the copies, same process after the headline")}

    kern_avg_s = st["kernel_ms"] / max(st["launches"], 1) / 1e3
    bytes_per_launch = st["bytes"] / max(st["launches"], 1)
    achieved = bytes_per_launch / kern_avg_s / 1e9 if kern_avg_s > 0 else 0.0
    traffic, traffic_src, traffic_prov = pmc_traffic(a.config, bytes_per_launch)

    rc = 0
    if rank == 0:
        value = D.aggregate_rate(1 if split else world, K, spb, el_med)
        geom_desc = (f"{paf_b2p.geometry.nchan(geom)} ch x {geom.npol} pol int{geom.nbit}"
                     + (" BE TFTFP" if geom.big_endian else ""))
        res = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": K,
            "warmup": a.warmup,
            "ms_per_step": round(el_med / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if split else "weak",
            "vs_baseline": None,
            "dtype": f"int{geom.nbit}" + ("-be" if geom.big_endian else ""),
            "data": "synthetic (counter-based SplitMix64 Gaussian, seed 20181105, sub-band = rank)",
            "verified": verified,
            "verification": vinfo or None,
            "ranks": world,
            # read back from the live process group after its first collective
            "rccl_ranks": world_seen["rccl_ranks"],
            "dist_backend": world_seen["backend"],
            "distinct_gpus": ngpu_seen,
            "rank_devices": [{k: v for k, v in i.items() if v is not None} for i in idents],
            "timed_regions": len(els_max),
            "timed_seconds": round(sum(els_max), 4),
            "ms_per_step_range": [round(min(els_max) / K * 1e3, 4), round(max(els_max) / K * 1e3, 4)],
            "ms_per_step_mean": round(statistics.fmean(els_max) / K * 1e3, 4),
            "per_rank_ms_per_step": per_rank_ms,
            # whole-job HBM read rate and its share of world x 8 TB/s
            # ("% of 8x roofline" for configs[4])
            "aggregate_hbm_gbs": round(value * 1e6 * (geom.nbit // 8) * 2 / 1e9, 1),
            "aggregate_frac_of_world_peak": round(value * 1e6 * (geom.nbit // 8) * 2 / 1e9
                                                  / (HBM_PEAK_GBS * (1 if split else world)), 4),
            "config": {
                "workload": workload_label(a.config, geom_desc, world, split, host_mode, ngpu_seen),
                "baseline_config": baseline_config(a.config, world, split),
                "nchan": int(paf_b2p.geometry.nchan(geom)),
                "npol": int(geom.npol),
                "nsamp_int": int(full_nsamp if split else geom.nsamp_int),
                "bytes_per_integration": int(bb * (world if split else 1)),
                "input": "pinned host buffer, H2D overlapped (PCIe-inclusive)" if host_mode
                         else f"HBM-resident, {len(blocks)} rotating blocks per GPU",
                "parallelism": parallelism_label(world, split, dist_on, rccl)
                + ("" if coll["op"] == "gather" else " (all_gather: the backend refused gather)"),
                "launcher": ("bench.py --gpus spawned torch.distributed.run"
                             if os.environ.get("BENCH_LAUNCHED_RANKS") else
                             ("torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process")),
                "blocks_per_launch": bpl,
                "blocks_per_launch_rule": ("set by --blocks-per-launch" if a.blocks_per_launch else
                                           "auto: floor(4 GiB / block), 1..8 -- the rule the stage "
                                           "applies to blocks queued in its input ring -- lowered to "
                                           "a divisor of --steps so every launch is the same size"),
                "launch": {"threads": it.info.threads, "columns": it.info.columns,
                           "row_groups": it.info.row_groups, "replicas": it.info.replicas,
                           "unroll": it.info.unroll, "nt_loads": bool(it.info.nontemporal)},
            },
            "roofline": {
                "bound": "hbm",
                # the instantiation rocprofv3 lists for these launches: MULTI
                # (last template argument) true when queued blocks share one
                "kernel": "b2p_integrate_kernel<..., MULTI=%s>" % ("true" if bpl > 1 else "false"),
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                # the same quantity from the line's own headline numbers: one
                # integration's algorithmic bytes per ms_per_step, per GPU
                # (each rank reads bb bytes per step; a time-split rank its share)
                "frac_of_value": round(bb / (el_med / K) / 1e9 / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_provenance": traffic_prov,
                "algorithmic_bytes_per_launch": int(bytes_per_launch),
                "avg_launch_us": round(kern_avg_s * 1e6, 2),
                # per-launch dispatch-packet events over 16 launches after the
                # timed regions: kernel duration only, as rocprofv3 counts it
                "kernel_only_us": round(calib_us, 2) if calib_us else None,
                "frac_kernel_only": (round(bytes_per_launch / (calib_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                                     if calib_us else None),
                "launches_timed": int(st["launches"]),
                "launch_phases": phases,
                "timing": ("frac: HIP events on the integrator stream bracketing each timed region's "
                           "launches, summed over the regions (region / launches: gaps and finalizes "
                           "included, the region's host bracketing not); frac_of_value: the host-timed "
                           "median region (barrier + device sync on both sides) that `value` and "
                           "`ms_per_step` come from -- the fraction that goes with `value`; "
                           "frac_kernel_only: per-launch dispatch-packet events (kernel only)"),
                "finalizes": ("carried by the next integrate launch; "
                              f"{st['finalizes']} standalone finalize launch(es) inside the regions"),
            },
            # the real-time stage launches one block at a time (blocks only
            # queue when it has fallen behind): that launch shape, timed in
            # the same run after the headline's regions, verified the same way
            "one_per_launch": one if one else (
                {"same_as_headline": True, "blocks_per_launch": 1} if bpl == 1 else None),
            "cpu_baseline": None,
            "provenance": {"kernel_sources_sha256": kernel_sources_sha(),
                           "kernel_sources": list(KERNEL_SOURCES),
                           "device_code_sha256": device_code_sha()},
        }
        if host_mode and h2d:
            # PCIe-bound: the ceiling is the bare H2D stream measured above;
            # the HBM fraction stays beside it as a secondary field
            pcie_gbs = bb / (el_med / K) / 1e9
            hbm = {k: res["roofline"][k] for k in ("achieved", "frac", "frac_of_value", "avg_launch_us",
                                                     "launches_timed", "kernel")}
            res["roofline"].update({
                "bound": "pcie",
                "achieved": round(pcie_gbs, 2),
                "peak": h2d["gbs"],
                "frac": round(pcie_gbs / h2d["gbs"], 4),
                "frac_of_value": round(pcie_gbs / h2d["gbs"], 4),
                "peak_source": h2d,
                "traffic": None,
                "traffic_source": "n/a: PCIe-bound (the kernel's HBM traffic is configs[4]'s, pmc_c5.json)",
                "hbm": {**hbm, "frac_of_8tbs": round(pcie_gbs / HBM_PEAK_GBS, 4), "peak": HBM_PEAK_GBS,
                        "note": "the block's bytes per ms_per_step against 8 TB/s (secondary)"},
                "timing": ("achieved: the block's bytes per ms_per_step (the host-timed median region: "
                           "pinned-host staging copies overlapped with the integrate launches); peak: "
                           "peak_source, the bare H2D stream of the same bytes in the same run"),
            })
        legs = [x for x in a.secondary.split(",") if x]
        if world == 1 and not split and a.config == "c2" and legs and a.secondary_seconds > 0:
            # the other BASELINE layouts and the one the drop-in serves, in the driver's own record
            res["secondary"] = {}
            for x in legs:
                try:
                    res["secondary"][x] = secondary_leg(x, dev, a.secondary_seconds, max(1, cpu_threads()),
                                                        not a.no_verify)
                except Exception as e:  # noqa: BLE001 -- the headline line still goes out, naming the leg's error
                    print(f"bench.py: secondary leg {x} failed: {type(e).__name__}: {e}", file=sys.stderr)
                    res["secondary"][x] = {"error": f"{type(e).__name__}: {e}", "verified": None}
            if any(v["verified"] is False for v in res["secondary"].values()):
                res["verified"] = verified = False
        if world == 1 and a.cpu_seconds > 0 and not host_mode:
            try:
                res["cpu_baseline"] = cpu_baseline(full_geom, a.cpu_seconds)
            except Exception as e:  # noqa: BLE001 -- the line still goes out, naming the leg's error
                print(f"bench.py: cpu_baseline failed: {type(e).__name__}: {e}", file=sys.stderr)
                res["cpu_baseline"] = {"error": f"{type(e).__name__}: {e}", "value": None}
        print(json.dumps(res), flush=True)
    if verified is False:
        print(f"bench.py: rank {rank}: spectra differ from the oracle", file=sys.stderr)
        rc = 3

    for b in blocks:
        if hasattr(b, "free"):
            b.free()
    if host_mode:
        it.unregister_host(blocks[0])
    it.close()
    if dist_on:
        dist.destroy_process_group()
    return rc


if __name__ == "__main__":
    sys.exit(main())
