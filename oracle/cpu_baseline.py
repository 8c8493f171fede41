"""oracle/cpu_baseline.py -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

Times the tuned CPU port (oracle/b2p_cpu_port.c: AVX-512 VNNI / AVX-512 /
AVX2 picked at run time, OpenMP over time tiles) -- and, beside it, the
scalar C restatement that serves as the checker (oracle/b2p_oracle.c) -- on one FULL integration
block of the bench's workload held in host RAM (no file I/O), so the passes
stream from DRAM rather than the L3 (the EPYC 9575F host has 512 MiB of L3;
a 1 GiB block does not fit).  SURVEY.md 8(d) "CPU baseline": the reference has
no CPU path, so the baseline is the port, at 1 thread and at every CPU this
process may use.  bench.py picks the CPUs (pick_cpus): one per physical core,
dealt over every L3 domain (CCD) of both NUMA nodes, listed as explicit OpenMP
places, one fewer than the cgroup quota grants, libgomp's default wait policy
(baseline_threads: threads that fill the quota exactly are throttled); every leg reports the cgroup's cpu.stat deltas (periods throttled, time throttled)
beside its median and interquartile range, so a slow box shows why.

Run as a child process of bench.py (never imported into the GPU process), so
that OpenMP reads OMP_PROC_BIND / OMP_PLACES / OMP_NUM_THREADS from an
environment set for it alone:

    python3 oracle/cpu_baseline.py '<geom json>' SECONDS SEED

and prints ONE JSON object.  Threads are bound one per OpenMP place
(OMP_PROC_BIND=close); the block is filled by the same threads first, so its
pages sit on the NUMA node of the thread that streams them.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))


def _read(path: str) -> str | None:
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _cpulist(text: str | None) -> set:
    """'0-3,8,10-11' -> {0,1,2,3,8,10,11}"""
    out = set()
    for part in (text or "").strip().split(","):
        if part:
            a, _, b = part.partition("-")
            out.update(range(int(a), int(b or a) + 1))
    return out


def cgroup_cpus() -> float | None:
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), None if
    unlimited or absent.  On the GPU box nproc shows the whole 256-CPU host
    while cpu.max grants this job 16 CPUs."""
    t = _read("/sys/fs/cgroup/cpu.max")
    try:
        q, p = t.split()[:2]
    except (AttributeError, ValueError):
        return None
    if q == "max":
        return None
    return int(q) / int(p)


def cgroup_info() -> dict:
    """the quota and the CPUs the job's cgroup lets it run on"""
    eff = _cpulist(_read("/sys/fs/cgroup/cpuset.cpus.effective"))
    return {"cpu.max": (_read("/sys/fs/cgroup/cpu.max") or "").strip() or None,
            "cpuset.cpus.effective": len(eff) or None}


def cpu_stat() -> dict:
    """cgroup v2 cpu.stat counters (usage / throttling), {} if absent"""
    out = {}
    for line in (_read("/sys/fs/cgroup/cpu.stat") or "").splitlines():
        k, _, v = line.partition(" ")
        if v.strip().isdigit():
            out[k] = int(v)
    return out


def cpu_stat_delta(before: dict, after: dict) -> dict | None:
    """what the cgroup's CPU controller did during a leg: periods, how many of
    them were throttled and for how long, CPU time used"""
    keys = ("nr_periods", "nr_throttled", "throttled_usec", "usage_usec")
    d = {k: after[k] - before[k] for k in keys if k in before and k in after}
    return d or None


def allowed_cpus() -> list:
    """logical CPUs this process may run on: its affinity, within the
    cgroup's effective cpuset when the cgroup names one"""
    cpus = set(os.sched_getaffinity(0))
    eff = _cpulist(_read("/sys/fs/cgroup/cpuset.cpus.effective"))
    if eff and cpus & eff:
        cpus &= eff
    return sorted(cpus)


def effective_cpus() -> int:
    n = len(allowed_cpus())
    q = cgroup_cpus()
    if q is not None:
        n = min(n, max(1, int(q)))
    return n


def baseline_threads() -> int:
    """threads of the timed CPU legs: every CPU the job may use, less one
    under a cgroup quota.  The quota covers the whole job (the GPU process
    that waits for this child, the HIP runtime's threads, this interpreter),
    so threads that fill it exactly are throttled -- round 4's 16 threads in
    a 16-CPU quota were throttled in 43 of 54 periods and their passes spread
    8x; at quota - 1 the job stays inside it (0 throttled periods)."""
    n = effective_cpus()
    if cgroup_cpus() is not None:
        n = min(n, max(1, int(cgroup_cpus()) - 1))
    return n


def numa_nodes() -> dict:
    """{node: set(cpu ids)} from sysfs"""
    base = "/sys/devices/system/node"
    out = {}
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                out[int(d[4:])] = _cpulist(_read(os.path.join(base, d, "cpulist")))
    except OSError:
        pass
    return out


def _idle_ticks() -> dict:
    """{cpu: (idle + iowait ticks, total ticks)} from /proc/stat"""
    out = {}
    for line in (_read("/proc/stat") or "").splitlines():
        if line.startswith("cpu") and line[3:4].isdigit():
            f = line.split()
            v = [int(x) for x in f[1:]]
            out[int(f[0][3:])] = (v[3] + (v[4] if len(v) > 4 else 0), sum(v[:8]))
    return out


def others_busy(a: dict, b: dict, mine: set) -> float | None:
    """mean busy fraction, between two /proc/stat samples, of the host's
    logical CPUs this leg did not run on: the other tenants of a shared host,
    whose memory traffic competes with a streaming pass"""
    fr = []
    for c in b:
        if c in a and c not in mine:
            dt = b[c][1] - a[c][1]
            if dt > 0:
                fr.append(1.0 - (b[c][0] - a[c][0]) / dt)
    return round(sum(fr) / len(fr), 4) if fr else None


def busy_fraction(cpus, seconds: float = 0.25) -> dict:
    """{cpu: fraction of the last `seconds` it spent busy}, from /proc/stat
    (other tenants of the host included: this job does not run meanwhile)"""
    import time
    a = _idle_ticks()
    time.sleep(seconds)
    b = _idle_ticks()
    out = {}
    for c in cpus:
        if c in a and c in b:
            dt = b[c][1] - a[c][1]
            out[c] = 1.0 - (b[c][0] - a[c][0]) / dt if dt > 0 else 0.0
    return out


def pick_cpus(n: int, sample_s: float = 0.25) -> dict:
    """n logical CPUs for the timed leg, one per physical core, dealt
    round-robin over every L3 domain (CCD) of every NUMA node, the idlest
    allowed core of each domain first (the GPU box's host is shared with other
    jobs whose threads are not confined to a cpuset).  Listed in CPU order,
    so with OMP_PROC_BIND=close the first threads sit on node 0 and the equal
    contiguous time tiles they first-touch stay on their own node.  Returns
    the CPUs, their nodes and L3 domains, and how busy they and the host were
    beforehand.

    Why every CCD of both sockets: a streaming pass is bound by each CCD's
    link to the IO die and then by each socket's DRAM, not by the cores.  On
    one GPU-box host (profiles/r04_cpu_spread.jsonl) the same 16 threads read
    77 x 10^3 Msamples/s packed into 2 CCDs, 238-240 x 10^3 dealt over the 8
    CCDs of one node and 299-305 x 10^3 over the 16 CCDs of both; round 3's
    rule (idlest cores of one node, in core order) landed on 3-6 CCDs and so
    moved between 54 and 133 x 10^3 from box to box."""
    allowed = allowed_cpus()
    busy = busy_fraction(allowed, sample_s)
    cores = {}   # (package, core) -> first allowed sibling
    for c in allowed:
        t = "/sys/devices/system/cpu/cpu%d/topology/" % c
        key = ((_read(t + "physical_package_id") or "0").strip(), (_read(t + "core_id") or str(c)).strip())
        cores.setdefault(key, c)
    reps = sorted(cores.values(), key=lambda c: (busy.get(c, 0.0), c))
    pick = spread_l3(reps, n)
    if len(pick) < n:   # fewer physical cores than threads: add SMT siblings
        pick += [c for c in sorted(allowed, key=lambda c: busy.get(c, 0.0)) if c not in pick][:n - len(pick)]
    nodes = numa_nodes()
    node_of = {c: nd for nd, cs in nodes.items() for c in cs}
    return {"cpus": sorted(pick), "nodes": sorted({node_of.get(c) for c in pick if c in node_of}),
            "l3_domains": len({l3_domain(c) for c in pick}),
            "l3_domains_allowed": len({l3_domain(c) for c in reps}),
            "busy_before": round(sum(busy.get(c, 0.0) for c in pick) / max(1, len(pick)), 4),
            "host_busy_before": round(sum(busy.values()) / max(1, len(busy)), 4),
            "sample_s": sample_s}


def l3_domain(cpu: int) -> str:
    """the L3 (on EPYC: the CCD) a logical CPU sits behind"""
    c = "/sys/devices/system/cpu/cpu%d/cache/index3/" % cpu
    return ((_read(c + "id") or "").strip() or (_read(c + "shared_cpu_list") or "").strip()
            or "cpu%d" % cpu)


def spread_l3(cores: list, n: int) -> list:
    """n of `cores` (idlest first), dealt round-robin over their L3 domains
    taken in CPU order"""
    doms = {}
    for c in cores:
        doms.setdefault(l3_domain(c), []).append(c)
    order = sorted(doms.values(), key=lambda cs: cs[0])
    pick = []
    while len(pick) < n and any(order):
        for cs in order:
            if cs and len(pick) < n:
                pick.append(cs.pop(0))
    return pick


def host_cpu() -> dict:
    model = "unknown"
    for line in (_read("/proc/cpuinfo") or "").splitlines():
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    return {"model": model, "logical_cpus": os.cpu_count(), "numa_nodes": len(numa_nodes()) or None,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpus": cgroup_cpus(),
            "cgroup": cgroup_info()}


def child_env(threads: int, places: str = "cores", wait: str = "default", cpus=None) -> dict:
    """environment of a timed child: with `cpus`, one OpenMP place per listed
    CPU (pick_cpus), else OMP_PLACES=`places` packed from the first CPU.
    wait: "default" leaves OMP_WAIT_POLICY unset (libgomp spins briefly
    between parallel regions, then sleeps), else "passive" / "active".
    On the GPU box at 15 threads in the 16-CPU quota (profiles/r05_cpu_wait.jsonl)
    the default measured 2.69-2.73 x 10^5 Msamples/s with an interquartile
    range within -8.6 / +4.9 % and no throttled period, passive 2.33-2.49 x
    10^5 (within +-3.6 %), active 2.57-2.71 x 10^5 (within -9.0 / +4.5 %)."""
    env = dict(os.environ)
    if cpus:
        places = ",".join("{%d}" % c for c in cpus[:threads])
    env.update(OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES=places)
    if wait == "default":
        env.pop("OMP_WAIT_POLICY", None)
    else:
        env["OMP_WAIT_POLICY"] = wait
    return env


def throttled_frac(delta: dict | None) -> float | None:
    """share of the leg's cgroup periods in which the job was throttled"""
    if not delta or not delta.get("nr_periods"):
        return None
    return round(delta.get("nr_throttled", 0) / delta["nr_periods"], 4)


def _quartiles(xs):
    q = statistics.quantiles(xs, n=4, method="inclusive") if len(xs) >= 2 else [xs[0]] * 3
    return [round(q[0], 2), round(q[2], 2)]


def run(geom: dict, seconds: float, seed: int, one_thread: bool = True, isa: str = "auto") -> dict:
    sys.path.insert(0, _HERE)
    import numpy as np

    import b2p_oracle as npo
    import oracle_c as co

    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    host = host_cpu()  # before OpenMP binds this thread to its first place
    pl = os.environ.get("OMP_PLACES", "")
    first = int(pl[1:pl.index("}")]) if pl.startswith("{") else min(os.sched_getaffinity(0))
    places = [int(x.strip("{}")) for x in pl.split(",")] if pl.startswith("{") else [first]
    g = npo.Geom(**geom)
    buf = np.empty(g.block_bytes, dtype=np.uint8)
    co.fill_synthetic(g, g.block_bytes, seed, 0, 0, out=buf)   # first touch by the bound threads
    per_pass = g.block_bytes // g.word_bytes * g.npol          # complex samples in the block

    def port(nt):
        return co.port_integrate(g, buf, nthreads=nt, isa=isa)

    def oracle(nt):
        return co.integrate(g, buf, nthreads=nt)

    def timed(fn, nt: int, budget: float, min_passes: int = 3):
        warm = buf[: g.frame_bytes * max(1, (64 << 20) // g.frame_bytes)]
        (co.integrate(g, warm, nthreads=nt) if fn is oracle
         else co.port_integrate(g, warm, nthreads=nt, isa=isa))
        st0, tk0 = cpu_stat(), _idle_ticks()
        rates, t_all = [], time.perf_counter()
        while len(rates) < min_passes or time.perf_counter() - t_all < budget:
            t0 = time.perf_counter()
            fn(nt)
            rates.append(per_pass / (time.perf_counter() - t0) / 1e6)
            if len(rates) >= 10000:
                break
        d = cpu_stat_delta(st0, cpu_stat()) or {}
        d["others_busy"] = others_busy(tk0, _idle_ticks(), set(places[:nt]))
        return rates, time.perf_counter() - t_all, d

    def leg(rates, el, thr):
        return {"value": round(statistics.median(rates), 2), "passes": len(rates), "seconds": round(el, 2),
                "iqr": _quartiles(rates), "passes_range": [round(min(rates), 2), round(max(rates), 2)],
                "cgroup_cpu_stat_delta": thr, "throttled_frac": throttled_frac(thr)}

    used = co.port_isa(isa)
    binding = (f"OMP_PLACES={os.environ.get('OMP_PLACES')} OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')} "
               f"OMP_WAIT_POLICY={os.environ.get('OMP_WAIT_POLICY')}")
    if not one_thread:  # one setting only (bench.py's every-logical-CPU leg)
        r_n, el_n, thr_n = timed(port, threads, seconds)
        return {"threads": threads, **leg(r_n, el_n, thr_n), "isa": used, "binding": binding}
    r_n, el_n, thr_n = timed(port, threads, seconds * 0.6)
    # the 1-thread leg streams a copy first-touched by that thread (the main
    # thread, bound to the first place): the block's own pages are spread
    # over both nodes by the threads that filled it, and half of them would
    # be remote to one thread
    buf1 = np.empty_like(buf)
    np.copyto(buf1, buf)

    def port1(nt):
        return co.port_integrate(g, buf1, nthreads=nt, isa=isa)
    r_1, el_1, thr_1 = timed(port1, 1, seconds * 0.25)
    del buf1
    r_o, el_o, _ = timed(oracle, threads, seconds * 0.15)
    # the port is a baseline, not the checker: its sums must equal the oracle's
    equal = bool(np.array_equal(port(threads), oracle(threads)))
    nodes = numa_nodes()
    used_nodes = sorted({n for n, c in nodes.items() for p in places if p in c})
    ln = leg(r_n, el_n, thr_n)
    quota = host.get("cgroup_cpus")
    return {
        "value": ln["value"], "unit": "Msamples/s", "cores": threads,
        # what `cores` is: the job's CPU share of a shared host, not the host
        "cores_scope": (f"{threads} threads = this job's cgroup CPU quota ({quota:g} CPUs, cpu.max) less one, "
                        f"on a {host.get('logical_cpus')}-logical-CPU host shared with other jobs: the "
                        "baseline is bound by the quota, not by the host's cores" if quota else
                        f"{threads} threads: every CPU this process may use, less one (no cgroup quota)"),
        "kind": "port",          # the contract's two kinds: "reference" | "port"
        "port": "tuned (oracle/b2p_cpu_port.c), not the scalar checker",
        "isa": used,
        "sample": (f"tuned port ({used}, OpenMP time tiles): {len(r_n)} passes ({el_n:.1f} s) at "
                   f"{threads} threads and {len(r_1)} passes ({el_1:.1f} s) at 1 thread over one "
                   f"full {g.block_bytes >> 20} MiB {g.nchan}-chan int{g.nbit} integration block "
                   "in host RAM (no file I/O); value = median pass"),
        "iqr": ln["iqr"],
        "passes_range": ln["passes_range"],
        "passes": ln["passes"],
        "leg_seconds": ln["seconds"],
        "cgroup_cpu_stat_delta": thr_n,
        # periods of the quota in which the job was throttled during the leg,
        # and the interquartile range relative to the median
        "throttled_frac": throttled_frac(thr_n),
        "iqr_rel": [round(q / ln["value"] - 1, 4) for q in ln["iqr"]] if ln["value"] else None,
        "value_1thread": round(statistics.median(r_1), 2),
        "iqr_1thread": _quartiles(r_1),
        "cgroup_cpu_stat_delta_1thread": thr_1,
        "equals_oracle": equal,
        "oracle_value": round(statistics.median(r_o), 2),
        "oracle": (f"scalar C restatement (the checker, oracle/b2p_oracle.c): {len(r_o)} passes "
                   f"({el_o:.1f} s) at {threads} threads, median"),
        "numa": {"nodes": used_nodes, "binding": binding + "; block first-touched by the same threads "
                 "(equal contiguous tiles, the split the passes use)"},
        "host": host,
    }


if __name__ == "__main__":
    geom = json.loads(sys.argv[1])
    one = not (len(sys.argv) > 4 and sys.argv[4] == "only")
    isa = sys.argv[5] if len(sys.argv) > 5 else "auto"
    print(json.dumps(run(geom, float(sys.argv[2]), int(sys.argv[3]), one_thread=one, isa=isa)),
          flush=True)
