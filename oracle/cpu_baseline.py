"""oracle/cpu_baseline.py -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).

Times the tuned CPU port (oracle/b2p_cpu_port.c: AVX-512 VNNI / AVX-512 /
AVX2 picked at run time, OpenMP over time tiles) -- and, beside it, the
scalar C restatement that serves as the checker (oracle/b2p_oracle.c) -- on one FULL integration
block of the bench's workload held in host RAM (no file I/O), so the passes
stream from DRAM rather than the L3 (the EPYC 9575F host has 512 MiB of L3;
a 1 GiB block does not fit).  SURVEY.md 8(d) "CPU baseline": the reference has
no CPU path, so the baseline is the port, at 1 thread and at every CPU this
process may use.

Run as a child process of bench.py (never imported into the GPU process), so
that OpenMP reads OMP_PROC_BIND / OMP_PLACES / OMP_NUM_THREADS from an
environment set for it alone:

    python3 oracle/cpu_baseline.py '<geom json>' SECONDS SEED

and prints ONE JSON object.  Threads are bound one per physical core, packed
from core 0 (OMP_PLACES=cores, OMP_PROC_BIND=close); the block is filled by the
same threads first, so its pages sit on the NUMA node those cores belong to.
"""
from __future__ import annotations

import json
import os
import statistics
import sys
import time

_HERE = os.path.dirname(os.path.abspath(__file__))


def cgroup_cpus() -> float | None:
    """CPUs granted by the cgroup v2 quota (cpu.max "quota period"), None if
    unlimited or absent.  On the GPU box nproc shows the whole 256-CPU host
    while cpu.max grants this job 16 CPUs."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
    except (OSError, ValueError):
        return None
    if q == "max":
        return None
    return int(q) / int(p)


def effective_cpus() -> int:
    n = len(os.sched_getaffinity(0))
    q = cgroup_cpus()
    if q is not None:
        n = min(n, max(1, int(q)))
    return n


def numa_nodes() -> dict:
    """{node: set(cpu ids)} from sysfs"""
    base = "/sys/devices/system/node"
    out = {}
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                cpus = set()
                for part in open(os.path.join(base, d, "cpulist")).read().strip().split(","):
                    if not part:
                        continue
                    a, _, b = part.partition("-")
                    cpus.update(range(int(a), int(b or a) + 1))
                out[int(d[4:])] = cpus
    except OSError:
        pass
    return out


def host_cpu() -> dict:
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "numa_nodes": len(numa_nodes()) or None,
            "affinity_cpus": len(os.sched_getaffinity(0)), "cgroup_cpus": cgroup_cpus()}


def child_env(threads: int, places: str = "cores", wait: str = "active") -> dict:
    env = dict(os.environ)
    env.update(OMP_NUM_THREADS=str(threads), OMP_PROC_BIND="close", OMP_PLACES=places,
               OMP_WAIT_POLICY=wait)
    return env


def run(geom: dict, seconds: float, seed: int, one_thread: bool = True, isa: str = "auto") -> dict:
    sys.path.insert(0, _HERE)
    import numpy as np

    import b2p_oracle as npo
    import oracle_c as co

    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    host = host_cpu()  # before OpenMP binds this thread to its first place
    first = min(os.sched_getaffinity(0))
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
        (co.port_integrate(g, warm, nthreads=nt, isa=isa) if fn is port
         else co.integrate(g, warm, nthreads=nt))
        rates, t_all = [], time.perf_counter()
        while len(rates) < min_passes or time.perf_counter() - t_all < budget:
            t0 = time.perf_counter()
            fn(nt)
            rates.append(per_pass / (time.perf_counter() - t0) / 1e6)
            if len(rates) >= 10000:
                break
        return rates, time.perf_counter() - t_all

    used = co.port_isa(isa)
    if not one_thread:  # one setting only (bench.py's every-logical-CPU leg)
        r_n, el_n = timed(port, threads, seconds)
        return {"threads": threads, "value": round(statistics.median(r_n), 2), "passes": len(r_n),
                "passes_range": [round(min(r_n), 2), round(max(r_n), 2)], "isa": used,
                "binding": f"OMP_PLACES={os.environ.get('OMP_PLACES')} "
                           f"OMP_WAIT_POLICY={os.environ.get('OMP_WAIT_POLICY')}"}
    r_n, el_n = timed(port, threads, seconds * 0.55)
    r_1, el_1 = timed(port, 1, seconds * 0.25)
    r_o, el_o = timed(oracle, threads, seconds * 0.2)
    # the port is a baseline, not the checker: its sums must equal the oracle's
    equal = bool(np.array_equal(port(threads), oracle(threads)))
    nodes = numa_nodes()
    node = next((n for n, c in nodes.items() if first in c), None)
    return {
        "value": round(statistics.median(r_n), 2), "unit": "Msamples/s", "cores": threads,
        "kind": "port-tuned",
        "isa": used,
        "sample": (f"tuned port ({used}, OpenMP time tiles): {len(r_n)} passes ({el_n:.1f} s) at "
                   f"{threads} threads and {len(r_1)} passes ({el_1:.1f} s) at 1 thread over one "
                   f"full {g.block_bytes >> 20} MiB {g.nchan}-chan int{g.nbit} integration block "
                   "in host RAM (no file I/O); value = median pass"),
        "value_1thread": round(statistics.median(r_1), 2),
        "passes_range": [round(min(r_n), 2), round(max(r_n), 2)],
        "equals_oracle": equal,
        "oracle_value": round(statistics.median(r_o), 2),
        "oracle": (f"scalar C restatement (the checker, oracle/b2p_oracle.c): {len(r_o)} passes "
                   f"({el_o:.1f} s) at {threads} threads, median"),
        "numa": {"node": node, "binding": "OMP_PLACES=cores OMP_PROC_BIND=close, packed from the "
                                          "first allowed CPU; block first-touched by the same threads"},
        "host": host,
    }


if __name__ == "__main__":
    geom = json.loads(sys.argv[1])
    one = not (len(sys.argv) > 4 and sys.argv[4] == "only")
    isa = sys.argv[5] if len(sys.argv) > 5 else "auto"
    print(json.dumps(run(geom, float(sys.argv[2]), int(sys.argv[3]), one_thread=one, isa=isa)),
          flush=True)
