"""Multi-GPU plumbing: one process per GPU.

SURVEY.md 8e, two modes:

* sub-band sharding (default): independent DADA sub-bands, one per rank,
  with no exchange during the integrate; the only collective is the final
  gather of the per-channel power spectra to rank 0.
* time split: ONE sub-band's integration is cut along time into one share
  per rank; each rank emits exact uint64 partial sums and rank 0 receives
  their total through a reduce (SUM), then rounds once to fp32, so the
  result is bit-identical to one GPU's.

RCCL over xGMI with the "nccl" backend on ROCm; gloo in the CPU tests.
Spectra and partials are a few KiB, so the collectives are latency-bound;
each is issued once per batch of integrations, not per block.
"""
from __future__ import annotations

import datetime
import os
import sys
import threading

import torch
import torch.distributed as dist

# How long one multi-rank phase may take before the rank gives up: the
# rendezvous, a communicator's first collective (RCCL sets up its channels
# there), one timed region.  Seconds; bench.py --dist-timeout overrides.
DEFAULT_TIMEOUT_S = 300.0
WATCHDOG_EXIT = 4


class Watchdog:
    """Bounds each multi-rank phase.  A rank stuck in a rendezvous or inside
    an RCCL call cannot be unwound from Python, so when a phase outlives its
    limit the rank names the phase on stderr and leaves with exit code 4
    (os._exit; torch.distributed.run then stops the other ranks).  This
    turns "the first 8-rank RCCL run hangs until the driver's limit" into a
    bounded, labelled failure."""

    def __init__(self, rank: int, limit_s: float, exit_code: int = WATCHDOG_EXIT, out=None):
        self.rank, self.limit_s, self.exit_code = rank, float(limit_s), exit_code
        self.out = out or sys.stderr
        self._timer = None
        self.phase_name = None

    def _expire(self, name: str, limit: float) -> None:
        print(f"bench.py: rank {self.rank}: {name} did not finish within {limit:g} s "
              f"(stuck rendezvous or collective); exiting {self.exit_code}", file=self.out, flush=True)
        os._exit(self.exit_code)

    def arm(self, name: str, limit_s: float | None = None) -> None:
        self.disarm()
        limit = self.limit_s if limit_s is None else float(limit_s)
        self.phase_name = name
        self._timer = threading.Timer(limit, self._expire, args=(name, limit))
        self._timer.daemon = True
        self._timer.start()

    def disarm(self) -> None:
        if self._timer is not None:
            self._timer.cancel()
            self._timer = None
        self.phase_name = None

    def phase(self, name: str, limit_s: float | None = None):
        wd = self

        class _P:
            def __enter__(self_):
                wd.arm(name, limit_s)

            def __exit__(self_, *exc):
                wd.disarm()
        return _P()


def env_ranks() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torch.distributed.run's env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def subband_of(rank: int) -> int:
    """sub-band r lives on rank / GPU r (ring key base + 0x10 r in the pipeline)"""
    return rank


def device_of(local_rank: int) -> int:
    """GPU of a local rank: rank r on GPU r when every GPU is visible; when a
    launcher gives each process fewer devices (one visible GPU), wrap
    (paf_baseband2power.cu:89-90 uses index 0 with one GPU)."""
    n = torch.cuda.device_count()  # does not initialise HIP
    return local_rank % n if n > 0 else 0


def init(backend: str, local_rank: int, timeout_s: float = DEFAULT_TIMEOUT_S) -> None:
    """init_process_group with an explicit timeout: it bounds the TCP-store
    rendezvous and, for "nccl" (RCCL), every collective (torch's watchdog
    aborts the communicator past it).  The eager RCCL set-up that device_id
    starts is bounded by the caller's Watchdog."""
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    td = datetime.timedelta(seconds=timeout_s)
    if backend == "nccl":
        dev = device_of(local_rank)
        torch.cuda.set_device(dev)
        dist.init_process_group("nccl", device_id=torch.device("cuda", dev), timeout=td)
    else:
        dist.init_process_group(backend, timeout=td)


def observed_world() -> dict:
    """what the live process group is, read back after its first collective
    (not what was asked for): backend, size, and RCCL ranks"""
    if not dist.is_initialized():
        return {"backend": None, "world_size": 1, "rccl_ranks": 0}
    be = str(dist.get_backend())
    n = dist.get_world_size()
    return {"backend": be, "world_size": n, "rccl_ranks": n if be == "nccl" else 0}


def gather_identities(ident: dict) -> list[dict]:
    """every rank's identity record (rank, host, device, PCI bus id ...), in
    rank order, on every rank"""
    if not dist.is_initialized():
        return [ident]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, ident)
    return out


def distinct_gpus(idents: list[dict]) -> int:
    """physical GPUs behind the ranks: distinct (host, PCI bus id) pairs"""
    return len({(i.get("host"), i.get("pci_bus_id")) for i in idents})


def gather_spectra(local: torch.Tensor) -> list[torch.Tensor] | None:
    """All ranks' [K, nout] spectra, in rank (= sub-band) order, on rank 0;
    None elsewhere.  A gather to rank 0 (configs[3]: "RCCL gather of
    per-channel power to rank 0"; ncclGather, rccl.h:745): peers send and
    receive nothing back."""
    world = dist.get_world_size()
    if dist.get_rank() == 0:
        bufs = [torch.empty_like(local) for _ in range(world)]
        dist.gather(local.contiguous(), gather_list=bufs, dst=0)
        return bufs
    dist.gather(local.contiguous(), dst=0)
    return None


def all_gather_spectra(local: torch.Tensor) -> list[torch.Tensor] | None:
    """gather_spectra through all_gather, for a backend that refuses gather:
    rank 0 keeps every rank's spectra, the peers drop theirs"""
    world = dist.get_world_size()
    bufs = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(bufs, local.contiguous())
    return bufs if dist.get_rank() == 0 else None


def time_share(rank: int, world: int, nframes: int) -> tuple[int, int]:
    """(first frame, frames) of rank's share of an nframes integration: the
    time axis is cut into world equal contiguous shares."""
    if world < 1 or nframes % world:
        raise ValueError(f"{nframes} frames do not split into {world} equal shares")
    n = nframes // world
    return rank * n, n


def reduce_sums(local: torch.Tensor) -> torch.Tensor | None:
    """Sum of every rank's [K, nout] exact partial sums on rank 0 (None
    elsewhere).  The sums are uint64 bit patterns held as int64: totals stay
    below 2**53, so the signed add is the exact one."""
    if local.dtype != torch.int64:
        raise TypeError("partial sums travel as int64")
    t = local.contiguous().clone()
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    return t if dist.get_rank() == 0 else None


def max_over_ranks(x: float, device: str = "cpu") -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(n_ranks: int, steps: int, samples_per_step: int, seconds_max: float) -> float:
    """whole-job Msamples/s: every rank's samples over the slowest rank's time"""
    return n_ranks * steps * samples_per_step / seconds_max / 1e6
