"""Multi-GPU plumbing: one process per GPU, one sub-band per process.

SURVEY.md 8e: independent DADA sub-bands shard with no exchange during the
integrate; the only collective is the final gather of the per-channel
power spectra to rank 0 (RCCL over xGMI with the "nccl" backend on ROCm;
gloo in the CPU tests).  Spectra are a few KiB, so the gather is
latency-bound; it is issued once per batch of integrations, not per block.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_ranks() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from torch.distributed.run's env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def subband_of(rank: int) -> int:
    """sub-band r lives on rank / GPU r (ring key base + 0x10 r in the pipeline)"""
    return rank


def init(backend: str, local_rank: int) -> None:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend)


def gather_spectra(local: torch.Tensor) -> list[torch.Tensor] | None:
    """All ranks' [K, nout] spectra, in rank (= sub-band) order, on rank 0;
    None elsewhere.  all_gather (supported by both RCCL and gloo) into
    preallocated buffers; rank 0 keeps them."""
    world = dist.get_world_size()
    bufs = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(bufs, local.contiguous())
    return bufs if dist.get_rank() == 0 else None


def max_over_ranks(x: float, device: str = "cpu") -> float:
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_rate(n_ranks: int, steps: int, samples_per_step: int, seconds_max: float) -> float:
    """whole-job Msamples/s: every rank's samples over the slowest rank's time"""
    return n_ranks * steps * samples_per_step / seconds_max / 1e6
