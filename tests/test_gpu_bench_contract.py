"""bench.py keeps the driver's contract: one JSON line on stdout with the
required keys, a roofline object for the integrate kernel and a CPU
baseline object (BASELINE.json metric, configs[1] workload)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def test_bench_prints_one_contract_line(gpu):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "4", "--warmup", "1",
                        "--cpu-seconds", "1", "--min-seconds", "0.05", "--bpl1-seconds", "0.2"],
                       capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["vs_baseline"] is None
    assert d["config"]["baseline_config"] == "configs[1]" and "workload" in d["config"]
    rf = d["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    # the kernel alone (per-launch packet events, >= 16 launches) is never
    # slower than the region average it sits inside
    assert rf["kernel_only_us"] > 0 and rf["frac_kernel_only"] >= rf["frac"] * 0.97
    assert rf["traffic"] is None or rf["traffic"] > 0
    # the fraction that goes with `value`: the headline's own numbers
    per_int = d["config"]["bytes_per_integration"]
    assert abs(rf["frac_of_value"] - per_int / (d["ms_per_step"] * 1e-3) / 1e9 / 8000.0) < 2e-3
    assert 0.5 * rf["frac"] < rf["frac_of_value"] <= rf["frac"] * 1.01
    assert rf["traffic_provenance"] is None or "stale" in rf["traffic_provenance"]
    assert len(d["provenance"]["kernel_sources_sha256"]) == 64
    # 4 queued 1 GiB blocks per launch in the headline; the real-time shape
    # (one per launch) timed and verified beside it
    assert d["config"]["blocks_per_launch"] == 4
    one = d["one_per_launch"]
    assert one["blocks_per_launch"] == 1 and one["verified"] is True and one["value"] > 0
    assert one["timed_regions"] >= 1 and 0.3 < one["frac_of_value"] < 1.0
    cb = d["cpu_baseline"]
    assert cb["unit"] == d["unit"] and cb["kind"] == "port" and cb["port"].startswith("tuned") and cb["cores"] >= 1
    assert d["value"] > 0 and cb["value"] > 0 and cb["value_1thread"] > 0
    assert cb["equals_oracle"] is True and cb["oracle_value"] > 0
    lo, hi = cb["iqr"]
    assert cb["passes_range"][0] <= lo <= cb["value"] <= hi <= cb["passes_range"][1]
    assert len(cb["cpus_picked"]["cpus"]) == cb["cores"] and "cgroup_cpu_stat_delta" in cb
    assert cb["isa"] in ("avx512vnni", "avx512bw", "avx2", "scalar")
    # the ranks that ran, read back from the process (no group at N = 1)
    assert d["rccl_ranks"] == 0 and d["distinct_gpus"] == 1
    rd = d["rank_devices"]
    assert len(rd) == 1 and rd[0]["rank"] == 0 and rd[0]["pci_bus_id"].count(":") == 2
    assert d["verified"] is True and d["ranks"] == 1 and d["timed_regions"] >= 1
    lo, hi = d["ms_per_step_range"]
    assert lo <= d["ms_per_step"] <= hi


def test_bench_blocks_per_launch(gpu):
    """--blocks-per-launch 4: queued HBM blocks in one b2p_integrate_n launch;
    still one spectrum per step (10 steps: two launches of 4 and one of 2),
    every one verified against the oracle; the roofline is per launch"""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "10", "--warmup", "1",
                        "--cpu-seconds", "0", "--min-seconds", "0.05", "--blocks-per-launch", "4"],
                       capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert d["verified"] is True and d["steps"] == 10
    assert d["config"]["blocks_per_launch"] == 4
    rf = d["roofline"]
    per_block = d["config"]["bytes_per_integration"]
    assert 3 * per_block < rf["algorithmic_bytes_per_launch"] < 4 * per_block  # (4+4+2)/3 blocks
    assert rf["launches_timed"] % 3 == 0


def test_bench_gpus2_gloo_spawns_two_ranks(gpu):
    """`bench.py --gpus 2` with no external launcher starts two ranks itself
    (gloo: both share the box's one GPU) and reports them"""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--dist-backend", "gloo", "--min-seconds", "0.02"],
                       capture_output=True, text=True, timeout=600, cwd=REPO,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["ranks"] == 2 and d["rccl_ranks"] == 0
    assert d["verified"] is True and d["verification"]["gather"].startswith("rank 0 holds")
    w = d["config"]["workload"]
    assert "2 ranks sharing 1 MI355X" in w or "over 2 MI355X" in w   # 1 or >= 2 GPUs visible
    assert d["config"]["launcher"].startswith("bench.py --gpus")
    assert len(d["per_rank_ms_per_step"]) == 2 and d["cpu_baseline"] is None
    assert d["dist_backend"] == "gloo" and [x["rank"] for x in d["rank_devices"]] == [0, 1]


def test_configs3_four_rank_rehearsal_full_size(gpu):
    """configs[3] as the driver's 4-GPU run would do it, rehearsed with gloo:
    4 ranks, each integrating full 1 GiB 256-ch int8 blocks of its own
    sub-band (4 distinct blocks per rank, 16 GiB in all), the K spectra of
    every rank gathered to rank 0, every spectrum checked against the C
    oracle.  The ranks share this box's GPU, so the rate means nothing; the
    plumbing (launcher, world check, watchdog, identities, gather,
    verification) is what runs."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "4",
                        "--warmup", "1", "--dist-backend", "gloo", "--min-seconds", "0",
                        "--dist-timeout", "120"],
                       capture_output=True, text=True, timeout=600, cwd=REPO,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 4 and d["ranks"] == 4 and d["verified"] is True
    assert d["config"]["bytes_per_integration"] == 1 << 30 and d["config"]["nchan"] == 256
    assert "configs[3]" in d["config"]["baseline_config"]
    assert d["verification"]["gather"].startswith("rank 0 holds")
    assert "4 distinct block" in d["verification"]["what"]
    assert [x["rank"] for x in d["rank_devices"]] == [0, 1, 2, 3]
    assert d["distinct_gpus"] >= 1 and d["dist_backend"] == "gloo" and d["rccl_ranks"] == 0


def test_configs4_eight_subbands_full_size(gpu):
    """configs[4] as the driver's 8-GPU run would do it, rehearsed with gloo
    on this box's one GPU: 8 ranks, each integrating full 4 GiB blocks of
    1024 ch x 2 pol int8 of its own sub-band (2 distinct blocks per rank, 64
    GiB in HBM), the spectra of every rank gathered to rank 0 and every one
    checked against the C oracle (BASELINE.json configs[4]; SURVEY 8d C5,
    8e).  The ranks share one GPU, so the rate is not a scaling figure."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "c5", "--gpus", "8",
                        "--dist-backend", "gloo", "--steps", "2", "--warmup", "1", "--min-seconds", "0",
                        "--cpu-seconds", "0", "--blocks", "2", "--dist-timeout", "240"],
                       capture_output=True, text=True, timeout=900, cwd=REPO,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK")})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["verified"] is True and d["n_gpus"] == 8 and d["ranks"] == 8
    assert d["config"]["baseline_config"] == "configs[4]"
    assert d["config"]["bytes_per_integration"] == 1 << 32 and d["config"]["nchan"] == 1024
    assert d["config"]["input"].startswith("HBM-resident, 2 rotating blocks")
    assert [x["rank"] for x in d["rank_devices"]] == list(range(8))
    assert d["distinct_gpus"] >= 1 and d["dist_backend"] == "gloo"
    assert d["verification"]["gather"] == "rank 0 holds every rank's K spectra"
    assert "2 distinct block" in d["verification"]["what"]
    assert len(d["per_rank_ms_per_step"]) == 8


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("split", ["subband", "time"])
def test_bench_rccl_world1_under_torchrun(gpu, split):
    """The driver's multi-GPU launch shape, torch.distributed.run + bench.py,
    with the RCCL ("nccl") group forced at world size 1 (--force-dist): the
    communicator set-up, the gather of the spectra to rank 0 (or, time split,
    the exact uint64 reduce of the partial sums), the identity all_gather,
    the max-over-ranks all_reduce and the barriers all run over RCCL, and the
    spectra are verified against the oracle.  RCCL refuses two ranks on one
    GPU, so world 1 is as far as a one-GPU box takes this path."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--steps", "8", "--warmup", "2", "--cpu-seconds", "0",
           "--min-seconds", "0.2", "--bpl1-seconds", "0.1", "--force-dist", "--dist-timeout", "180"]
    if split == "time":
        cmd += ["--split", "time"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=500, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["dist_backend"] == "nccl" and d["rccl_ranks"] == 1 and d["ranks"] == 1
    assert d["config"]["launcher"] == "torch.distributed.run"
    assert d["verified"] is True and d["distinct_gpus"] == 1
    assert [x["rank"] for x in d["rank_devices"]] == [0]
    if split == "time":
        assert d["scaling"] == "strong" and d["config"]["blocks_per_launch"] == 1
    else:
        assert d["verification"]["gather"] == "rank 0 holds every rank's K spectra"
        assert d["config"]["blocks_per_launch"] == 4 and d["one_per_launch"]["verified"] is True
