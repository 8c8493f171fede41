"""bench.py's rank plumbing, on CPU (no GPU is touched):

* `--gpus N` without a launcher starts N ranks through torch.distributed.run
  as a child (never exec), with the same arguments;
* a launched rank whose WORLD_SIZE differs from --gpus refuses (exit 2)
  before anything touches the GPU;
* RCCL with fewer visible GPUs than ranks refuses rather than stacking ranks
  on one device;
* the labels name the world size actually running.
"""
import os
import subprocess
import sys
import textwrap

import pytest

from conftest import REPO

sys.path.insert(0, REPO)
import bench  # noqa: E402


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=300, cwd=REPO)


def test_world_mismatch_refused_before_gpu():
    r = _run(["--gpus", "8", "--steps", "2"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2 but --gpus 8" in r.stderr
    assert r.stdout.strip() == ""


def test_rccl_needs_one_gpu_per_rank(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "visible_gpus", lambda: 1)
    called = []
    monkeypatch.setattr(bench.subprocess, "run", lambda *a, **k: called.append(a))
    a = bench.parse(["--gpus", "2"])
    assert bench.launch_ranks(a, ["--gpus", "2"]) == 2
    assert called == []            # nothing was started


def test_launcher_passes_arguments_through(monkeypatch):
    seen = {}

    class R:
        returncode = 0

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return R()

    monkeypatch.setattr(bench, "visible_gpus", lambda: 8)
    monkeypatch.setattr(bench.subprocess, "run", fake_run)
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5", "--config", "c5"]
    assert bench.launch_ranks(bench.parse(argv), argv) == 0
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-len(argv) - 1:] == [os.path.join(REPO, "bench.py"), *argv]
    assert seen["env"]["BENCH_LAUNCHED_RANKS"] == "8"
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_launcher_really_starts_n_ranks(monkeypatch, tmp_path):
    """the same torch.distributed.run line, pointed at a probe script, starts
    N ranks that see WORLD_SIZE == N (gloo-free: no rendezvous beyond the
    launcher's own)"""
    probe = tmp_path / "probe.py"
    out = tmp_path / "ranks"
    out.mkdir()
    probe.write_text(textwrap.dedent(f"""
        import os
        open(os.path.join({str(out)!r}, os.environ["RANK"]), "w").write(
            os.environ["WORLD_SIZE"] + " " + os.environ.get("BENCH_LAUNCHED_RANKS", ""))
    """))
    real = bench.launcher_cmd

    def cmd_for_probe(a, argv, port):
        c = real(a, argv, port)
        i = c.index(os.path.abspath(bench.__file__))
        return c[:i] + [str(probe)]

    monkeypatch.setattr(bench, "launcher_cmd", cmd_for_probe)
    a = bench.parse(["--gpus", "3", "--dist-backend", "gloo"])
    assert bench.launch_ranks(a, []) == 0
    got = {p: (out / p).read_text() for p in os.listdir(out)}
    assert got == {"0": "3 3", "1": "3 3", "2": "3 3"}


@pytest.mark.parametrize("world,split", [(1, False), (2, False), (8, False), (4, True)])
def test_labels_follow_world(world, split):
    w = bench.workload_label("c5", "1024 ch x 2 pol int8", world, split, False)
    p = bench.parallelism_label(world, split, world > 1, True)
    assert f"over {world} MI355X" in w
    assert f"x{world}" in p
    if world == 1 and not split:
        assert "gathered" not in w
    if world > 1 and not split:
        assert "gather of spectra to rank 0" in p


def test_label_of_ranks_sharing_a_gpu():
    w = bench.workload_label("c2", "256 ch x 2 pol int8", 8, False, False, ndev=1)
    assert "8 ranks sharing 1 MI355X (rehearsal" in w and "1 per MI355X" not in w
    assert "over 8 MI355X" in bench.workload_label("c2", "x", 8, False, False, ndev=8)


def test_bad_counts_rejected():
    for args in (["--gpus", "0"], ["--steps", "0"]):
        r = _run(args)
        assert r.returncode == 2 and "must be >= 1" in r.stderr


def test_pmc_traffic_follows_the_launch_size():
    """the committed PMC summary (profiles/pmc_c2.json) scales to this run's
    bytes per launch; the measured launch size itself is taken as is"""
    import json
    d = json.load(open(os.path.join(REPO, "profiles", "pmc_c2.json")))
    alg, hbm = d["algorithmic_bytes_per_launch"], d["hbm_bytes_per_launch"]
    t, src, prov = bench.pmc_traffic("c2", alg)
    assert t == hbm and src.startswith("profiles/pmc_c2.json")
    t1, src1, _ = bench.pmc_traffic("c2", 1 << 30)
    assert abs(t1 / (1 << 30) - hbm / alg) < 1e-6 and "scaled to 1073741824 B" in src1
    assert 1.0 <= hbm / alg < 1.01          # no wasted re-reads
    assert bench.pmc_traffic("no_such_config", 1 << 30) == (None, None, None)
    # provenance: the summary names the kernel sources it was measured on
    if "kernel_sources_sha256" in d:
        assert prov["stale"] == (d["kernel_sources_sha256"] != bench.kernel_sources_sha())
        assert ("STALE" in src) == prov["stale"]


def test_pmc_traffic_is_marked_stale_when_kernel_sources_change(tmp_path, monkeypatch):
    """a PMC summary stamped with other kernel sources' sha256 is quoted as
    STALE; one stamped with today's is not"""
    import json
    prof = tmp_path / "profiles"
    prof.mkdir()
    base = {"hbm_bytes_per_launch": 1074, "algorithmic_bytes_per_launch": 1073, "commit": "abc"}
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    for f in bench.KERNEL_SOURCES:   # a copy of today's sources under the fake repo
        (tmp_path / f).parent.mkdir(parents=True, exist_ok=True)
        (tmp_path / f).write_bytes(open(os.path.join(REPO, f), "rb").read())
    sha = bench.kernel_sources_sha()
    (prof / "pmc_c2.json").write_text(json.dumps({**base, "kernel_sources_sha256": sha}))
    t, src, prov = bench.pmc_traffic("c2", 1073)
    assert t == 1074 and prov["stale"] is False and "STALE" not in src and prov["measured_commit"] == "abc"
    (prof / "pmc_c2.json").write_text(json.dumps({**base, "kernel_sources_sha256": "0" * 64}))
    t, src, prov = bench.pmc_traffic("c2", 1073)
    assert prov["stale"] is True and "STALE" in src
    (tmp_path / bench.KERNEL_SOURCES[0]).write_bytes(b"// edited\n")
    (prof / "pmc_c2.json").write_text(json.dumps({**base, "kernel_sources_sha256": sha}))
    assert bench.pmc_traffic("c2", 1073)[2]["stale"] is True
    (prof / "pmc_c2.json").write_text(json.dumps(base))     # unstamped: freshness unknown
    assert bench.pmc_traffic("c2", 1073)[2]["stale"] is None


def test_baseline_config_names():
    assert bench.baseline_config("c2", 1, False) == "configs[1]"
    assert bench.baseline_config("c2", 4, False) == "configs[3]"
    assert bench.baseline_config("c5", 8, False) == "configs[4]"
    assert bench.baseline_config("c2", 8, False).startswith("configs[1] per GPU x8")
    assert "split over 2" in bench.baseline_config("c2", 2, True)


def test_chunked_oracle_equals_one_shot():
    """bench.py's verification feeds the oracle whole-frame chunks of <= 256
    MiB; the exact uint64 sums make that equal to one pass (BMF frames of
    344 064 B do not divide 256 MiB, so the chunk is rounded down to frames)"""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import b2p_oracle as npo
    import oracle_c as co
    g = npo.Geom(nbit=16, big_endian=1, nchunk=48, nsamp_df=128, nchan_chunk=7, nsamp_int=128 * 900)
    buf = co.fill_synthetic(g, g.block_bytes, 20181105, 0, 3)       # 310 MB: two chunks
    geom = g.asdict()
    got = bench.oracle_spectrum(geom, lambda off, n: buf[off:off + n], g.block_bytes, 4)
    assert np.array_equal(got.view(np.uint32), co.power(g, buf, nthreads=4).view(np.uint32))
    # and the host-regenerated blocks of the time-split check equal the block itself
    rd = bench.synthetic_reader(geom, 0, 3, 4)
    assert np.array_equal(rd(g.frame_bytes * 5, g.frame_bytes * 2),
                          buf[g.frame_bytes * 5:g.frame_bytes * 7])


def test_cpu_share_parsing(monkeypatch, tmp_path):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import cpu_baseline as cb
    f = tmp_path / "cpu.max"
    real_open = open

    def fake_open(path, *a, **k):
        return real_open(f if path == "/sys/fs/cgroup/cpu.max" else path, *a, **k)

    monkeypatch.setattr("builtins.open", fake_open)
    f.write_text("1600000 100000\n")
    assert cb.cgroup_cpus() == 16.0
    assert cb.effective_cpus() == min(16, len(os.sched_getaffinity(0)))
    # the timed legs leave one CPU of a quota to the rest of the job
    assert cb.baseline_threads() == min(15, len(os.sched_getaffinity(0)))
    f.write_text("max 100000\n")
    assert cb.cgroup_cpus() is None
    assert cb.effective_cpus() == len(os.sched_getaffinity(0))
    assert cb.baseline_threads() == len(os.sched_getaffinity(0))
    env = cb.child_env(16)
    assert env["OMP_NUM_THREADS"] == "16" and env["OMP_PLACES"] == "cores"
    assert "OMP_WAIT_POLICY" not in env or env["OMP_WAIT_POLICY"] == os.environ.get("OMP_WAIT_POLICY")
    assert cb.child_env(4, wait="passive")["OMP_WAIT_POLICY"] == "passive"
    assert cb.throttled_frac({"nr_periods": 50, "nr_throttled": 2}) == 0.04
    assert cb.throttled_frac(None) is None


def test_watchdog_names_the_stuck_phase_and_exits_4(tmp_path):
    """a phase that outlives its limit ends the rank with exit 4 and a line
    naming the phase (a rank stuck inside RCCL cannot be unwound)"""
    code = ("import time, sys; sys.path.insert(0, %r)\n"
            "from paf_b2p.distributed import Watchdog\n"
            "w = Watchdog(3, 0.5)\n"
            "with w.phase('quick phase'):\n    time.sleep(0.1)\n"
            "w.arm('first nccl collective (communicator set-up)')\n"
            "time.sleep(30)\n" % os.path.join(REPO, "paf-baseband2power_amd"))
    t0 = __import__("time").time()
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 4
    assert __import__("time").time() - t0 < 20
    assert "rank 3: first nccl collective (communicator set-up) did not finish within 0.5 s" in r.stderr


def test_missing_rank_rendezvous_is_bounded():
    """a launched rank whose peer never arrives gives up within
    --dist-timeout (non-zero exit) instead of waiting for the driver's limit"""
    import socket
    import time
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    t0 = time.time()
    r = _run(["--gpus", "2", "--steps", "2", "--dist-backend", "gloo", "--dist-timeout", "6"],
             {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
              "MASTER_PORT": str(port)})
    assert r.returncode != 0
    assert time.time() - t0 < 120
    assert r.stdout.strip() == ""


def test_trace_legs_cuts_a_kernel_trace_by_the_bench_phases(tmp_path):
    """tools/trace_legs.py: the bench line's launch_phases slice the trace's
    integrate dispatches (in dispatch order) into legs of one shape each"""
    import json
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import trace_legs
    hdr = ('"Kind","Agent_Id","Queue_Id","Stream_Id","Thread_Id","Dispatch_Id","Kernel_Id","Kernel_Name",'
           '"Correlation_Id","Start_Timestamp","End_Timestamp"\n')
    rows, t, did = [], 1000, 0
    plan = [("warmup", 2, 600), ("headline", 10, 596), ("one_per_launch_warmup", 1, 150),
            ("one_per_launch", 20, 149), ("calibration_warmup", 1, 597), ("calibration", 16, 591)]
    for _, n, us in plan:
        for _ in range(n):
            did += 1
            rows.append(f'"KERNEL_DISPATCH","Agent 2",1,1,1,{did},7,"void b2p::b2p_integrate_kernel<0, 1, 4, true>'
                        f'(b2p::IntegrateArgs)",{did},{t},{t + us * 1000}\n')
            did += 1   # another kernel in between (a finalize) is skipped
            rows.append(f'"KERNEL_DISPATCH","Agent 2",1,1,1,{did},8,"b2p::b2p_finalize_kernel(b2p::FinalizeArgs)",'
                        f'{did},{t},{t + 4000}\n')
            t += us * 1000 + 5000
    tr = tmp_path / "trace.csv"
    tr.write_text(hdr + "".join(rows[::-1]))   # order is restored by dispatch id
    line = {"config": {"bytes_per_integration": 1 << 30},
            "roofline": {"launch_phases": [[n, c] for n, c, _ in plan], "algorithmic_bytes_per_launch": 4 << 30,
                         "peak": 8000.0, "avg_launch_us": 596.5, "kernel_only_us": 591.0}}
    out = trace_legs.legs(str(tr), line)
    assert out["counts_agree"] and out["integrate_dispatches"] == 50
    assert out["legs"]["headline"]["avg_us"] == 596.0 and out["legs"]["headline"]["launches"] == 10
    assert out["legs"]["one_per_launch"]["avg_us"] == 149.0
    assert out["legs"]["calibration"]["launches"] == 16
    assert abs(out["legs"]["headline"]["frac_of_8TBps"] - (4 << 30) / 596e-6 / 1e9 / 8000) < 1e-4
    assert json.dumps(out)


@pytest.mark.parametrize("n,config,baseline", [(2, "c2", "configs[1] per GPU x2"), (4, "c2", "configs[3]"),
                                               (8, "c5", "configs[4]")])
def test_bench_ranks_end_to_end_on_cpu(n, config, baseline):
    """bench.py's whole multi-rank path on CPU for --gpus 2/4/8: its own
    launcher spawns torch.distributed.run, the ranks meet over gloo, every
    rank reports its device from the live group, each timed region gathers
    the K spectra to rank 0, and the line rank 0 prints says so -- ranks ==
    n_gpus == N, distinct GPUs read back from the identities (N), rank 0
    holding every rank's spectra, each spectrum equal to the C oracle's.  The
    GPU is a host-memory double (tests/bench_cpu_rehearsal.py); the driver's
    8-GPU run takes the same code path with RCCL and the HIP library."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "bench_cpu_rehearsal.py"), "--gpus", str(n),
                        "--steps", "4", "--warmup", "1", "--min-seconds", "0.3", "--bpl1-seconds", "0.2",
                        "--dist-backend", "gloo", "--cpu-seconds", "0", "--config", config, "--dist-timeout", "120"],
                       capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]          # rank 0 alone prints the line
    d = json.loads(lines[0])
    assert d["n_gpus"] == d["ranks"] == n
    assert d["dist_backend"] == "gloo" and d["rccl_ranks"] == 0
    assert d["distinct_gpus"] == n
    assert [x["device"] for x in d["rank_devices"]] == list(range(n))
    assert len({x["pci_bus_id"] for x in d["rank_devices"]}) == n
    assert d["verified"] is True
    assert d["verification"]["gather"] == "rank 0 holds every rank's K spectra"
    assert d["config"]["launcher"] == "bench.py --gpus spawned torch.distributed.run"
    assert d["config"]["baseline_config"].startswith(baseline)
    assert f"over {n} MI355X" in d["config"]["workload"] and "spectra gathered to rank 0" in d["config"]["workload"]
    assert "gloo gather to rank 0" in d["config"]["parallelism"]
    assert d["one_per_launch"]["verified"] is True
    assert d["value"] > 0 and d["cpu_baseline"] is None and "secondary" not in d


def test_bench_line_carries_the_secondary_layouts_on_cpu():
    """the default one-rank line carries `secondary`: the reference-native
    BMF layout (int16 BE TFTFP, 48 x 7 channels), configs[4]'s per-GPU share
    (1024 ch int8) and configs[2] (pinned host, PCIe-bound against a bare
    H2D of the same block), each timed after the headline and verified
    against the oracle, each with a roofline of its own and the PMC summary
    of its layout"""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "bench_cpu_rehearsal.py"), "--steps", "4",
                        "--warmup", "1", "--min-seconds", "0.2", "--bpl1-seconds", "0.1", "--secondary-seconds",
                        "0.2", "--cpu-seconds", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["verified"] is True and sorted(d["secondary"]) == ["bmf", "c3", "c5"]
    b = d["secondary"]["bmf"]
    assert b["verified"] is True and b["baseline_config"] == "reference-native"
    assert "int16 BE TFTFP" in b["workload"] and "336 ch" in b["workload"]
    assert b["roofline"]["bound"] == "hbm" and b["roofline"]["bytes_per_sample"] == 4
    assert b["roofline"]["algorithmic_bytes_per_launch"] == 336 * 2 * (4 * 128) * 4  # ch x pol x samples x 4 B
    assert b["roofline"]["traffic_source"].startswith("profiles/pmc_bmf.json")
    c5 = d["secondary"]["c5"]
    assert c5["verified"] is True and c5["baseline_config"] == "configs[4] per GPU"
    assert c5["roofline"]["bytes_per_sample"] == 2 and c5["roofline"]["traffic_source"].startswith("profiles/pmc_c5")
    c3 = d["secondary"]["c3"]
    assert c3["verified"] is True and c3["baseline_config"] == "configs[2]"
    assert c3["roofline"]["bound"] == "pcie" and c3["roofline"]["peak_source"]["copies"] >= 3
    assert "frac" in c3["roofline"]["hbm"]
    assert all(v["value"] > 0 and v["timed_regions"] >= 1 for v in d["secondary"].values())
    # the headline stays configs[1]
    assert d["config"]["baseline_config"] == "configs[1]" and d["dtype"] == "int8"
    # and the list is the caller's
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--secondary", "c9"], capture_output=True,
                       text=True, timeout=120, env=env, cwd=REPO)
    assert r.returncode == 2 and "unknown layout" in r.stderr


def test_a_failed_secondary_leg_keeps_the_headline_line():
    """a secondary layout whose leg raises (here its context cannot be
    opened) is reported as that leg's `error`; the headline line still goes
    out, verified, and bench.py exits 0 -- the driver's record of configs[1]
    never depends on a secondary leg"""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["REHEARSAL_FAIL_NCHAN"] = "336"  # the BMF leg
    r = subprocess.run([sys.executable, os.path.join(REPO, "tests", "bench_cpu_rehearsal.py"), "--steps", "4",
                        "--warmup", "1", "--min-seconds", "0.2", "--bpl1-seconds", "0.1", "--secondary-seconds",
                        "0.2", "--cpu-seconds", "0"], capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["verified"] is True and d["value"] > 0
    assert d["secondary"]["bmf"]["verified"] is None and "HIP error" in d["secondary"]["bmf"]["error"]
    assert d["secondary"]["c5"]["verified"] is True and d["secondary"]["c3"]["verified"] is True
    assert "secondary leg bmf failed" in r.stderr


def test_device_code_sha_is_the_code_object_section():
    """bench.py's provenance names the sha256 of the library's gfx950 code
    objects (.hip_fatbin), read by a small ELF parse: the same bytes
    llvm-objcopy extracts"""
    import hashlib
    import shutil
    import tempfile
    sys.path.insert(0, REPO)
    import bench
    sha = bench.device_code_sha()
    assert sha and len(sha) == 64
    objcopy = shutil.which("llvm-objcopy") or "/opt/rocm/lib/llvm/bin/llvm-objcopy"
    if not os.path.exists(objcopy):
        pytest.skip("no llvm-objcopy")
    from paf_b2p import _lib
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "fatbin")
        subprocess.run([objcopy, "--dump-section", f".hip_fatbin={out}", _lib.LIB_PATH, os.path.join(d, "x")],
                       check=True)
        assert hashlib.sha256(open(out, "rb").read()).hexdigest() == sha
