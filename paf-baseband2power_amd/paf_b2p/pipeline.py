"""Pipeline launcher: the role of the reference's paf-baseband2power.py.

    python -m paf_b2p.pipeline -a paf-baseband2power.conf -b DIR -c GPU -f DATAFILE
           [-d VISIBLEGPU] [-e MEMCHECK] [-s NSUB] [-g LAYOUT] [-p NPOL_OUT] [-m]

Reads the same INI sections/keys (paf-baseband2power.py:49-80), writes the key
files (:98-112), creates the two rings with dada_db (:114-115), runs the three
stages as separate processes -- paf_diskdb, paf_baseband2power, paf_dbdisk
(:85-95, :117-127) -- and destroys the rings (:129-130).  Differences: it
parses (the reference's launcher is a SyntaxError at :90 and reads undefined
args.psrname / args.dfname at :37-38), stops the other stages if one fails,
and with -s N runs N independent sub-band chains, chain r on GPU r with ring
keys KEY + 0x10*r (one GPU, one stream, one ring per sub-band).
-e 1 (the reference's cuda-memcheck run) puts the stage on the bounds-checked
debug build of libpafb2p.  With --pin it binds the stages to CPUs as the reference does (`taskset -c`,
`dada_dbdisk -b`: paf-baseband2power.py:68,80,83,86-95).
"""
from __future__ import annotations

import argparse
import configparser
import os
import subprocess
import sys
import time

from . import dada

CONF_DIR = os.path.join(os.path.dirname(dada.BIN_DIR), "conf")


def read_conf(path: str) -> dict:
    cp = configparser.ConfigParser(inline_comment_prefixes=(";", "#"))
    cp.read(path)
    b, d, o = cp["BasicConf"], cp["DiskdbConf"], cp["Baseband2powerConf"]
    c = {
        "nsamp_df": int(b["nsamp_df"]), "npol_samp": int(b["npol_samp"]),
        "ndim_pol": int(b["ndim_pol"]), "nchk_nic": int(b["nchk_nic"]),
        "diskdb_ndf": int(d["ndf"]), "diskdb_nbuf": int(d["nblk"]),
        "diskdb_key": int(d["key"], 16), "diskdb_kfname": f"{d['kfname_prefix']}.key",
        "diskdb_hfname": d["hfname"], "diskdb_nreader": int(d["nreader"]),
        "diskdb_sod": int(d["sod"]),
        "b2p_key": int(o["key"], 16), "b2p_kfname": f"{o['kfname_prefix']}.key",
        "b2p_nreader": int(o["nreader"]), "b2p_nbuf": int(o["nblk"]),
        "b2p_nchan": int(o["nchan"]), "b2p_nbyte": int(o["nbyte"]),
    }
    # ring block sizes (paf-baseband2power.py:67, :79)
    c["diskdb_rbufsz"] = c["diskdb_ndf"] * c["nchk_nic"] * 7168
    c["b2p_rbufsz"] = c["b2p_nchan"] * c["b2p_nbyte"]
    if "bytes_per_df" in b:
        c["diskdb_rbufsz"] = c["diskdb_ndf"] * c["nchk_nic"] * int(b["bytes_per_df"])
    return c


def _bin(name: str, bin_dir: str | None = None) -> str:
    return os.path.join(bin_dir or dada.BIN_DIR, name)


def pin_cpus(pin: int | None, r: int, gather: bool = False) -> tuple:
    """(paf_diskdb, paf_baseband2power, paf_dbdisk) CPUs of chain r, or Nones
    without pinning.  The reference's launcher binds its one chain to CPUs 0,
    1, 2 (diskdb_cpu, baseband2power_cpu, dbdisk_cpu, paf-baseband2power.py
    :68,80,83); here chain r takes pin + 3r .. pin + 3r + 2.  One gathered
    process (-n N) has one stage and one sink: pin + 1 and pin + 2, the
    diskdb of sub-band 0 on pin and of sub-band r > 0 on pin + 2 + r."""
    if pin is None:
        return None, None, None
    if gather:
        return (pin if r == 0 else pin + 2 + r), pin + 1, pin + 2
    return pin + 3 * r, pin + 3 * r + 1, pin + 3 * r + 2


def _check_pin(pin: int | None, nsub: int, gather: bool) -> None:
    if pin is None:
        return
    import shutil
    if not shutil.which("taskset"):
        raise FileNotFoundError("--pin binds the stages with taskset (util-linux), which is not on PATH")
    want = {c for r in range(nsub) for c in pin_cpus(pin, r, gather)}
    bad = sorted(want - os.sched_getaffinity(0))
    if pin < 0 or bad:
        raise ValueError(f"--pin {pin}: CPU(s) {bad or [pin]} not available to this process "
                         f"(allowed: {sorted(os.sched_getaffinity(0))})")


def _taskset(cpu: int | None, cmd: list) -> list:
    return cmd if cpu is None else ["taskset", "-c", str(cpu)] + cmd


def _dbdisk(kout: int, out: str, cpu: int | None) -> list:
    return [_bin("paf_dbdisk"), "-k", f"{kout:x}", "-o", out, "-W"] + ([] if cpu is None else ["-b", str(cpu)])


def stage_env(memcheck: int) -> dict | None:
    """the stage's environment: with memcheck (the reference's -e, which runs
    the stage under cuda-memcheck, paf-baseband2power.py:89-90) the stage
    loads the bounds-checked debug build of libpafb2p (lib/debug: every span
    load of the integrate kernel and every output slot checked, an
    out-of-bounds access fails the run with its index) ahead of the release
    one its RUNPATH names"""
    if not memcheck:
        return None
    dbg = os.path.join(os.path.dirname(dada.BIN_DIR), "lib", "debug")
    if not os.path.exists(os.path.join(dbg, "libpafb2p.so")):
        raise FileNotFoundError(f"{dbg}/libpafb2p.so not built (make -C paf-baseband2power_amd)")
    env = dict(os.environ)
    env["LD_LIBRARY_PATH"] = dbg + (":" + env["LD_LIBRARY_PATH"] if env.get("LD_LIBRARY_PATH") else "")
    return env


def _ring_device(gpu: int, r: int) -> int:
    """GPU of sub-band r's input ring: the same (d + r) mod visible-devices
    rule paf_baseband2power applies to its contexts (paf_baseband2power.cu:
    89-90 picks 0 with one GPU).  torch counts devices without starting HIP."""
    import torch
    n = torch.cuda.device_count()
    return (gpu + r) % n if n > 0 else gpu + r


def run(conf_path: str, directory: str, gpu: int, datafile: str, nsub: int = 1,
        layout: str = "", npol_out: int = 1, mean: bool = False, timeout: float = 3600,
        hfname: str | None = None, outfiles: list | None = None, gather: bool = False,
        device_ring: bool = False, split: int = 1, bin_dir: str | None = None,
        stage_args: list | None = None, stage_exe: str | None = None, pin: int | None = None,
        memcheck: int = 0) -> list:
    """Run the chains; returns the output file path of every sub-band (one
    combined file with gather=True: one paf_baseband2power process serves all
    sub-bands and gathers their spectra to its first GPU).
    device_ring=True puts each input ring's blocks on its chain's GPU
    (dada_db -g): paf_diskdb copies into HBM and
    paf_baseband2power integrates the block in place.  split=N cuts every
    integration of a (single) chain by time over N GPUs (paf_baseband2power
    -t N, SURVEY.md 8e second mode).  stage_args: extra paf_baseband2power
    options (e.g. ["-G", "rccl", "-T", "30"]).  stage_exe: another build of
    paf_baseband2power (e.g. a sanitizer build in tests/test_sanitizers.py).
    pin: first CPU of the stages' bindings (pin_cpus), None: unbound.
    memcheck: the stage on the bounds-checked debug library (stage_env)."""
    _check_pin(pin, nsub, gather)
    senv = stage_env(memcheck)
    if gather:
        return _run_gathered(conf_path, directory, gpu, datafile, nsub, layout, npol_out, mean,
                             timeout, hfname, device_ring, stage_args, stage_exe, pin, senv)
    c = read_conf(conf_path)
    hdr = hfname or c["diskdb_hfname"]
    if not os.path.isabs(hdr):
        cand = [os.path.join(os.path.dirname(os.path.abspath(conf_path)), hdr),
                os.path.join(CONF_DIR, hdr)]
        hdr = next((p for p in cand if os.path.exists(p)), cand[0])
    os.makedirs(directory, exist_ok=True)
    outs, procs, keys = [], [], []
    try:
        for r in range(nsub):
            kin, kout = c["diskdb_key"] + 0x10 * r, c["b2p_key"] + 0x10 * r
            for kf, k in ((c["diskdb_kfname"], kin), (c["b2p_kfname"], kout)):
                with open(os.path.join(directory, kf if nsub == 1 else f"{r}_{kf}"), "w") as f:
                    f.write("DADA INFO:\n")
                    f.write(f"key {k:x}\n")
            dada.destroy_ring(kin)
            dada.destroy_ring(kout)
            # dada_db -p, as the reference's launcher (paf-baseband2power.py:114;
            # its -l needs CAP_IPC_LOCK and is left out)
            dada.create_ring(kin, c["diskdb_nbuf"], c["diskdb_rbufsz"], c["diskdb_nreader"],
                             device=_ring_device(gpu, r) if device_ring else -1, page=not device_ring)
            keys.append(kin)
            obytes = c["b2p_rbufsz"] * npol_out
            dada.create_ring(kout, c["b2p_nbuf"], obytes, c["b2p_nreader"])
            keys.append(kout)
            sub_dir = directory if nsub == 1 else os.path.join(directory, f"subband{r}")
            os.makedirs(sub_dir, exist_ok=True)
            out = (outfiles[r] if outfiles else os.path.join(sub_dir, "power.dada"))
            outs.append(out)
            dfile = datafile if isinstance(datafile, str) else datafile[r]
            b2p_cmd = [stage_exe or _bin("paf_baseband2power", bin_dir), "-a", f"{kin:x}", "-b", f"{kout:x}",
                       "-c", sub_dir, "-d", str(gpu + r), "-p", str(npol_out)]
            if layout:
                b2p_cmd += ["-f", layout]
            if mean:
                b2p_cmd.append("-m")
            if split > 1:
                b2p_cmd += ["-t", str(split)]
            b2p_cmd += list(stage_args or [])
            cpu_db, cpu_stage, cpu_sink = pin_cpus(pin, r)
            procs.append(subprocess.Popen(_dbdisk(kout, out, cpu_sink), stderr=subprocess.PIPE))
            procs.append(subprocess.Popen(_taskset(cpu_stage, b2p_cmd), stderr=subprocess.PIPE, env=senv))
            procs.append(subprocess.Popen(_taskset(cpu_db, [
                _bin("paf_diskdb", bin_dir), "-a", f"{kin:x}", "-b", os.path.dirname(os.path.abspath(dfile)),
                "-c", os.path.basename(dfile), "-d", hdr, "-e", str(c["diskdb_sod"])]),
                stderr=subprocess.PIPE))
        _wait_all(procs, timeout)
        return outs
    finally:
        for k in keys:  # paf-baseband2power.py:129-130
            dada.destroy_ring(k)


def _resolve_header(c, conf_path, hfname):
    hdr = hfname or c["diskdb_hfname"]
    if not os.path.isabs(hdr):
        cand = [os.path.join(os.path.dirname(os.path.abspath(conf_path)), hdr),
                os.path.join(CONF_DIR, hdr)]
        hdr = next((p for p in cand if os.path.exists(p)), cand[0])
    return hdr


def _wait_all(procs, timeout, grace=30.0):
    """until every stage has ended; the first failure (or the timeout) stops
    the rest.  Ctrl-C reaches the stages too (one process group): they end
    their transfers and exit, which is waited for (up to `grace` s) before
    the rings go, so the spectra written so far stay whole"""
    t_end = time.time() + timeout
    failed = None
    try:
        while any(p.poll() is None for p in procs):
            failed = next((p for p in procs if p.poll() not in (None, 0)), None)
            if failed or time.time() > t_end:
                break
            time.sleep(0.05)
    except KeyboardInterrupt:
        t_grace = time.time() + grace
        for p in procs:
            try:
                p.wait(max(0.0, t_grace - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        raise
    failed = failed or next((p for p in procs if p.poll() not in (None, 0)), None)
    if failed is not None or any(p.poll() is None for p in procs):
        for p in procs:  # stop the rest (exact PIDs we started)
            if p.poll() is None:
                p.kill()
                p.wait()
        msgs = [f"{p.args[0]}: rc={p.returncode} {p.stderr.read().decode(errors='replace')[-400:]}"
                for p in procs]
        raise RuntimeError("pipeline failed:\n" + "\n".join(msgs))


def _run_gathered(conf_path, directory, gpu, datafiles, nsub, layout, npol_out, mean, timeout,
                  hfname, device_ring=False, stage_args=None, stage_exe=None, pin=None, senv=None):
    c = read_conf(conf_path)
    hdr = _resolve_header(c, conf_path, hfname)
    os.makedirs(directory, exist_ok=True)
    kout = c["b2p_key"]
    procs, keys = [], []
    try:
        dada.destroy_ring(kout)
        dada.create_ring(kout, c["b2p_nbuf"], nsub * c["b2p_rbufsz"] * npol_out, c["b2p_nreader"])
        keys.append(kout)
        for r in range(nsub):
            kin = c["diskdb_key"] + 0x10 * r
            dada.destroy_ring(kin)
            # dada_db -p, as the reference's launcher (paf-baseband2power.py:114;
            # its -l needs CAP_IPC_LOCK and is left out)
            dada.create_ring(kin, c["diskdb_nbuf"], c["diskdb_rbufsz"], c["diskdb_nreader"],
                             device=_ring_device(gpu, r) if device_ring else -1, page=not device_ring)
            keys.append(kin)
        out = os.path.join(directory, "power.dada")
        procs.append(subprocess.Popen(_dbdisk(kout, out, pin_cpus(pin, 0, True)[2]), stderr=subprocess.PIPE))
        cmd = [stage_exe or _bin("paf_baseband2power"), "-a", f"{c['diskdb_key']:x}", "-b", f"{kout:x}",
               "-c", directory, "-d", str(gpu), "-p", str(npol_out), "-n", str(nsub)]
        if layout:
            cmd += ["-f", layout]
        if mean:
            cmd.append("-m")
        cmd += list(stage_args or [])
        procs.append(subprocess.Popen(_taskset(pin_cpus(pin, 0, True)[1], cmd), stderr=subprocess.PIPE, env=senv))
        for r in range(nsub):
            dfile = datafiles[r]
            procs.append(subprocess.Popen(_taskset(pin_cpus(pin, r, True)[0], [
                _bin("paf_diskdb"), "-a", f"{c['diskdb_key'] + 0x10 * r:x}",
                "-b", os.path.dirname(os.path.abspath(dfile)), "-c", os.path.basename(dfile),
                "-d", hdr, "-e", str(c["diskdb_sod"])]), stderr=subprocess.PIPE))
        _wait_all(procs, timeout)
        return [out]
    finally:
        for k in keys:
            dada.destroy_ring(k)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="baseband -> power pipeline (DADA rings)")
    ap.add_argument("-a", "--cfname", required=True, help="configuration file")
    ap.add_argument("-b", "--directory", required=True, help="output / log directory")
    ap.add_argument("-c", "--gpu", type=int, default=0, help="index of the first GPU")
    ap.add_argument("-d", "--visiblegpu", default="", help="accepted for compatibility")
    ap.add_argument("-e", "--memcheck", type=int, default=0,
                    help="1: the stage on the bounds-checked debug build of libpafb2p (lib/debug), "
                         "where the reference runs it under cuda-memcheck")
    ap.add_argument("-f", "--dfname", required=True, nargs="+", help="DADA data file(s)")
    ap.add_argument("-s", "--subbands", type=int, default=1)
    ap.add_argument("-g", "--layout", default="")
    ap.add_argument("-p", "--npol-out", type=int, default=1)
    ap.add_argument("-m", "--mean", action="store_true")
    ap.add_argument("--gather", action="store_true",
                    help="one process for all sub-bands, spectra gathered to the first GPU")
    ap.add_argument("-t", "--split", type=int, default=1,
                    help="split each integration by time over N GPUs (exact partials reduced)")
    ap.add_argument("--device-ring", action="store_true",
                    help="input ring blocks in GPU memory (dada_db -g): no H2D in the integrator")
    ap.add_argument("--bin-dir", default=None,
                    help="where paf_diskdb / paf_baseband2power live (e.g. bin/psrdada: the "
                         "PSRDADA builds, INTEGRATION.md); paf_dbdisk stays the default one")
    ap.add_argument("--pin", type=int, nargs="?", const=0, default=None, metavar="CPU",
                    help="bind the stages to CPUs as the reference's launcher does: paf_diskdb on CPU "
                         "(default 0), paf_baseband2power on CPU+1, paf_dbdisk on CPU+2; sub-band chain r "
                         "shifted by 3r")
    a = ap.parse_args(argv)
    if a.bin_dir and a.device_ring:
        ap.error("--device-ring needs libpafdada's hosts (GPU-resident rings are an extension)")
    files = a.dfname if a.subbands > 1 or a.gather else a.dfname[0]
    outs = run(a.cfname, a.directory, a.gpu, files, a.subbands, a.layout, a.npol_out, a.mean,
               gather=a.gather, device_ring=a.device_ring, split=a.split, bin_dir=a.bin_dir, pin=a.pin,
               memcheck=a.memcheck)
    print("\n".join(outs))
    return 0


if __name__ == "__main__":
    sys.exit(main())
