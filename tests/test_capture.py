"""UDP capture on the loopback interface: paf_dfsend
replays a paf_dfgen frame stream to several ports, paf_capture -o records
what arrives (no GPU).  Every frame arrives once, unchanged, with the chunk
the -m freq mapping gives."""
import os
import re
import subprocess
import time

import numpy as np
import pytest

import b2p_oracle as npo
from paf_b2p import dada

BIN = dada.BIN_DIR


def make_stream(tmp_path, nchunk=4, nblk=3, block_ndf=32, window=48, seed=3, epoch=0):
    g = npo.Geom(nbit=16, big_endian=1, nchunk=nchunk, nsamp_df=128, nchan_chunk=7,
                 nsamp_int=block_ndf * 128)
    payload = npo.fill_synthetic(g, g.block_bytes * nblk, 7, 0, 0)
    src = tmp_path / "in.dada"
    dada.write_dada_file(str(src), "NBIT 16\n", payload)
    df, ck = tmp_path / "s.df", tmp_path / "s.chunks"
    subprocess.run([os.path.join(BIN, "paf_dfgen"), "-i", str(src), "-o", str(df), "-n", str(nchunk),
                    "-c", str(ck), "-x", "249990", "-s", "54", "-f", "1300", "-r", str(seed),
                    "-w", str(window), "-e", str(epoch)], check=True, capture_output=True)
    return g, payload, df, ck


@pytest.mark.parametrize("rx_threads", [0, 1, 2])
def test_capture_records_every_frame(tmp_path, rx_threads):
    """every frame arrives once and unchanged, with one receive thread per
    port (default, as the reference's capture threads), one thread for all
    ports, or two threads sharing three ports"""
    g, _, df, ck = make_stream(tmp_path)
    port = 21000 + (os.getpid() % 500) * 8 + rx_threads * 3
    out, outc = tmp_path / "r.df", tmp_path / "r.chunks"
    cap = subprocess.Popen([os.path.join(BIN, "paf_capture"), "-o", str(out), "-O", str(outc),
                            "-P", str(port), "-N", "3", "-m", "freq:1300", "-t", "1",
                            "-R", str(rx_threads)],
                           stderr=subprocess.PIPE, text=True)
    time.sleep(0.5)
    snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck),
                          "-P", str(port), "-N", "3", "-r", "100"], capture_output=True, text=True)
    assert snd.returncode == 0, snd.stderr
    _, err = cap.communicate(timeout=60)
    assert cap.returncode == 0, err
    sent = np.fromfile(df, np.uint8).reshape(-1, npo.DF_BYTES)
    sent_ck = np.fromfile(ck, np.uint8)
    got = np.fromfile(out, np.uint8).reshape(-1, npo.DF_BYTES)
    got_ck = np.fromfile(outc, np.uint8)
    assert got.shape == sent.shape, err
    # arrival order across ports may differ: compare as sets of (frame, chunk)
    key = lambda a, c: sorted(zip((r.tobytes() for r in a), c.tolist()))  # noqa: E731
    assert key(got, got_ck) == key(sent, sent_ck)
    assert f"capture: {sent.shape[0]} frames received (0 not frames)" in err
    assert f"{rx_threads or 3} receive thread(s) over 3 port(s)" in err
    # per-port table (capture.c:700-725): every port's frames are counted
    rows = [ln for ln in err.splitlines() if "\t" in ln]
    counts = {}
    for ln in err.splitlines():
        m = re.search(r"(\d+)\t(\d+)\t(\d+)\t-\t-$", ln)
        if m:
            counts[int(m.group(1))] = int(m.group(3))
    assert sorted(counts) == [port, port + 1, port + 2] and sum(counts.values()) == sent.shape[0], rows


def test_capture_flags_non_frames(tmp_path):
    # datagrams of the wrong size are counted, not recorded
    import socket
    port = 23000 + (os.getpid() % 500) * 8
    out, outc = tmp_path / "r.df", tmp_path / "r.chunks"
    cap = subprocess.Popen([os.path.join(BIN, "paf_capture"), "-o", str(out), "-O", str(outc),
                            "-P", str(port), "-N", "1", "-m", "freq:1300", "-t", "0.5"],
                           stderr=subprocess.PIPE, text=True)
    time.sleep(0.5)
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    for n in (100, 7232, 9000):
        s.sendto(bytes(n), ("127.0.0.1", port))
    s.close()
    _, err = cap.communicate(timeout=60)
    assert cap.returncode == 0, err
    assert "capture: 1 frames received (2 not frames)" in err
    assert os.path.getsize(out) == 7232


def test_capture_stops_cleanly_on_sigterm(tmp_path):
    """SIGTERM ends the capture at once (no idle wait), with everything
    received so far recorded and exit status 0"""
    import signal
    import socket
    port = 24000 + (os.getpid() % 500) * 8
    out, outc = tmp_path / "r.df", tmp_path / "r.chunks"
    cap = subprocess.Popen([os.path.join(BIN, "paf_capture"), "-o", str(out), "-O", str(outc),
                            "-P", str(port), "-N", "1", "-m", "freq:1300", "-t", "60"],
                           stderr=subprocess.PIPE, text=True)
    time.sleep(0.5)
    s = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
    for _ in range(3):
        s.sendto(bytes(npo.DF_BYTES), ("127.0.0.1", port))
    s.close()
    time.sleep(0.5)
    t0 = time.time()
    cap.send_signal(signal.SIGTERM)
    _, err = cap.communicate(timeout=30)
    assert cap.returncode == 0, err
    assert time.time() - t0 < 5
    assert "stopped by a signal" in err and "capture: 3 frames received" in err
    assert os.path.getsize(out) == 3 * npo.DF_BYTES


def test_capture_refuses_missing_epoch_file(tmp_path):
    """-g names an epoch file that does not exist: the capture stops at once
    (capture.c:798-805), before touching a ring or waiting for frames"""
    hdr = tmp_path / "hdr.txt"
    hdr.write_text("HDR_SIZE 4096\n")
    r = subprocess.run([os.path.join(BIN, "paf_capture"), "-a", "7e00", "-f", str(hdr), "-g",
                        str(tmp_path / "missing_epoch.txt"), "-i", "1340.5"],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "cannot open epoch file" in r.stderr


def test_capture_refuses_bad_freq(tmp_path):
    hdr = tmp_path / "hdr.txt"
    hdr.write_text("HDR_SIZE 4096\n")
    r = subprocess.run([os.path.join(BIN, "paf_capture"), "-a", "7e00", "-f", str(hdr), "-i", "abc"],
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and "-i takes" in r.stderr


@pytest.mark.parametrize("args,msg", [(["-d", "1"], "only payload-only blocks"),
                                      (["-b", "on"], "-b takes 0 or 1")])
def test_capture_refuses_unsupported_record_flags(tmp_path, args, msg):
    """-d 1 (frames recorded with their headers, capture.c:216,222) is refused
    rather than ignored, and -b (start of data) must be 0 or 1"""
    hdr = tmp_path / "hdr.txt"
    hdr.write_text("HDR_SIZE 4096\n")
    r = subprocess.run([os.path.join(BIN, "paf_capture"), "-a", "7e00", "-f", str(hdr)] + args,
                       capture_output=True, text=True, timeout=30)
    assert r.returncode == 1 and msg in r.stderr


def test_capture_nic_option_like_the_reference(tmp_path):
    """-e NIC (paf_capture.c:88-90): the reference binds 10.17.<node>.<NIC>,
    <node> the 8th character of the host name (:115-118, HN_LEN 8); -I gives
    the address instead and wins over -e"""
    import socket
    hn = socket.gethostname()
    port = 24500 + (os.getpid() % 500) * 4
    out, outc = tmp_path / "r.df", tmp_path / "r.chunks"
    cmd = [os.path.join(BIN, "paf_capture"), "-o", str(out), "-O", str(outc), "-P", str(port), "-N", "1",
           "-m", "freq:1300", "-t", "0.5"]
    cap = subprocess.Popen(cmd + ["-e", "3"], stderr=subprocess.PIPE, text=True)
    try:
        _, err = cap.communicate(timeout=10)
    except subprocess.TimeoutExpired:  # the address exists here: bound, waiting for frames
        cap.kill()
        _, err = cap.communicate()
        assert len(hn) >= 8 and hn[7].isdigit(), err
        return
    assert cap.returncode == 1
    if len(hn) >= 8 and hn[7].isdigit():
        assert f"cannot bind 10.17.{hn[7]}.3:{port}" in err, err
    else:
        assert "has no node digit at its 8th character" in err, err
    # -I wins: the loopback address, one frame stream recorded whole
    g, _, df, ck = make_stream(tmp_path, nchunk=2, nblk=1)
    cap = subprocess.Popen(cmd + ["-e", "3", "-I", "127.0.0.1"], stderr=subprocess.PIPE, text=True)
    time.sleep(0.5)
    snd = subprocess.run([os.path.join(BIN, "paf_dfsend"), "-i", str(df), "-k", str(ck), "-H", "127.0.0.1",
                          "-P", str(port), "-N", "1", "-r", "100"], capture_output=True, text=True)
    assert snd.returncode == 0, snd.stderr
    _, err = cap.communicate(timeout=60)
    assert cap.returncode == 0, err
    assert os.path.getsize(out) == os.path.getsize(df), err
