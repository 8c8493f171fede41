"""b2p_group (csrc/b2p_group.hip) with RCCL and the HIP runtime stubbed, on
CPU: the argument plumbing of an 8-member group that the one-GPU test box
cannot run over RCCL (rank order, devices, member-major gathers, the
non-blocking set-up polled through ncclInProgress, bounded waits that abort
the communicators).  tests/c/group_rccl_stub.cpp holds the stand-ins and the
checks; the group's object is the same source the library builds, compiled
host side by hipcc (it has no kernels of its own)."""
import os
import shutil
import subprocess

import pytest

from conftest import REPO

PKG = os.path.join(REPO, "paf-baseband2power_amd")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC) or not shutil.which("g++"), reason="needs hipcc and g++")
def test_group_plumbing_with_rccl_stubbed(tmp_path):
    grp = tmp_path / "b2p_group.o"
    subprocess.run([HIPCC, "-c", "-fPIC", "-O1", "-std=c++17", "--offload-arch=gfx950",
                    "-I", os.path.join(REPO, "include"), "-I", os.path.join(PKG, "csrc"),
                    os.path.join(PKG, "csrc", "b2p_group.hip"), "-o", str(grp)], check=True)
    und = subprocess.run(["nm", "-u", str(grp)], capture_output=True, text=True, check=True).stdout
    # the group reaches the GPU only through HIP runtime calls and RCCL: no
    # kernel of its own, so no code object to register
    assert "__hipRegisterFatBinary" not in und
    assert "ncclCommInitRankConfig" in und and "ncclGather" in und and "ncclReduce" in und
    stub = tmp_path / "stub.o"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-Wall", "-Werror", "-fPIC", "-c",
                    "-I", "/opt/rocm/include", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "c", "group_rccl_stub.cpp"), "-o", str(stub)], check=True)
    exe = tmp_path / "group_stub"
    subprocess.run(["g++", str(grp), str(stub), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "group stub: all checks passed (n = 8" in r.stdout
