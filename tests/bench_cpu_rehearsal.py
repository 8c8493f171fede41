"""TEST HARNESS, CPU only: runs bench.py's real rank plumbing -- its
launcher (`--gpus N` spawning torch.distributed.run), the gloo rendezvous,
the identities read back from the live group, the timed regions with their
gather to rank 0, the oracle verification and the JSON line -- with the GPU
replaced by a host-memory double of paf_b2p.Integrator whose spectra come
from the C oracle.  tests/test_bench_launcher.py starts it for --gpus
2/4/8; the driver's 8-GPU run takes the same code with RCCL and the HIP
library.

The double stands for N visible GPUs (device r behind PCI bus r), so
`distinct_gpus` is what bench.py reads back from every rank's identity, not
a number this script supplies.  Blocks are small (64 samples of 256
channels), so 8 ranks fit a CPU test."""
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "paf-baseband2power_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import b2p_oracle as npo  # noqa: E402
import bench  # noqa: E402
import oracle_c as co  # noqa: E402
import paf_b2p  # noqa: E402
from paf_b2p import geometry  # noqa: E402

NDEV = int(os.environ.get("REHEARSAL_NDEV", "8"))
NSAMP = 64


class _Buf:
    def __init__(self, n):
        self.arr = np.zeros(max(n, 16), dtype=np.uint8)
        self.ptr, self.nbytes = self.arr.ctypes.data, n

    def free(self):
        self.ptr = 0


class _Info:
    def __init__(self, device, nout):
        self.device, self.nout = device, nout
        self.threads, self.columns, self.row_groups, self.replicas, self.unroll, self.nontemporal = 64, 1, 1, 1, 1, 1


class FakeIntegrator:
    """paf_b2p.Integrator's surface as bench.py uses it, on host memory"""

    def __init__(self, geom, device=0, **_):
        self.g = npo.Geom(**{f: int(getattr(geom, f)) for f, _ in geom._fields_ if f != "reserved"})
        # REHEARSAL_FAIL_NCHAN=N: opening a context of N channels fails, as a
        # HIP error (out of memory, a lost device) would in one secondary leg
        if os.environ.get("REHEARSAL_FAIL_NCHAN") == str(self.g.nchunk * self.g.nchan_chunk):
            raise RuntimeError(f"b2p_open: HIP error (rehearsal: {self.g.nchunk * self.g.nchan_chunk} channels)")
        self.device = device
        self.nout, self.block_bytes = self.g.nout, self.g.block_bytes
        self.info = _Info(device, self.nout)
        self._bufs, self._timing, self._stats = {}, 0, None
        self.reset_stats()

    def alloc(self, n):
        b = _Buf(n)
        self._bufs[b.ptr] = b
        return b

    def fill_synthetic(self, d, seed, subband, block, elem0=0):
        d.arr[:d.nbytes] = co.fill_synthetic(self.g, d.nbytes, seed, subband, block, elem0=elem0).view(np.uint8)

    def _spectrum_into(self, blk, dst):
        sp = co.power(self.g, blk.arr[:self.block_bytes], nthreads=1)
        C.memmove(dst, sp.ctypes.data, self.nout * 4)

    def _launch(self, nblk):
        self._stats["launches"] += 1
        self._stats["bytes"] += nblk * self.block_bytes
        self._stats["kernel_ms"] += 1e-3 * nblk

    # the host-span path (configs[2]): push a registered host block, finish into device memory
    def register_host(self, arr):
        self._pushed = None

    def unregister_host(self, arr):
        pass

    def push(self, blk):
        self._pushed = blk if isinstance(blk, np.ndarray) else blk.arr[:self.block_bytes]
        self._launch(1)

    def finish_async(self, dst, out_is_device):
        sp = co.power(self.g, self._pushed, nthreads=1)
        C.memmove(dst, sp.ctypes.data, self.nout * 4)
        return 0

    def upload_into(self, d, arr, offset=0):
        d.arr[offset:offset + arr.nbytes] = arr.view(np.uint8).reshape(-1)

    def integrate(self, blk, dst, out_is_device):
        self._spectrum_into(blk, dst)
        self._launch(1)

    def integrate_n(self, blks, dst, out_is_device):
        for i, b in enumerate(blks):
            self._spectrum_into(b, dst + i * self.nout * 4)
        self._launch(len(blks))

    def download(self, d, nbytes=None, offset=0):
        n = d.nbytes - offset if nbytes is None else nbytes
        return d.arr[offset:offset + n].copy()

    def sync(self):
        pass

    def set_timing(self, mode):
        self._timing = mode

    def stats(self):
        return dict(self._stats)

    def reset_stats(self):
        self._stats = {"launches": 0, "bytes": 0, "kernel_ms": 0.0, "finalize_ms": 0.0, "finalizes": 0}

    def close(self):
        self._bufs.clear()


def _small(nchan):
    return lambda: geometry.generic_geom(nchan, nsamp_int=NSAMP)


geometry.CONFIGS["c2"]["geom"] = _small(256)
geometry.CONFIGS["c5"]["geom"] = _small(1024)
geometry.CONFIGS["c3"]["geom"] = _small(1024)
geometry.CONFIGS["bmf"]["geom"] = lambda: geometry.bmf_geom(nsamp_int=4 * 128)
paf_b2p.Integrator = FakeIntegrator
paf_b2p.pci_bus_id = lambda d: f"0000:{0x10 + d:02x}:00.0"
torch.cuda.device_count = lambda: NDEV
torch.cuda.set_device = lambda d: None
torch.cuda.get_device_name = lambda d: "host-memory double of an MI355X"
bench.cpu_threads = lambda: 1

# the launcher starts THIS script as every rank, with bench.py's arguments
_real_cmd = bench.launcher_cmd
bench.launcher_cmd = lambda a, argv, port: [c if c != os.path.abspath(bench.__file__) else os.path.abspath(__file__)
                                            for c in _real_cmd(a, argv, port)]

if __name__ == "__main__":
    sys.exit(bench.main())
