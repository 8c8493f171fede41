"""paf_b2p -- MI355X-native baseband->power integrator (host-side mirror).

The compute lives in libpafb2p.so (hand-written gfx950 HIP behind the C ABI
of include/b2p.h); this package binds it and mirrors the reference's
interfaces (CLI, DADA rings, .conf launcher).  No CPU fallback: if the HIP
library is missing every entry point raises.
"""
from ._lib import B2PError, Geom, Tuning, lib  # noqa: F401
from .geometry import (CONFIGS, NSAMP_INT, TSAMP_US, blocks_per_launch, bmf_geom, block_bytes,  # noqa: F401
                       frame_bytes, generic_geom, make_geom, nchan, samples_per_block)
from .integrator import DeviceBuffer, Group, Integrator, device_count, pci_bus_id  # noqa: F401

__all__ = ["B2PError", "Geom", "Integrator", "DeviceBuffer", "CONFIGS", "bmf_geom",
           "generic_geom", "make_geom", "device_count", "pci_bus_id", "Tuning", "lib"]
