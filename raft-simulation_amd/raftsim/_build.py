"""Which sources libraftsim.so is built from, and the hash that keys the build.

`__graft_entry__.build_lib()` compiles the library with the hash of these files embedded
(RAFTSIM_SRC_HASH) and rebuilds whenever the embedded hash differs from the sources' hash;
`raftsim.Simulator` refuses a library whose embedded hash is not the hash of the sources next to
it, so a box never runs a stale binary shipped beside newer sources. bench.py keys its PMC
traffic records (pmc_traffic.json) on the same hash.
"""
from __future__ import annotations

import hashlib
import re
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent.parent
KERNEL_SOURCES = ["raft-simulation_amd/csrc/tick_kernel.hip",
                  "raft-simulation_amd/csrc/steady_kernel.hip",
                  "raft-simulation_amd/csrc/storm_kernel.hip",
                  "raft-simulation_amd/csrc/tick_wave.hpp", "raft-simulation_amd/csrc/device.hpp",
                  "raft-simulation_amd/csrc/raftsim.hip", "include/raftsim.h"]
_TAG = re.compile(rb"RAFTSIM_SRC_HASH=([0-9a-f]{16}|unknown)")


def source_hash(root: Path = REPO) -> str | None:
    """sha256 of the kernel sources under root (first 16 hex digits); None if any is missing."""
    h = hashlib.sha256()
    for f in KERNEL_SOURCES:
        try:
            h.update((Path(root) / f).read_bytes())
        except OSError:
            return None
    return h.hexdigest()[:16]


def embedded_hash(lib: Path) -> str | None:
    """The source hash a built libraftsim.so carries (None if it carries none)."""
    try:
        m = _TAG.search(Path(lib).read_bytes())
    except OSError:
        return None
    return m.group(1).decode() if m else None
