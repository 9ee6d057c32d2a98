"""raftsim — host side of the MI355X batched Raft simulator (libraftsim.so).

`Simulator` is the drop-in for the reference's per-process node loop (`-main`/`wait`,
src/raft/core.clj:176-203): it advances `n_clusters` independent N-node clusters in lockstep on one
GPU through the C ABI of include/raftsim.h. There is no CPU fallback: if libraftsim.so is missing,
was not built for this machine, or was built from other kernel sources than the ones beside it
(raftsim/_build.py), construction raises.
"""
from __future__ import annotations

import os
from pathlib import Path

from . import _build
from ._abi import COUNTER_NAMES  # noqa: F401
from ._backend import FAULT_NAMES, ROLE_NAMES, Backend, RaftSimError  # noqa: F401

PKG_DIR = Path(__file__).resolve().parent.parent          # raft-simulation_amd/
LIB_PATH = Path(os.environ.get("RAFTSIM_LIB", PKG_DIR / "build" / "libraftsim.so"))


_checked = []


def check_build():
    """Refuse a libraftsim.so built from other kernel sources than the ones in this tree (the
    library embeds the hash of the sources it was compiled from; RAFTSIM_LIB overrides skip it)."""
    if _checked or "RAFTSIM_LIB" in os.environ:
        return
    want, got = _build.source_hash(), _build.embedded_hash(LIB_PATH)
    if want is None:
        raise RaftSimError("kernel sources missing beside the library: cannot check which sources "
                           f"{LIB_PATH} was built from")
    if got != want:
        raise RaftSimError(f"{LIB_PATH} was built from kernel sources {got}, the tree holds "
                           f"{want}: rebuild with __graft_entry__.build()")
    _checked.append(True)


class Simulator(Backend):
    """Batched simulator on the GPU (HIP kernels for gfx950)."""

    def __init__(self, **config):
        if not LIB_PATH.exists():
            raise RaftSimError(f"{LIB_PATH} not built: run __graft_entry__.build()")
        check_build()
        super().__init__(LIB_PATH, "raft_sim_", **config)

    def diag_last_bails(self):
        """Diagnostic: clusters the steady kernel handed to the general kernel in the last tick
        launch (steady_kernel.hip), or -1 if that launch did not take the steady path."""
        import ctypes

        f = self._lib.raftsim_diag_last_bails
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p]
        return int(f(self._h))

    def diag_storm_bails(self):
        """Diagnostic: clusters the storm kernel (storm_kernel.hip) listed for the lane-per-node
        STORM body in the last storm launch, summed over shards; -1 if no storm-kernel launch ran
        on this handle."""
        import ctypes

        f = self._lib.raftsim_diag_storm_bails
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p]
        return int(f(self._h))

    def timed_launches(self):
        """Launches of the last sync window that carried HIP events: last_step_timing's average
        is over these (every general launch, the first steady launch after a sync)."""
        import ctypes

        f = self._lib.raftsim_last_timed_launches
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p]
        return int(f(self._h))
