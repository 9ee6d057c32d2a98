"""The C ABI: header <-> ctypes layouts, exported symbols, loud failure without a GPU."""
import ctypes
import re
import subprocess
from pathlib import Path

import pytest

import raftsim
from raftsim import _abi

ROOT = Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "raftsim.h"


def header_functions():
    text = HEADER.read_text()
    return sorted(set(re.findall(r"\b(raft_sim_\w+)\s*\(", text)))


def test_header_declares_exactly_the_bound_symbols():
    assert header_functions() == sorted(_abi.PRODUCT_SYMBOLS)


def test_library_exports_every_header_symbol():
    assert raftsim.LIB_PATH.exists(), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", str(raftsim.LIB_PATH)],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (raft_sim_\w+)", out))
    missing = set(header_functions()) - exported
    assert not missing, missing
    lib = ctypes.CDLL(str(raftsim.LIB_PATH))        # loads without a GPU
    for sym in header_functions():
        assert hasattr(lib, sym)


def test_library_is_built_from_these_sources():
    """libraftsim.so embeds the hash of the kernel sources it was compiled from; it must be this
    tree's (a stale binary would ship to the GPU box beside newer sources, and Simulator refuses
    it there). build_lib() rebuilds on a mismatch."""
    from raftsim import _build

    assert raftsim.LIB_PATH.exists(), "run __graft_entry__.build() first"
    assert _build.embedded_hash(raftsim.LIB_PATH) == _build.source_hash()
    lib = ctypes.CDLL(str(raftsim.LIB_PATH))
    lib.raftsim_src_hash.restype = ctypes.c_char_p
    assert lib.raftsim_src_hash().decode() == _build.source_hash()


def test_oracle_mirrors_the_abi():
    import helpers
    lib = ctypes.CDLL(str(helpers.ORACLE_LIB))
    for sym in header_functions():
        if sym in ("raft_sim_last_step_timing", "raft_sim_last_span"):   # device timing only
            continue
        assert hasattr(lib, sym.replace("raft_sim_", "raft_ref_")), sym


def test_struct_layouts_match_the_c_compiler(tmp_path):
    structs = {"raft_sim_config_t": _abi.Config, "raft_node_t": _abi.Node,
               "raft_msg_t": _abi.Msg, "raft_entry_t": _abi.Entry, "raft_cluster_t": _abi.Cluster,
               "raft_counters_t": _abi.Counters}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"',
             "int main(void) {"]
    for cname, cls in structs.items():
        lines.append(f'printf("{cname} size %zu\\n", sizeof({cname}));')
        for f, _ in cls._fields_:
            lines.append(f'printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True).stdout.splitlines():
        c, f, v = line.split()
        got[(c, f)] = int(v)
    for cname, cls in structs.items():
        assert got[(cname, "size")] == ctypes.sizeof(cls), cname
        for f, _ in cls._fields_:
            assert got[(cname, f)] == getattr(cls, f).offset, (cname, f)


def test_product_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(raftsim.RaftSimError, match="gfx950|HIP|device"):
        raftsim.Simulator(n_clusters=4)


def test_config_validation_matches_oracle():
    import helpers
    bad = [dict(nodes=1), dict(nodes=10), dict(inbox_cap=0), dict(inbox_cap=17),
           dict(log_cap=8, arena_cap=15), dict(dmin=0), dict(dmin=5, dmax=4), dict(dmax=256),
           dict(drop_ppm=1000001), dict(hb=0), dict(part_epoch=0)]
    for b in bad:
        with pytest.raises(raftsim.RaftSimError):
            helpers.oracle(n_clusters=2, **b)
