"""F1: the Clojure facade clojure/src/raft/sim.clj binds include/raftsim.h through JNA.
No JVM exists in this image, so the facade cannot run here; this test pins what can be checked
statically: its struct offsets and sizes equal the C compiler's (via the ctypes mirror that
tests/test_abi.py checks against gcc), its counter order equals the header's enum, and every
raft_sim_* symbol it calls is declared by the header."""
import ctypes
import re
from pathlib import Path

from raftsim import _abi

ROOT = Path(__file__).resolve().parent.parent
CLJ = (ROOT / "clojure" / "src" / "raft" / "sim.clj").read_text()
HEADER = (ROOT / "include" / "raftsim.h").read_text()


def clj_map(name):
    body = re.search(r"\(def " + name + r"\s*\{(.*?)\}\)", CLJ, re.S).group(1)
    return {k.replace("-", "_"): int(v) for k, v in re.findall(r":([a-z0-9-]+)\s+(\d+)", body)}


def test_config_offsets():
    got = clj_map("config-offsets")
    assert got == {f: getattr(_abi.Config, f).offset for f, _ in _abi.Config._fields_}
    assert int(re.search(r"\(def config-size (\d+)\)", CLJ).group(1)) == ctypes.sizeof(_abi.Config)


def test_node_offsets():
    got = clj_map("node-offsets")
    want = {f: getattr(_abi.Node, f).offset for f, _ in _abi.Node._fields_ if f != "reserved0"}
    assert got == want
    assert int(re.search(r"\(def node-size (\d+)\)", CLJ).group(1)) == ctypes.sizeof(_abi.Node)


def test_counters():
    names = re.findall(r":([a-z-]+)", re.search(r"\(def counter-names\s*\[(.*?)\]\)", CLJ, re.S).group(1))
    assert [n.replace("-", "_") for n in names] == _abi.COUNTER_NAMES
    assert int(re.search(r"\(def counters-size (\d+)\)", CLJ).group(1)) == ctypes.sizeof(_abi.Counters)
    assert "(.getLong m 240)" in CLJ and _abi.Counters.payload_max.offset == 240


def test_symbols_exist_in_header():
    used = set(re.findall(r'"(raft_sim_\w+)"', CLJ))
    declared = set(re.findall(r"\b(raft_sim_\w+)\s*\(", HEADER))
    assert used and used <= declared, used - declared
    assert "(def abi-version 2)" in CLJ and "#define RAFT_SIM_ABI_VERSION 2" in HEADER
