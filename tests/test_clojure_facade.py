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


HARNESS = (ROOT / "clojure" / "src" / "raft" / "sim" / "harness.clj").read_text()


def test_harness_word_arithmetic_is_unchecked():
    """Clojure's checked long * and + throw on Philox-sized products and bit-shift-right is
    arithmetic: the harness's 32-bit word arithmetic must use unchecked-multiply, unchecked-add and
    unsigned-bit-shift-right ((* 0xD2511F53 c0) overflowed from round 2 on)."""
    code = "\n".join(l.split(";")[0] for l in HARNESS.splitlines())   # strip comments
    for op in ("(* ", "(+ ", "(bit-shift-right "):
        assert op not in code, op
    assert "(unchecked-multiply 0xD2511F53 c0)" in code
    assert "(unsigned-bit-shift-right p1 32)" in code


def test_harness_drives_every_phase():
    """The per-tick cluster driver covers P0 (client injection), the D3 choice and one wait per
    node (P1) with D8 halts, D4 re-arm, P2 delivery with the fault draws, and the D15 redirects."""
    for name in ("defn- p0", "defn- p1", "defn- p2", "defn step-tick", "defn run-cluster",
                 "defn canonical-nodes", "defn compare-golden", "halt-code", "timeout-deadline",
                 "client-gap", ":client-abandoned", ":redirects", "P-NET", "P-PART"):
        assert name in HARNESS, name
    # the hooks SURVEY §8(b) names
    for hook in ("server/incoming-rpc", "client/response-rpc", "core/generate-timeout",
                 "client/rpc", "clojure.core/rand-nth", ":resp-chan"):
        assert hook in HARNESS, hook
