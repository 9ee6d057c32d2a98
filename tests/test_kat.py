"""Hand-derived known-answer tests (tests/scenarios.py) on the Python restatement and the C oracle,
plus a three-way state comparison after every scenario."""
import pytest

import helpers
import scenarios


@pytest.mark.parametrize("kat", scenarios.ALL, ids=lambda f: f.__name__)
def test_kat_python_restatement(kat):
    kat(lambda scn: scenarios.run(scn, "py"))


@pytest.mark.parametrize("kat", scenarios.ALL, ids=lambda f: f.__name__)
def test_kat_c_oracle(kat):
    kat(lambda scn: scenarios.run(scn, "oracle", helpers.oracle))


@pytest.mark.parametrize("kat", scenarios.ALL, ids=lambda f: f.__name__)
def test_kat_python_equals_oracle(kat):
    """Every scenario leaves the Python restatement and the C oracle in the same state."""
    pairs = []

    def view_of(scn):
        py, be = scenarios.run(scn, "py"), scenarios.run(scn, "oracle", helpers.oracle)
        pairs.append((py, be))
        return _Both(py, be)

    kat(view_of)
    for py, be in pairs:
        helpers.compare_py_backend(py.pc, be.be, 0)


class _Both:
    """Steps two views together; reads come from the Python one (assertions apply to it)."""

    def __init__(self, py, be):
        self.py, self.be = py, be

    def step(self, n):
        self.py.step(n)
        self.be.step(n)

    def node(self, i):
        return self.py.node(i)

    def log(self, i):
        return self.py.log(i)

    def commit_stream(self, i):
        return self.py.commit_stream(i)

    def edn(self, i):
        return self.py.edn(i)

    def counters(self):
        return self.py.counters()
