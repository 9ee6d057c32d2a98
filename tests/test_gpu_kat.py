"""The hand-derived known-answer scenarios on the GPU (libraftsim.so), and GPU == oracle state."""
import numpy as np
import pytest

import helpers
import scenarios

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kat", scenarios.ALL, ids=lambda f: f.__name__)
def test_kat_gpu(kat):
    kat(lambda scn: scenarios.run(scn, "gpu", helpers.gpu))


@pytest.mark.parametrize("kat", scenarios.ALL, ids=lambda f: f.__name__)
def test_kat_gpu_equals_oracle(kat):
    pairs = []

    def view_of(scn):
        g = scenarios.run(scn, "gpu", helpers.gpu)
        r = scenarios.run(scn, "oracle", helpers.oracle)
        pairs.append((g, r))
        return _Both(g, r)

    kat(view_of)
    for g, r in pairs:
        assert np.array_equal(g.be.digest(), r.be.digest()), \
            helpers.describe_cluster_diff(g.be, r.be, 0)
        assert g.be.counters() == r.be.counters()


class _Both:
    def __init__(self, a, b):
        self.a, self.b = a, b

    def step(self, n):
        self.a.step(n)
        self.b.step(n)

    def node(self, i):
        return self.a.node(i)

    def log(self, i):
        return self.a.log(i)

    def commit_stream(self, i):
        return self.a.commit_stream(i)

    def edn(self, i):
        return self.a.edn(i)

    def counters(self):
        return self.a.counters()
