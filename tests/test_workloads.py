"""The synthetic workload generator (workloads/gen.cpp): topics drawn without the
filters (bench.py's further distinct batches) equal the topics of the full draw."""
import numpy as np
import pytest

import workloads


@pytest.mark.parametrize("cfg,nf", [(1, 10000), (2, 20000), (3, 50000), (4, 101000)])
def test_topics_only_equals_full_draw(cfg, nf):
    a = workloads.generate(cfg, nf, 2000, None, 99)
    b = workloads.generate(cfg, nf, 2000, None, 99, topics_only=True)
    assert b.nf == 0 and a.nf == nf
    assert np.array_equal(a.tbytes, b.tbytes) and np.array_equal(a.toff, b.toff)
    c = workloads.generate(cfg, nf, 2000, None, 99 + 7919, topics_only=True)
    assert not np.array_equal(a.tbytes[: len(c.tbytes)], c.tbytes[: len(a.tbytes)])
