"""Shared parity helpers: run the engine and the oracle on identical inputs."""
import math

import numpy as np


def run_place(stack_cls, nodes, allocs, job, perm, tg=0, count=None, **kw):
    st = stack_cls(**kw)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    limit = st.SetNodes(list(perm))
    res = st.Place(tg, count if count is not None else job.task_groups[tg].count)
    return st, limit, res


def assert_same_placements(a, b, rel=0.0):
    """Bit-exact rows/offsets/metrics; scores bit-exact (rel=0) or within rel."""
    assert len(a) == len(b), (len(a), len(b))
    for i, (x, y) in enumerate(zip(a, b)):
        assert x.row == y.row, ("placement %d: row %d vs %d" % (i, x.row, y.row))
        assert x.new_offset == y.new_offset, ("placement %d offset" % i, x.new_offset, y.new_offset)
        assert x.nodes_evaluated == y.nodes_evaluated, ("placement %d evaluated" % i, x.nodes_evaluated, y.nodes_evaluated)
        assert x.nodes_filtered == y.nodes_filtered, ("placement %d filtered" % i, x.nodes_filtered, y.nodes_filtered)
        assert x.nodes_exhausted == y.nodes_exhausted, ("placement %d exhausted" % i, x.nodes_exhausted, y.nodes_exhausted)
        if x.row < 0:
            continue
        assert len(x.scores) == len(y.scores), ("placement %d nscores" % i, x.scores, y.scores)
        for s, t in zip([x.final_score] + x.scores, [y.final_score] + y.scores):
            if rel == 0.0:
                assert s == t or (math.isnan(s) and math.isnan(t)), ("placement %d score" % i, s, t)
            else:
                assert abs(s - t) <= rel * max(abs(s), abs(t)), ("placement %d score" % i, s, t)
