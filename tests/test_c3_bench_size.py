"""GPU parity at the exact C3 shape the bench times, plus RE2-syntax constraints.

`bench.py` section c3 runs job_c3(1000) on cluster_c3(10000, seed=7) with the
visit order shuffle(10000, 17). At 10k nodes (>= loop_sweep_min) the engine's
default path is the device-resident full-pass count loop, a different regime
from the smaller clusters the other tests use. Both the
batched count loop (Place) and the unchanged caller's Select -> Commit protocol
are compared with the oracle for all 1000 placements, with no env overrides.
Reference: spread.go:110-257, select.go:79-116, generic_sched.go:552-627.
"""
import dataclasses

import pytest

from nomad_amd import synth
from nomad_amd.structs import Constraint
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place

pytestmark = pytest.mark.gpu

N, COUNT, PERM_SEED = 10000, 1000, 17


@pytest.fixture(scope="module")
def c3_oracle():
    nodes, allocs = synth.cluster_c3(N, seed=7)
    job = synth.job_c3(COUNT)
    perm = synth.shuffle(len(nodes), PERM_SEED)
    _, limit, res = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert len(res) == COUNT and all(r.row >= 0 for r in res)
    return nodes, allocs, job, perm, limit, res


def test_c3_bench_size_count_loop(c3_oracle):
    from nomad_amd.stack import GenericStack
    nodes, allocs, job, perm, limit, ro = c3_oracle
    _, le, re_ = run_place(GenericStack, nodes, allocs, job, perm)
    assert le == limit
    assert_same_placements(re_, ro)


def test_c3_bench_size_select_commit(c3_oracle):
    """The unchanged GenericScheduler loop: Select, then the plan append (Commit)."""
    from nomad_amd.stack import GenericStack
    nodes, allocs, job, perm, _, ro = c3_oracle
    e = GenericStack()
    e.SetState(nodes, allocs)
    e.SetJob(job)
    e.SetNodes(list(perm))
    got = []
    for _ in range(COUNT):
        r = e.SelectRaw(0)
        got.append(r)
        assert r.row >= 0
        e.Commit(0, r.row)
    e.close()
    assert_same_placements(got, ro)


def test_c3_bench_size_served_from_the_view(c3_oracle):
    """The caller's Select / Commit pairs answered from the served-Select view
    (pe_spec_view), as the bench's C3 drop-in loop takes them: every answer
    equals the oracle's placement, cursor included."""
    from nomad_amd.stack import GenericStack
    from tests.test_dropin import _key
    from tests.test_spec_view import ViewAnswers, protocol_answers
    nodes, allocs, job, perm, _, ro = c3_oracle
    e = GenericStack()
    e.SetState(nodes, allocs)
    e.SetJob(job)
    e.SetNodes(list(perm))
    vc = ViewAnswers(e)
    got = protocol_answers(vc, COUNT, preempt=False)
    e.close()
    want = [_key(r) for r in ro]
    assert len(got) == len(want)
    for i, (x, y) in enumerate(zip(got, want)):
        assert x[:7] == y[:7], ("Select %d" % i, x, y)
    assert vc.served >= COUNT - 8, vc.served


def _with_constraints(job, cons):
    return dataclasses.replace(job, constraints=cons)


def test_c3_re2_syntax_constraints():
    """(?i), \\pL and named groups evaluate as Go does, on the device path: the
    rewritten job filters exactly the nodes job_c3 filters, so placements equal
    both the oracle's and the plain job's."""
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c3(3000, seed=7)
    plain = synth.job_c3(300)
    re2 = _with_constraints(plain, [
        Constraint("${attr.kernel.name}", "(?i)^LINUX$", "regexp"),
        Constraint("${attr.os.version}", ">= 5.4.0", "semver"),
        Constraint("${meta.rack}", "(?i)^(?P<row>R)[0-4]\\pN", "regexp"),
        Constraint("${node.datacenter}", "^\\pL+\\d\\z", "regexp"),
    ])
    perm = synth.shuffle(len(nodes), 5)
    _, _, ro = run_place(OracleGenericStack, nodes, allocs, re2, perm)
    _, _, re_ = run_place(GenericStack, nodes, allocs, re2, perm)
    assert_same_placements(re_, ro)
    _, _, rp = run_place(GenericStack, nodes, allocs, plain, perm)
    assert_same_placements(re_, rp)
    # a pattern Go rejects filters every node on both sides
    bad = _with_constraints(plain, [Constraint("${meta.rack}", "^r(?=0)", "regexp")])
    _, _, rb = run_place(GenericStack, nodes, allocs, bad, perm)
    _, _, ob = run_place(OracleGenericStack, nodes, allocs, bad, perm)
    assert rb[0].row == -1 and ob[0].row == -1
    assert_same_placements(rb, ob)
