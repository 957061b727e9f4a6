"""Full-pass count loops routed through the multi-CU sweep (pe_place when the
list is at least sweep_min long): identical placements to the oracle. The
threshold is lowered with PE_LOOP_SWEEP_MIN so the path runs at test sizes."""
import os

import pytest

from nomad_amd import synth
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _engine_low_threshold():
    from nomad_amd.stack import GenericStack
    old = os.environ.get("PE_LOOP_SWEEP_MIN")
    os.environ["PE_LOOP_SWEEP_MIN"] = "1000"
    try:
        return GenericStack()
    finally:
        if old is None:
            del os.environ["PE_LOOP_SWEEP_MIN"]
        else:
            os.environ["PE_LOOP_SWEEP_MIN"] = old


@pytest.mark.gpu
@pytest.mark.parametrize("n,count,seed", [(2500, 120, 7), (4000, 60, 9)])
def test_sweep_count_loop_matches_oracle(n, count, seed):
    nodes, allocs = synth.cluster_c3(n, seed=seed)
    job = synth.job_c3(count)
    perm = synth.shuffle(n, seed + 1)
    _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert_same_placements(got, want)


@pytest.mark.gpu
def test_sweep_count_loop_until_full():
    # more asks than room: the loop ends on the first nil Select like the chain
    nodes, allocs = synth.cluster_c3(1500, seed=3)
    job = synth.job_c3(5000)
    job.task_groups[0].tasks[0].cpu = 6000
    perm = synth.shuffle(1500, 4)
    _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert got[-1].row == -1
    assert_same_placements(got, want)


@pytest.mark.gpu
def test_sweep_count_loop_devices():
    # device asks on the device-resident loop: the step kernel commits the
    # record's device offers (AssignDevice choice) like pe_commit does
    from nomad_amd.structs import Affinity
    nodes, allocs = synth.cluster_c5(1500, seed=6, busy=0.3)
    job = synth.job_c5(150)
    job.affinities.append(Affinity("${node.datacenter}", "dc1", "=", 40))   # full pass (limit MaxInt32)
    perm = synth.shuffle(1500, 2)
    _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert_same_placements(got, want)
    assert [g.device_offers for g in got] == [w.device_offers for w in want]


@pytest.mark.gpu
def test_persistent_count_loop_matches_oracle():
    # the opt-in persistent variant (one launch, grid barriers) gives the same placements
    os.environ["PE_LOOP_PERSISTENT"] = "1"
    os.environ["PE_FULL_LDS"] = "0"   # the one-workgroup loop would take it first
    try:
        nodes, allocs = synth.cluster_c3(2500, seed=11)
        job = synth.job_c3(100)
        perm = synth.shuffle(2500, 12)
        _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    finally:
        del os.environ["PE_LOOP_PERSISTENT"]
        del os.environ["PE_FULL_LDS"]
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert_same_placements(got, want)


# ---- the one-workgroup loop (k_fullpass_lds) against the oracle and the
# multi-workgroup loop, over the job shapes that take its different branches

def _c3_variant(kind, count):
    from nomad_amd.structs import Affinity, Constraint, Spread, SpreadTarget
    job = synth.job_c3(count)
    if kind == "even":          # evenSpreadScoreBoost: the table is rebuilt every placement
        job.spreads = [Spread("${node.datacenter}", 100, [])]
    elif kind == "two":         # two spread properties (NP = 2)
        job.spreads.append(Spread("${node.class}", 50, [SpreadTarget("c1", 40), SpreadTarget("c2", 20)]))
    elif kind == "affinity":    # no spread (NP = 0)
        job.spreads = []
    elif kind == "distinct":    # distinct_hosts: a committed node leaves the options
        job.constraints.append(Constraint("", "", "distinct_hosts"))
    elif kind == "negative":    # every score <= 0: the LimitIterator skip rule decides
        job.spreads = [Spread("${node.datacenter}", 100, [SpreadTarget("dc9", 100)])]
        job.affinities = [Affinity("${node.class}", "c3", "!=", -100)]
    return job


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["even", "two", "affinity", "distinct", "negative"])
def test_one_workgroup_loop_variants(kind):
    nodes, allocs = synth.cluster_c3(3000, seed=21)
    job = _c3_variant(kind, 150)
    perm = synth.shuffle(3000, 22)
    _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert_same_placements(got, want)
    os.environ["PE_FULL_LDS"] = "0"
    try:
        _, _, multi = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    finally:
        del os.environ["PE_FULL_LDS"]
    assert_same_placements(multi, want)


@pytest.mark.gpu
def test_one_workgroup_loop_option_overflow():
    # more options than LDS entries (9216): the kernel stops before any commit
    # and the multi-workgroup loop places instead
    from nomad_amd.structs import Affinity
    nodes, allocs = synth.cluster_c2(12000, seed=23)
    job = synth.job_c2(40)
    job.affinities = [Affinity("${node.datacenter}", "dc1", "=", 30)]   # full pass
    perm = synth.shuffle(12000, 24)
    _, _, got = run_place(_engine_low_threshold, nodes, allocs, job, perm)
    _, _, want = run_place(OracleGenericStack, nodes, allocs, job, perm)
    assert_same_placements(got, want)
