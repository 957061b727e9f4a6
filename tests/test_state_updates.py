"""Incremental snapshot updates (SoA ingest): an
allocation delta of the state store (allocs turning terminal — client status
complete / failed / lost — and allocs placed by other workers' applied plans,
nomad/state UpsertAllocs / UpsertPlanResults) applied to the resident HBM
snapshot with pe_update_allocs must behave exactly like a full pe_set_state of
the updated tables: same placements, scores, metrics counters, preemptions.
The reference is the oracle run on the updated state from scratch.
"""
import copy
import random

import pytest

from nomad_amd import synth
from nomad_amd.structs import Allocation, SchedulerConfig
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _delta(nodes, allocs, seed, frac_terminal=0.3, n_new=150):
    rng = random.Random(seed)
    changed, index = [], []
    for i, a in enumerate(allocs):
        if not a.terminal and rng.random() < frac_terminal:
            b = copy.deepcopy(a)
            b.terminal = True
            changed.append(b)
            index.append(i)
    for k in range(n_new):
        nd = rng.choice(nodes)
        changed.append(Allocation(node_id=nd.id, job_id="other-%d" % (k % 7), task_group="web",
                                  cpu_shares=rng.choice([250, 500, 1000]), memory_mb=rng.choice([128, 512]),
                                  disk_mb=150, priority=rng.choice([20, 50])))
        index.append(None)
    updated = list(allocs)
    for a, i in zip(changed, index):
        if i is None:
            updated.append(a)
        else:
            updated[i] = a
    return changed, index, updated


@pytest.mark.gpu
def test_update_allocs_equals_fresh_state():
    from nomad_amd.stack import GenericStack
    nodes, allocs = synth.cluster_c2(1500, seed=21)
    changed, index, updated = _delta(nodes, allocs, 1)
    job = synth.job_c2(300)
    perm = synth.shuffle(len(nodes), 7)
    st = GenericStack()
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.SetNodes(list(perm))
    st.Place(0, 50)                      # an evaluation on the old snapshot
    st.UpdateAllocs(changed, index)      # state delta: plan / memo / job reset
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, 300)
    _, _, want = run_place(OracleGenericStack, nodes, updated, job, perm)
    assert_same_placements(got, want)
    # a second delta on top of the first
    changed2, index2, updated2 = _delta(nodes, updated, 2, frac_terminal=0.2, n_new=80)
    st.UpdateAllocs(changed2, index2)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got2 = st.Place(0, 300)
    _, _, want2 = run_place(OracleGenericStack, nodes, updated2, job, perm)
    assert_same_placements(got2, want2)


@pytest.mark.gpu
def test_update_allocs_devices_and_preemption():
    # device holders turning terminal free instances; new low-priority holders
    # become preemption candidates (PreemptForDevice / PreemptForTaskGroup)
    from nomad_amd.stack import GenericStack
    cfg = SchedulerConfig(preempt_service=True)
    nodes, allocs = synth.cluster_c5(600, seed=4, busy=0.9)
    rng = random.Random(5)
    changed, index = [], []
    for i, a in enumerate(allocs):
        if a.devices and not a.terminal and rng.random() < 0.25:
            b = copy.deepcopy(a)
            b.terminal = True
            changed.append(b)
            index.append(i)
    updated = list(allocs)
    for a, i in zip(changed, index):
        updated[i] = a
    job = synth.job_c5(120)
    perm = synth.shuffle(len(nodes), 9)
    st = GenericStack(config=cfg)
    st.SetState(nodes, allocs)
    st.UpdateAllocs(changed, index)
    st.SetJob(job)
    st.SetNodes(list(perm))
    got = st.Place(0, 120)
    _, _, want = run_place(OracleGenericStack, nodes, updated, job, perm, config=cfg)
    assert_same_placements(got, want)
    assert [g.preempted for g in got] == [w.preempted for w in want]
