"""Edge cases of the Stack boundary, engine against oracle (oracle alone on CPU):
empty and one-node lists, count 0, nothing feasible, zero-capacity nodes, a
full cluster, the batch limit of 2, a count larger than the cluster holds,
preferred nodes combined with penalties, and device / eviction corner cases."""
import pytest

from nomad_amd import synth
from nomad_amd.stack import SelectOptions
from nomad_amd.structs import (Allocation, Constraint, DeviceGroup, Job, RequestedDevice, SchedulerConfig, Task,
                               TaskGroup)
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements


def _engine(**kw):
    from nomad_amd.stack import GenericStack
    return GenericStack(**kw)


BOTH = [pytest.param(OracleGenericStack, id="oracle"),
        pytest.param(_engine, id="engine", marks=pytest.mark.gpu)]


def place(stack_cls, nodes, allocs, job, perm, count=None, **kw):
    st = stack_cls(**kw)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    lim = st.SetNodes(list(perm))
    return lim, st.Place(0, job.task_groups[0].count if count is None else count)


def same_as_oracle(nodes, allocs, job, perm, count=None, **kw):
    ro = place(OracleGenericStack, nodes, allocs, job, perm, count, **kw)
    re = place(_engine, nodes, allocs, job, perm, count, **kw)
    assert ro[0] == re[0]
    assert_same_placements(re[1], ro[1])
    return ro[1]


@pytest.mark.parametrize("stack_cls", BOTH)
def test_empty_visit_list(stack_cls):
    nodes, allocs = synth.cluster_c2(50, seed=1)
    lim, res = place(stack_cls, nodes, allocs, synth.job_c2(3), [])
    assert lim == 2
    assert len(res) == 1 and res[0].row == -1


@pytest.mark.parametrize("stack_cls", BOTH)
def test_count_zero_places_nothing(stack_cls):
    nodes, allocs = synth.cluster_c2(50, seed=1)
    _, res = place(stack_cls, nodes, allocs, synth.job_c2(5), synth.shuffle(50, 2), count=0)
    assert res == []


@pytest.mark.parametrize("stack_cls", BOTH)
def test_single_node_list_fills_then_nil(stack_cls):
    nodes, allocs = synth.cluster_c2(20, seed=3)
    perm = [7]
    cap = (nodes[7].cpu_shares - nodes[7].reserved_cpu) // 500
    _, res = place(stack_cls, nodes, [], synth.job_c2(100), perm)
    placed = [r for r in res if r.row >= 0]
    assert all(r.row == 7 for r in placed)
    assert 0 < len(placed) <= cap
    assert res[-1].row == -1 and res[-1].nodes_exhausted == 1


@pytest.mark.gpu
def test_nothing_feasible():
    nodes, allocs = synth.cluster_c2(300, seed=4)
    job = synth.job_c2(10)
    job.constraints.append(Constraint("${attr.kernel.name}", "plan9", "="))
    res = same_as_oracle(nodes, allocs, job, synth.shuffle(300, 1))
    assert len(res) == 1 and res[0].row == -1 and res[0].nodes_filtered == 300


@pytest.mark.gpu
def test_zero_capacity_and_full_nodes():
    nodes, allocs = synth.cluster_c2(400, seed=5)
    for nd in nodes[::3]:
        nd.cpu_shares = nd.reserved_cpu          # no allocatable cpu
    for nd in nodes[1::3]:
        allocs.append(Allocation(node_id=nd.id, job_id="hog", task_group="tg",
                                 cpu_shares=nd.cpu_shares - nd.reserved_cpu, memory_mb=64))
    same_as_oracle(nodes, allocs, synth.job_c2(600), synth.shuffle(400, 2))


@pytest.mark.gpu
def test_batch_limit_two():
    nodes, allocs = synth.cluster_c2(500, seed=6)
    same_as_oracle(nodes, allocs, synth.job_c2(200), synth.shuffle(500, 3), batch=True)


@pytest.mark.gpu
def test_count_beyond_cluster_capacity():
    nodes, allocs = synth.cluster_c2(40, seed=7)
    res = same_as_oracle(nodes, allocs, synth.job_c2(5000), synth.shuffle(40, 4))
    assert res[-1].row == -1 and len(res) < 5000


@pytest.mark.parametrize("stack_cls", BOTH)
def test_preferred_nodes_with_penalty(stack_cls):
    """stack.go:121-132: the preferred list is tried first; the penalty
    (NodeReschedulingPenaltyIterator) still applies there."""
    nodes, allocs = synth.cluster_c2(60, seed=8)
    st = stack_cls()
    st.SetState(nodes, allocs)
    st.SetJob(synth.job_c2(3))
    st.SetNodes(list(synth.shuffle(60, 5)))
    pref = [nodes[11].id, nodes[12].id]
    r = st.Select(0, SelectOptions(preferred_nodes=pref, penalty_node_ids=[nodes[11].id]))
    assert r is not None and r.row in (11, 12)
    if r.row == 11:
        assert -1.0 in r.scores


@pytest.mark.gpu
def test_preferred_and_penalty_parity():
    nodes, allocs = synth.cluster_c2(200, seed=9)
    out = []
    for cls in (OracleGenericStack, _engine):
        st = cls()
        st.SetState(nodes, allocs)
        st.SetJob(synth.job_c2(3))
        st.SetNodes(list(synth.shuffle(200, 6)))
        rs = []
        for k in range(20):
            opts = SelectOptions(preferred_nodes=[nodes[(7 * k) % 200].id],
                                 penalty_node_ids=[nodes[(3 * k) % 200].id, nodes[(5 * k) % 200].id])
            r = st.Select(0, opts)
            rs.append((r.row, r.final_score, r.scores, r.new_offset) if r else None)
            if r:
                st.Commit(0, r.row)
        out.append(rs)
    assert out[0] == out[1]


def gpu_node(nid, healthy):
    nd = synth.mock_node(nid)
    nd.devices = [DeviceGroup("nvidia", "gpu", "h100", healthy, dict(synth.GPU_MODELS["h100"]))]
    nd.compute_class()
    return nd


@pytest.mark.parametrize("stack_cls", BOTH)
def test_device_request_larger_than_any_group(stack_cls):
    nodes = [gpu_node("a", 2), gpu_node("b", 4)]
    job = Job(id="big", task_groups=[TaskGroup(name="t", count=1, tasks=[
        Task(name="t", cpu=100, memory_mb=64, devices=[RequestedDevice("nvidia/gpu", 5)])])])
    _, res = place(stack_cls, nodes, [], job, [0, 1])
    assert res[0].row == -1 and res[0].nodes_filtered == 2


@pytest.mark.parametrize("stack_cls", BOTH)
def test_eviction_without_candidates_is_nil(stack_cls):
    """Only higher-priority work on the node: nothing is preemptible
    (filterAndGroupPreemptibleAllocs, priority delta < 10)."""
    nd = gpu_node("a", 2)
    allocs = [Allocation(node_id="a", job_id="vip", task_group="t", cpu_shares=3800, memory_mb=64, priority=75,
                         devices=[(0, 2)])]
    job = synth.job_c5(1)
    job.priority = 80
    st = stack_cls(config=SchedulerConfig(preempt_service=True))
    st.SetState([nd], allocs)
    st.SetJob(job)
    st.SetNodes([nd])
    assert st.SelectRaw(0).row == -1
    assert st.SelectRaw(0, SelectOptions(preempt=True)).row == -1
