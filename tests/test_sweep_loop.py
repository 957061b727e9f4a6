"""Full-pass count loops routed through the multi-CU sweep (pe_place when the
list is at least sweep_min long): identical placements to the oracle. The
threshold is lowered with PE_SWEEP_MIN so the path runs at test sizes."""
import os

import pytest

from nomad_amd import synth
from oracle.oracle import OracleGenericStack
from tests.helpers import assert_same_placements, run_place


def _engine_low_threshold():
    from nomad_amd.stack import GenericStack
    old = os.environ.get("PE_SWEEP_MIN")
    os.environ["PE_SWEEP_MIN"] = "1000"
    try:
        return GenericStack()
    finally:
        if old is None:
            del os.environ["PE_SWEEP_MIN"]
        else:
            os.environ["PE_SWEEP_MIN"] = old


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
