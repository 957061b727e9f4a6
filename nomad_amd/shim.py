"""Python mirror of the cgo shim of INTEGRATION.md (what a maintainer adds
under scheduler/): a `Stack` whose callers stay byte-for-byte unchanged.

GenericScheduler.computePlacements (generic_sched.go:472-652) only calls
SetNodes / SetJob / Select on its stack and mutates the plan
(Plan.AppendAlloc :627, AppendStoppedAlloc :382 and :546, PopUpdate :644,
AppendPreemptedAlloc through handlePreemptions :794-816). The shim therefore
keeps a mirror of what it has told the engine about the plan and, at every
stack call, replays the plan's changes since then:

- NodeUpdate: per node, the mirrored entries that are no longer a prefix of
  the plan's list are popped (pe_plan_pop_update, newest first), the new
  ones stopped (pe_plan_stop);
- NodeAllocation: every new placement is committed in plan order
  (pe_commit), together with the NodePreemptions entries it caused
  (pe_commit_preempt, matched by PreemptedByAllocation).

A placement is committed before the next Select, which is exactly when the
engine's speculative count loop expects it, so the unchanged
caller gets the device loop. `Plan` here is the subset of structs.Plan
(structs.go:10540-10714) the protocol reads.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .stack import GenericStack, SelectOptions


@dataclass
class PlanAlloc:
    """A placed allocation in Plan.NodeAllocation."""
    id: str
    node_row: int
    task_group: str
    preempted_by: str = ""      # for NodePreemptions entries: the placing alloc's ID


@dataclass
class Plan:
    """structs.Plan: NodeAllocation / NodeUpdate / NodePreemptions per node row.
    Stops and preemptions name snapshot allocs by alloc-table row."""
    node_allocation: Dict[int, List[PlanAlloc]] = field(default_factory=dict)
    node_update: Dict[int, List[int]] = field(default_factory=dict)
    node_preemptions: Dict[int, List[tuple]] = field(default_factory=dict)   # (alloc row, preempting alloc ID)

    def AppendAlloc(self, alloc: PlanAlloc):                       # structs.go:10707-10714
        self.node_allocation.setdefault(alloc.node_row, []).append(alloc)

    def AppendStoppedAlloc(self, alloc_row: int, node_row: int):  # structs.go:10628-10660
        self.node_update.setdefault(node_row, []).append(alloc_row)

    def PopUpdate(self, alloc_row: int, node_row: int):            # structs.go:10691-10702
        ex = self.node_update.get(node_row, [])
        if ex and ex[-1] == alloc_row:
            ex.pop()
            if not ex:
                del self.node_update[node_row]

    def AppendPreemptedAlloc(self, alloc_row: int, node_row: int, preempting_id: str):   # :10664-10689
        self.node_preemptions.setdefault(node_row, []).append((alloc_row, preempting_id))


class DeviceStack:
    """scheduler.Stack on the engine, driven by an unchanged caller that only
    mutates `plan`. One handle per worker: the snapshot stays resident across
    evaluations (`new_eval` = NewEvalContext)."""

    def __init__(self, engine: GenericStack, plan: Plan):
        self.eng = engine
        self.plan = plan
        self._tg_names: List[str] = []
        self._reset_mirror()

    def _reset_mirror(self):
        self._upd: Dict[int, List[int]] = {}
        self._alloc_seen: Dict[int, int] = {}
        self._pre_seen: Dict[int, int] = {}

    def new_eval(self, plan: Plan):
        """A new evaluation on the resident snapshot (pe_reset_plan)."""
        self.eng.ResetPlan()
        self.plan = plan
        self._reset_mirror()

    # -- plan replay ----------------------------------------------------------
    def _sync(self):
        p = self.plan
        for node in sorted(set(self._upd) | set(p.node_update)):
            have, want = self._upd.get(node, []), p.node_update.get(node, [])
            k = 0
            while k < len(have) and k < len(want) and have[k] == want[k]:
                k += 1
            for a in reversed(have[k:]):
                self.eng.PopUpdate(a)
            if want[k:]:
                self.eng.StopAllocs(want[k:])
            self._upd[node] = list(want)
        for node, allocs in p.node_allocation.items():
            seen = self._alloc_seen.get(node, 0)
            pre = p.node_preemptions.get(node, [])
            for a in allocs[seen:]:
                by = [r for r, pid in pre if pid == a.id]
                self.eng.Commit(self._tg_names.index(a.task_group), a.node_row, by)
            self._alloc_seen[node] = len(allocs)

    # -- scheduler.Stack (stack.go:23-32) ------------------------------------
    def SetNodes(self, rows):
        self._sync()
        return self.eng.SetNodes(rows)

    def SetJob(self, job):
        self._sync()
        self._tg_names = [g.name for g in job.task_groups]
        self.eng.SetJob(job)

    def Select(self, tg, options: Optional[SelectOptions] = None):
        self._sync()
        return self.eng.Select(tg, options)
