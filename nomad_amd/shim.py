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
caller gets the device loop. structs.Plan keeps NodeAllocation as a map of
per-node lists, so plan order across nodes is not recoverable; new placements
are replayed node by node, in list order within a node. Commits of different
nodes commute (resource sums, collision counts, device and core picks are per
node), and between two Selects the caller appends at most the last Select's
placement, which is the one the speculation checks.

EvalEligibility: the Go EvalContext's memo is read by the caller after the
Selects (createBlockedEval, generic_sched.go:177-203), so after every engine
Select the shim mirrors the entries that changed (pe_get_eligibility with
changed_only) into `ctx_eligibility`.

PE_EUNSUPPORTED: the Select is answered by `fallback`, the reference chain on
the same EvalContext (here the oracle restatement). Before it runs, the
fallback takes the engine's StaticIterator offset and LimitIterator limit
(pe_get_cursor), the SpreadIterator.SetTaskGroup of every group the engine
has selected for, and the ctx memo; afterwards the engine takes the chain's
offset, limit, group and memo back (pe_set_cursor, pe_put_eligibility), so
later Selects continue exactly where the reference chain would be.
`Plan` here is the subset of structs.Plan (structs.go:10540-10714) the
protocol reads.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

from .stack import GenericStack, SelectOptions, Unsupported


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
    evaluations (`new_eval` = NewEvalContext). `fallback`: the reference chain
    (a stack with the same interface, given the same snapshot) that answers
    PE_EUNSUPPORTED Selects."""

    def __init__(self, engine: GenericStack, plan: Plan, fallback=None):
        self.eng = engine
        self.fallback = fallback
        self.plan = plan
        self._tg_names: List[str] = []
        self.fallback_selects = 0
        self._reset_mirror()

    def _reset_mirror(self):
        self._upd: Dict[int, List[int]] = {}
        self._alloc_seen: Dict[int, int] = {}
        self.ctx_eligibility = {"job": {}, "tgs": {}}
        self._seen_tgs: List[str] = []     # groups the engine selected for, in order
        self._fb_tgs = set()               # groups the fallback's SpreadIterator has seen

    def _stacks(self):
        return (self.eng,) if self.fallback is None else (self.eng, self.fallback)

    def new_eval(self, plan: Plan):
        """A new evaluation on the resident snapshot (pe_reset_plan)."""
        for st in self._stacks():
            st.ResetPlan()
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
                for st in self._stacks():
                    st.PopUpdate(a)
            if want[k:]:
                for st in self._stacks():
                    st.StopAllocs(want[k:])
            self._upd[node] = list(want)
        for node, allocs in p.node_allocation.items():
            seen = self._alloc_seen.get(node, 0)
            pre = p.node_preemptions.get(node, [])
            for a in allocs[seen:]:
                by = [r for r, pid in pre if pid == a.id]
                for st in self._stacks():
                    st.Commit(self._tg_names.index(a.task_group), a.node_row, by)
            self._alloc_seen[node] = len(allocs)

    def _mirror_eligibility(self, delta):
        self.ctx_eligibility["job"].update(delta["job"])
        for tg, m in delta["tgs"].items():
            self.ctx_eligibility["tgs"].setdefault(tg, {}).update(m)

    # -- scheduler.Stack (stack.go:23-32) ------------------------------------
    def SetNodes(self, rows):
        self._sync()
        if self.fallback is not None:
            self.fallback.SetNodes(rows)
        return self.eng.SetNodes(rows)

    def SetJob(self, job):
        self._sync()
        self._tg_names = [g.name for g in job.task_groups]
        if self.fallback is not None:
            self.fallback.SetJob(job)
        self.eng.SetJob(job)

    def Select(self, tg, options: Optional[SelectOptions] = None):
        self._sync()
        name = tg if isinstance(tg, str) else self._tg_names[tg]
        try:
            r = self.eng.Select(tg, options)
        except Unsupported:
            if self.fallback is None:
                raise
            return self._fallback_select(tg, name, options)
        if name not in self._seen_tgs:
            self._seen_tgs.append(name)
        self._mirror_eligibility(self.eng.Eligibility(changed_only=True))
        return r

    def _fallback_select(self, tg, name, options):
        """The reference chain answers; both sides then hold the same iterator
        state, plan and memo (pe_get_cursor / pe_set_cursor / pe_put_eligibility)."""
        fb = self.fallback
        off, lim = self.eng.GetCursor()
        fb.SetCursor(off, lim)
        for g in self._seen_tgs:            # SpreadIterator.SetTaskGroup the engine has done
            if g not in self._fb_tgs:
                fb.SetCursor(off, lim, g)
                self._fb_tgs.add(g)
        fb.PutEligibility(self.ctx_eligibility)
        r = fb.Select(tg, options)
        self.fallback_selects += 1
        self._fb_tgs.add(name)
        self.ctx_eligibility = fb.Eligibility()
        self.ctx_eligibility.pop("escaped", None)
        self.eng.PutEligibility(self.ctx_eligibility)
        off, lim = fb.GetCursor()
        self.eng.SetCursor(off, lim, name)
        if name not in self._seen_tgs:
            self._seen_tgs.append(name)
        return r
