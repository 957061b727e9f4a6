"""Multi-GPU sharding of the placement path, one process per GPU.

Every rank holds the same snapshot, job, SetNodes list and plan (replicated
state, ~64 B per node in HBM); what is split is the work:

* SystemScheduler (scheduler_system.go:283-425): each node's single-node Select
  is independent, so the SetNodes list is cut into contiguous ranges, one per
  rank, with no data-path collective (`system_place_sharded`).
* Full-pass Selects (affinities / spreads, limit MaxInt32): each rank sweeps the
  snapshot rows it owns into an 80-byte record of the LimitIterator +
  MaxScoreIterator state (pe_select_shard); one all-gather of the records per
  placement, then every rank resolves the same winner (pe_select_merge) and
  applies the same commit (`ShardedFullScan`). The all-gather is the one
  exchange step of the path and is latency-bound; `last_exchange_us` reports it.
* Windowed binpack (limit = ceil(log2 n)) does not shard: ranks run replicas.

The collective is torch.distributed's all_gather: RCCL over xGMI on GPU tensors
(backend "nccl"), gloo on CPU tensors for the multi-process CPU tests. On GPUs
the whole sharded count loop also runs inside the engine (`device_place`,
pe_place_sharded): each rank's sweep merges its workgroup records into one
80-byte record in the same launch, the engine's own RCCL communicator
all-gathers the N records on the engine stream between k_sweep and
k_sweep_step, so no placement returns to the host. `host_comm_init` runs the
same engine loop over a torch.distributed transport instead.
"""
from __future__ import annotations

import time
from typing import List, Optional, Sequence, Tuple

import numpy as np

REC_BYTES = 80   # sizeof(pe_shard_rec)


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [begin, end) of n items owned by `rank`."""
    return n * rank // world, n * (rank + 1) // world


def all_gather_bytes(dist, payload: bytes, device=None) -> List[bytes]:
    """All-gather one fixed-size byte record per rank (rank order)."""
    import torch
    t = torch.tensor(np.frombuffer(payload, dtype=np.uint8).copy())
    if device is not None:
        t = t.to(device)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [bytes(o.cpu().numpy().tobytes()) for o in outs]


class ShardedFullScan:
    """Full-pass Selects of one evaluation split over the ranks of `dist`.

    `stack` is a GenericStack (or any object with SelectShard / SelectMerge /
    Commit) on which SetState, SetJob and SetNodes were called identically on
    every rank. With dist None (or world 1) it degenerates to local Selects."""

    def __init__(self, stack, n_rows: int, dist=None, device=None):
        self.stack = stack
        self.dist = dist
        self.rank = dist.get_rank() if dist is not None else 0
        self.world = dist.get_world_size() if dist is not None else 1
        self.device = device
        self.rows = shard_range(n_rows, self.rank, self.world)
        self.last_exchange_us = 0.0

    def Select(self, tg):
        rec = self.stack.SelectShard(tg, *self.rows)
        if self.world > 1:
            t0 = time.perf_counter()
            recs = all_gather_bytes(self.dist, rec, self.device)
            self.last_exchange_us = (time.perf_counter() - t0) * 1e6
        else:
            recs = [rec]
        return self.stack.SelectMerge(tg, recs)

    def Place(self, tg, count: int):
        """The count loop (generic_sched.go:493-649): Select, then the same
        Plan.AppendAlloc on every rank; stops at the first nil Select."""
        out = []
        for _ in range(count):
            r = self.Select(tg)
            out.append(r)
            if r.row < 0:
                break
            self.stack.Commit(tg, r.row)
        return out


def comm_init(stack, dist=None):
    """Join every rank's engine into one RCCL communicator: rank 0 draws the
    unique id (pe_comm_unique_id) and torch.distributed broadcasts it."""
    from .stack import comm_unique_id
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    uid = comm_unique_id() if rank == 0 else bytes(128)
    if world > 1:
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    stack.CommInit(world, rank, uid)
    return rank, world


def host_comm_init(stack, dist):
    """Join every rank's engine over torch.distributed instead of RCCL
    (pe_comm_init_host): the engine hands each placement's 80-byte record to
    an all-gather on CPU tensors (gloo), e.g. ranks without an RCCL path, or
    the one-GPU rehearsal of the per-GPU processes."""
    world = dist.get_world_size()
    rank = dist.get_rank()
    stack.CommInitHost(world, rank, lambda rec: all_gather_bytes(dist, rec))
    return rank, world


def device_place(stack, tg, count: int, n_rows: int, rank: int, world: int):
    """The sharded full-pass count loop inside the engine (pe_place_sharded)."""
    b, e = shard_range(n_rows, rank, world)
    return stack.PlaceSharded(tg, count, b, e)


def system_place_sharded(stack, rows: Sequence[int], rank: int, world: int, tg=0, view: bool = False):
    """SystemScheduler placements over this rank's range of the SetNodes list.
    Returns (begin, end, scores, statuses, placed) for the range; with `view`
    the arrays are the engine's staging (valid until its next SystemPlace)."""
    rows = np.asarray(rows, dtype=np.uint32)
    b, e = shard_range(len(rows), rank, world)
    stack.SetNodes(rows[b:e])
    score, status, placed = stack.SystemPlaceView(tg) if view else stack.SystemPlace(tg)
    return b, e, score, status, placed


def shard_plan(nodes, allocs, plan, rank: int, world: int):
    """Plan applier (plan_apply.go:439-582) over GPUs: evaluateNodePlan is
    independent per node, so each rank owns a contiguous range of the node
    list, holds only those nodes and their allocs as its resident snapshot, and
    evaluates the plan nodes that fall in it. Plan nodes outside every range
    (nodes that do not exist) go to the last rank. No data-path collective:
    the per-node outcomes are concatenated by whoever assembles the PlanResult.
    Returns (nodes, allocs, plan) of this rank."""
    from .plan import Plan
    b, e = shard_range(len(nodes), rank, world)
    mine = {n.id for n in nodes[b:e]}
    known = {n.id for n in nodes}

    def owns(nid):
        return nid in mine or (rank == world - 1 and nid not in known)

    sub = Plan(node_update={k: v for k, v in plan.node_update.items() if owns(k)},
               node_allocation={k: v for k, v in plan.node_allocation.items() if owns(k)},
               node_preemptions={k: v for k, v in plan.node_preemptions.items() if owns(k)},
               all_at_once=plan.all_at_once)
    return nodes[b:e], [a for a in allocs if a.node_id in mine], sub
