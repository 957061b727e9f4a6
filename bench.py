"""Benchmark: placements/sec for a count=1000 service job on a 10k-node cluster.

Workload (BASELINE.json configs[1]): 10,000 heterogeneous
synthetic nodes (seed 42) with 0-3 foreign allocs each, a count=1000 binpack
service job (cpu 500 / mem 256 / disk 150), limit = ceil(log2 n) = 14.

A step = one evaluation's placement pass: ResetPlan (fresh EvalContext on the
HBM-resident snapshot) + SetJob + SetNodes (seeded shuffle) + the fused count
loop (1000 Select -> AppendAlloc on device). The snapshot upload (pe_set_state)
happens once before timing: inputs are resident in HBM.

Multi-GPU: the windowed binpack path does not shard: each rank
runs independent evaluations on its own GPU (replicas, weak scaling).
value = placements completed by all ranks / max-over-ranks wall time.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
BYTES_PER_NODE_EVAL = 56       # cls 4 + cap 3x8 + used 3x8 + coll 4 (56 B read, no score write)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--nodes", type=int, default=10000)
    p.add_argument("--count", type=int, default=1000)
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    return p.parse_args()


def dist_init(n):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        pg = dist
    return rank, world, local, pg


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allmax(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def allsum(pg, x):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def cpu_baseline(nodes, allocs, job, seconds):
    """Oracle (C++ restatement of the reference chain), 1 thread, bounded sample."""
    from oracle.oracle import OracleGenericStack
    from nomad_amd import synth
    st = OracleGenericStack()
    st.SetState(nodes, allocs)
    placed, evals = 0, 0
    t0 = time.perf_counter()
    while True:
        st.ResetPlan()
        st.SetJob(job)
        st.SetNodes(list(synth.shuffle(len(nodes), 1000 + evals)))
        rows, _, p, _ = st.PlaceArrays(0, job.task_groups[0].count)
        placed += p
        evals += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": placed / dt, "unit": "placements/s", "cores": 1, "kind": "port",
            "sample": "%d evals x count=%d on the same %d-node cluster in %.1f s (oracle/liboracle.so, "
                      "C++ restatement of the reference iterator chain; Go toolchain unavailable)"
                      % (evals, job.task_groups[0].count, len(nodes), dt)}


def main():
    args = parse()
    rank, world, local, pg = dist_init(args.gpus)
    from nomad_amd import synth
    from nomad_amd.stack import GenericStack

    nodes, allocs = synth.cluster_c2(args.nodes, seed=42)
    job = synth.job_c2(args.count)
    perms = [synth.shuffle(len(nodes), 1000 + 7919 * rank + i) for i in range(args.warmup + args.steps)]

    st = GenericStack(device=local)
    st.SetState(nodes, allocs)

    def step(i):
        st.ResetPlan()
        st.SetJob(job)
        st.SetNodes(perms[i])
        rows, scores, placed, raw = st.PlaceArrays(0, args.count)
        evaluated = int(raw["nodes_evaluated"][:max(placed, 1)].sum())
        return placed, evaluated, st.last_kernel_ms()

    for i in range(args.warmup):
        step(i)
    barrier(pg)
    t0 = time.perf_counter()
    placed = evaluated = 0
    kernel_ms = 0.0
    for i in range(args.steps):
        p, e, k = step(args.warmup + i)
        placed += p
        evaluated += e
        kernel_ms += k
    elapsed = time.perf_counter() - t0
    barrier(pg)
    elapsed = allmax(pg, elapsed)
    total_placed = allsum(pg, placed)

    if rank == 0:
        value = total_placed / elapsed
        avg_kernel_s = kernel_ms / 1000.0 / args.steps
        algo_bytes = evaluated / args.steps * BYTES_PER_NODE_EVAL
        achieved = algo_bytes / avg_kernel_s / 1e9
        line = {
            "metric": "placements/sec (count=1000 service job, 10k nodes, binpack)",
            "value": value,
            "unit": "placements/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1000.0,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64+f64",
            "data": "synthetic (seeded 10k-node cluster, SURVEY.md §8d C2)",
            "config": {"workload": "C2: service job count=%d, %d heterogeneous nodes, binpack, limit 14"
                                   % (args.count, args.nodes),
                       "parallelism": "replicas x%d (windowed binpack does not shard)" % world},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "k_place<256>", "kernel_ms": avg_kernel_s * 1000.0,
                         "node_evals_per_launch": evaluated / args.steps,
                         "bytes_per_node_eval": BYTES_PER_NODE_EVAL},
        }
        if not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(nodes, allocs, job, args.cpu_seconds)
        print(json.dumps(line))
    st.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
