"""Benchmark: placements/sec for a count=1000 service job on a 10k-node cluster.

Workload (BASELINE.json configs[1]): 10,000 heterogeneous
synthetic nodes (seed 42) with 0-3 foreign allocs each, a count=1000 binpack
service job (cpu 500 / mem 256 / disk 150), limit = ceil(log2 n) = 14.

A step = one batch of E concurrent evaluations of that job (the NumSchedulers
worker model, nomad/config.go:468: each worker evaluates against its own
snapshot with its own shuffle), each placing all 1000 allocations with the exact
reference semantics (fused count loop, one workgroup per eval, pe_place_batch).
The snapshot and the E visit orders are resident in HBM before timing; result
records come back to the host inside the timed region.
value = E * placements / step time. The single-eval latency path (pe_place) is
reported beside it.

Multi-GPU: the windowed binpack path does not shard; each rank
runs its own batches on its own GPU (replicas, weak scaling).
"""
import argparse
import concurrent.futures as cf
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
# per node-evaluation: cls 4 + cap cpu/mem/disk 24 + used cpu/mem/disk 24
# + (job,tg) collisions 4 = 56 B read; perm entry 4 B; no per-node write. Node
# evaluations = the nodes the reference chain visits (Σ nodes_evaluated over the
# placements); the device evaluates each row once per launch (k_base) and
# gathers the result per visit position (k_chain), see DESIGN.md §3.
BYTES_PER_NODE_EVAL = 60


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--nodes", type=int, default=10000)
    p.add_argument("--count", type=int, default=1000)
    p.add_argument("--evals", type=int, default=4096, help="concurrent evaluations per step")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--sweep-nodes", type=int, default=1 << 24,
                   help="nodes of the scoring-sweep roofline measurement (0 = skip)")
    return p.parse_args()


def dist_init():
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


def reduce(pg, x, op):
    if pg is None:
        return x
    import torch
    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=op(pg))
    return float(t.item())


def cpu_eval_loop(nodes, allocs, job, seconds, seed0):
    from oracle.oracle import OracleGenericStack
    from nomad_amd import synth
    st = OracleGenericStack()
    st.SetState(nodes, allocs)
    rng = np.random.Generator(np.random.PCG64(seed0))
    perms = [rng.permutation(len(nodes)).astype(np.uint32) for _ in range(64)]
    placed = evals = 0
    t0 = time.perf_counter()
    while True:
        st.ResetPlan()
        st.SetJob(job)
        st.SetNodes(perms[evals % len(perms)])
        _, _, p, _ = st.PlaceArrays(0, job.task_groups[0].count)
        placed += p
        evals += 1
        if time.perf_counter() - t0 >= seconds:
            break
    return placed, evals, time.perf_counter() - t0


def cpu_baseline(nodes, allocs, job, seconds):
    """oracle/liboracle.so (C++ restatement of the reference chain) on host cores."""
    placed, evals, dt = cpu_eval_loop(nodes, allocs, job, seconds, 1000)
    one = {"value": placed / dt, "unit": "placements/s", "cores": 1, "kind": "port",
           "sample": "%d evals x count=%d on the %d-node cluster in %.1f s, 1 thread "
                     "(oracle/liboracle.so: C++ restatement of the reference iterator chain; "
                     "Go toolchain unavailable)" % (evals, job.task_groups[0].count, len(nodes), dt)}
    threads = min(16, os.cpu_count() or 1)
    with cf.ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(cpu_eval_loop, nodes, allocs, job, seconds / 2, 50000 * (t + 1)) for t in range(threads)]
        res = [f.result() for f in futs]
    tot = sum(r[0] for r in res)
    wall = max(r[2] for r in res)
    multi = {"value": tot / wall, "unit": "placements/s", "cores": threads, "kind": "port",
             "sample": "%d threads x independent evals for %.1f s (box CPU share)" % (threads, wall)}
    return one, multi


# Scoring sweep bytes per node (pe_last_sweep_bytes): 64 B NodeRec + 4 B folded
# score word (verdict, affinity index, spread values; 1 B verdict when the word
# does not apply: 73 B) + 4 B (job,tg) collisions + 4 B visit rank = 76 B.
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r01", "sweep_traffic.json")


def sweep_traffic(n, bytes_per_node):
    """HBM bytes per sweep launch from the committed rocprofv3 PMC passes
    (tools/pmc_traffic.py: FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md
    gfx950 correction), if they were taken on this workload."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, None
    if t.get("nodes") != n or t.get("bytes_per_node") != bytes_per_node:
        return None, None
    return t["bytes_per_launch"], os.path.relpath(TRAFFIC_FILE, ROOT)


def sweep_roofline(n, device, selects=6):
    """Scoring-sweep roofline: full-scan Selects (C3-like job: constraints,
    affinity, spread => limit MaxInt32) over an n-node columnar cluster in HBM.
    One Select = spread-table kernel + k_sweep over all rows + record merge."""
    from nomad_amd import synth, synth_columnar
    from nomad_amd.stack import GenericStack
    t0 = time.perf_counter()
    cs = synth_columnar.ColumnarState(n, seed=7, kind="c3")
    st = GenericStack(device=device)
    st.SetStateColumnar(cs)
    st.SetJob(synth.job_c3(1000))
    perm = np.random.Generator(np.random.PCG64(3)).permutation(n).astype(np.uint32)
    st.SetNodes(perm)
    setup_s = time.perf_counter() - t0
    times = []
    row = None
    for i in range(selects):
        t1 = time.perf_counter()
        r = st.SelectRaw(0)
        wall = time.perf_counter() - t1
        if i >= 1:
            times.append((st.last_kernel_ms(), wall))
        row = r.row
    kernel_ms = float(np.median([t[0] for t in times]))
    wall_ms = float(np.median([t[1] for t in times])) * 1000.0
    bpn = st.last_sweep_bytes()
    achieved = n * bpn / (kernel_ms / 1000.0) / 1e9
    st.close()
    traffic, source = sweep_traffic(n, bpn)
    return {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": source,
            "kernel": "k_sweep<256,aux> + k_sweep_merge",
            "nodes": n, "bytes_per_node_eval": bpn, "kernel_ms": kernel_ms,
            "select_wall_ms": wall_ms, "nodes_scored_per_s": n / (kernel_ms / 1000.0),
            "winner_row": row, "setup_s": setup_s}


def main():
    args = parse()
    rank, world, local, pg = dist_init()
    from nomad_amd import synth
    from nomad_amd.stack import GenericStack

    nodes, allocs = synth.cluster_c2(args.nodes, seed=42)
    job = synth.job_c2(args.count)
    E = args.evals
    rng_base = 1000 + 104729 * rank
    orders = np.stack([synth.shuffle(len(nodes), rng_base + e) if e < 64 else
                       np.random.Generator(np.random.PCG64(rng_base + e)).permutation(len(nodes)).astype(np.uint32)
                       for e in range(E)])

    st = GenericStack(device=local)
    st.SetState(nodes, allocs)
    st.SetJob(job)
    st.StageOrders(orders)

    def step():
        # results land in the engine's page-locked buffer (zero-copy views)
        rows, scores, evaluated, placed = st.PlaceBatch(0, args.count, copy=False)
        return int(placed.sum()), st.last_kernel_ms(), st.last_phase_ms()

    for _ in range(args.warmup):
        step()
    barrier(pg)
    t0 = time.perf_counter()
    placed = 0
    kernel_ms = 0.0
    phases = np.zeros(4)
    for _ in range(args.steps):
        p, k, ph = step()
        placed += p
        kernel_ms += k
        phases += ph
    elapsed = time.perf_counter() - t0
    # every step evaluates the same staged orders: node evaluations per launch
    # from the last step's records (outside the timed region)
    evaluated = int(st.PlaceBatch(0, args.count, copy=False)[2].sum(dtype=np.uint64)) * args.steps
    barrier(pg)
    elapsed = reduce(pg, elapsed, lambda d: d.ReduceOp.MAX)
    total_placed = reduce(pg, placed, lambda d: d.ReduceOp.SUM)

    # single-evaluation latency (pe_place on the stack's own plan)
    lat = GenericStack(device=local)
    lat.SetState(nodes, allocs)
    lat_times = []
    for i in range(5):
        lat.ResetPlan()
        lat.SetJob(job)
        lat.SetNodes(orders[i % E])
        t1 = time.perf_counter()
        lat.PlaceArrays(0, args.count)
        lat_times.append(time.perf_counter() - t1)
    single = args.count / float(np.median(lat_times[1:]))
    single_kernel_ms = lat.last_kernel_ms()

    if rank == 0:
        value = total_placed / elapsed
        avg_kernel_s = kernel_ms / 1000.0 / args.steps
        evals_per_launch = evaluated / args.steps
        algo_bytes = evals_per_launch * BYTES_PER_NODE_EVAL
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
            "config": {"workload": "C2: %d concurrent evals/step x service job count=%d, %d heterogeneous "
                                   "nodes, binpack, limit 14" % (E, args.count, args.nodes),
                       "evals_per_step": E,
                       "parallelism": "replicas x%d (windowed binpack does not shard)" % world},
            "step_phases_ms": dict(zip(("host_prep", "kernel", "d2h_results", "call_total"),
                                       (phases / args.steps).round(4).tolist())),
            "single_eval": {"placements_per_s": single, "kernel_ms": single_kernel_ms,
                            "note": "one eval, pe_place fused count loop, host call included"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                         "kernel": "k_base + k_chain", "kernel_ms": avg_kernel_s * 1000.0,
                         "node_evals_per_launch": evals_per_launch,
                         "bytes_per_node_eval": BYTES_PER_NODE_EVAL},
        }
        if args.sweep_nodes > 0:
            line["sweep_roofline"] = sweep_roofline(args.sweep_nodes, local)
        if not args.no_cpu:
            one, multi = cpu_baseline(nodes, allocs, job, args.cpu_seconds)
            line["cpu_baseline"] = one
            line["cpu_baseline_multicore"] = multi
        print(json.dumps(line))
    st.close()
    lat.close()
    if pg is not None:
        pg.destroy_process_group()


if __name__ == "__main__":
    main()
