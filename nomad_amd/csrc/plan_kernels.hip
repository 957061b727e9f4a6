// Plan applier fit check on gfx950: evaluateNodePlan (nomad/plan_apply.go:611-674)
// → AllocsFit(node, proposed, nil, checkDevices=true) (nomad/structs/funcs.go:148-211)
// for every node of a plan, one wavefront per plan node, four per workgroup.
//
// Per plan node the wave
//   1. applies the node checks in the reference's order (evict-only plan ⇒ fit,
//      plan_apply.go:614-616; missing / not ready / ineligible, :627-633);
//   2. walks the node's snapshot allocs (contiguous 32-byte records) minus the
//      plan's removals (binary search in the node's sorted removal list;
//      RemoveAllocs, funcs.go:47-64) plus the plan's allocs, skipping terminal
//      ones, and sums cpu / memory / disk (ComparableResources.Add);
//   3. stages the static node keys and the counted allocs' keys into a
//      wave-private LDS buffer (global scratch when a node exceeds it) and runs
//      one pairwise pass that answers core overlap, core subset, port collision
//      and device oversubscription together (plan_types.h);
//   4. writes the first failing dimension in AllocsFit order.
// HBM-bound integer work: no MFMA. Bytes per plan node are the records and keys
// read plus one reason byte (pe_planner_last_bytes).
#include <hip/hip_runtime.h>
#include "../../include/nomad_pe.h"
#include "plan_types.h"

namespace pa {

__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void wave_sync_global() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
}

__device__ __forceinline__ int64_t wave_sum64(int64_t v) {
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v >> 32), off);
        v += (int64_t)((uint64_t)hi << 32 | lo);
    }
    return v;
}

__device__ __forceinline__ bool removed(const uint32_t* rm, uint32_t n, uint32_t q) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t v = rm[mid];
        if (v == q) return true;
        if (v < q) lo = mid + 1; else hi = mid;
    }
    return false;
}

// Stage one counted alloc: sums and keys.
__device__ __forceinline__ void take(const AllocRec& ar, const uint64_t* keys, uint64_t* buf, uint32_t* fill,
                                     int64_t& cpu, int64_t& mem, int64_t& disk, bool& bad) {
    cpu += ar.cpu;
    mem += ar.mem;
    disk += ar.disk;
    bad |= ar.bad_port != 0;
    if (ar.n_keys) {
        const uint32_t base = atomicAdd(fill, (uint32_t)ar.n_keys);
        for (uint32_t k = 0; k < ar.n_keys; k++) buf[base + k] = keys[ar.key_off + k];
    }
}

__device__ uint8_t fit_node(const PlanArgs& a, const PlanNodeRec& pn, const NodeRec& nd, uint32_t lane,
                            uint64_t* lds_buf, uint32_t* fill) {
    const bool global = pn.scratch_off != kNone;
    uint64_t* buf = global ? a.scratch + pn.scratch_off : lds_buf;
    for (uint32_t i = lane; i < nd.n_keys; i += 64) buf[i] = a.node_keys[nd.key_off + i];
    if (lane == 0) *fill = nd.n_keys;
    wave_sync_lds();

    int64_t cpu = 0, mem = 0, disk = 0;
    bool bad = false;
    const uint32_t* rm = a.rm + pn.rm_off;
    for (uint32_t i = lane; i < nd.alloc_cnt; i += 64) {
        const uint32_t q = nd.alloc_off + i;
        const AllocRec ar = a.pool[q];
        if (ar.terminal || (pn.rm_cnt && removed(rm, pn.rm_cnt, q))) continue;
        take(ar, a.pool_keys, buf, fill, cpu, mem, disk, bad);
    }
    for (uint32_t i = lane; i < pn.place_cnt; i += 64) {
        const AllocRec ar = a.pallocs[pn.place_off + i];
        if (ar.terminal) continue;
        take(ar, a.pkeys, buf, fill, cpu, mem, disk, bad);
    }
    if (global) wave_sync_global(); else wave_sync_lds();
    const uint32_t k = *fill;
    cpu = wave_sum64(cpu);
    mem = wave_sum64(mem);
    disk = wave_sum64(disk);
    bad = __ballot(bad) != 0;

    // One pairwise pass: for each staged key, look for an earlier equal key of
    // the same kind (a second holder) and for its AVAIL / NODE twin (kind + 1).
    bool core_dup = false, core_missing = false, port_hit = false, dev_dup = false;
    const uint32_t trips = (k + 63) & ~63u;
    for (uint32_t i = lane; i < trips; i += 64) {
        const bool valid = i < k;
        const uint64_t x = valid ? buf[i] : ~0ull;
        const uint32_t kx = (uint32_t)(x >> 60);
        const uint64_t vx = x & kValMask;
        bool dupe = false, twin = false;
        if (valid && (kx & 1u) == 0) {
            for (uint32_t j = 0; j < k; j++) {
                const uint64_t y = buf[j];
                if ((y & kValMask) == vx) {
                    const uint32_t ky = (uint32_t)(y >> 60);
                    dupe |= (ky == kx) & (j < i);
                    twin |= ky == kx + 1;
                }
            }
            if (kx == K_CORE_USED) { core_dup |= dupe; core_missing |= !twin; }
            else if (kx == K_PORT_USED) port_hit |= dupe | twin;
            else if (kx == K_DEV_USED) dev_dup |= dupe & twin;
        }
    }
    core_dup = __ballot(core_dup) != 0;
    core_missing = __ballot(core_missing) != 0;
    port_hit = __ballot(port_hit) != 0;
    dev_dup = __ballot(dev_dup) != 0;

    // AllocsFit order (funcs.go:173-208, Superset structs.go:3891-3905)
    if (core_dup) return PE_PLAN_CORES;
    if (nd.cpu < cpu) return PE_PLAN_CPU;
    if (nd.has_cores && core_missing) return PE_PLAN_CORES;
    if (nd.mem < mem) return PE_PLAN_MEMORY;
    if (nd.disk < disk) return PE_PLAN_DISK;
    if (nd.setnode_collide || bad || port_hit) return PE_PLAN_PORTS;
    if (dev_dup) return PE_PLAN_DEVICES;
    return PE_PLAN_FIT;
}

__global__ void __launch_bounds__(64 * kWaves) k_plan_eval(PlanArgs a) {
    __shared__ uint64_t lds_keys[kWaves][kLdsKeys];
    __shared__ uint32_t fill[kWaves];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t p = blockIdx.x * kWaves + w;
    if (p >= a.n_plan) return;   // whole wave exits; no workgroup barrier below
    const PlanNodeRec pn = a.pn[p];
    uint8_t r;
    if (pn.place_cnt == 0) {
        r = PE_PLAN_FIT;                       // evict-only (plan_apply.go:614-616)
    } else if (pn.row == kNone) {
        r = PE_PLAN_NODE_MISSING;
    } else {
        const NodeRec nd = a.nodes[pn.row];
        if (!nd.ready) r = PE_PLAN_NODE_NOT_READY;
        else if (!nd.eligible) r = PE_PLAN_NODE_INELIGIBLE;
        else r = fit_node(a, pn, nd, lane, lds_keys[w], &fill[w]);
    }
    if (lane == 0) a.reason[p] = r;
}

}  // namespace pa

hipError_t pe_launch_plan_eval(const pa::PlanArgs* a, hipStream_t st) {
    if (a->n_plan == 0) return hipSuccess;
    const uint32_t blocks = (a->n_plan + pa::kWaves - 1) / pa::kWaves;
    hipLaunchKernelGGL(pa::k_plan_eval, dim3(blocks), dim3(64 * pa::kWaves), 0, st, *a);
    return hipGetLastError();
}
