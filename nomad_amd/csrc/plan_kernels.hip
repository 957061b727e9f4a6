// Plan applier fit check on gfx950: evaluateNodePlan (nomad/plan_apply.go:611-674)
// → AllocsFit(node, proposed, nil, checkDevices=true) (nomad/structs/funcs.go:148-211)
// for every node of a plan.
//
// k_plan_eval<G>   a group of G lanes per plan node (default 4: sixteen nodes per
//                  wavefront), keys staged in a per-node LDS buffer (ds_* only).
// k_plan_eval_big  one wavefront per plan node whose key bound exceeds that
//                  buffer (nodes with hundreds of cores / ports), keys staged in
//                  global scratch. Rare; listed by the host.
//
// Per plan node a group
//   1. applies the node checks in the reference's order (evict-only plan ⇒ fit,
//      plan_apply.go:614-616; missing / not ready / ineligible, :627-633);
//   2. walks the node's snapshot allocs (contiguous 32-byte records) minus the
//      plan's removals (binary search in the node's sorted removal list;
//      RemoveAllocs, funcs.go:47-64) plus the plan's allocs, skipping terminal
//      ones, and sums cpu / memory / disk (ComparableResources.Add);
//   3. folds held cores with id < 64 into an LDS mask with atomicOr (overlap =
//      a bit already set, funcs.go:166-175; subset test against the node's
//      available-core mask, structs.go:3896-3898), stages every other key and
//      runs one pairwise pass that answers the remaining core, port-collision
//      and device-oversubscription questions together (plan_types.h);
//   4. writes the first failing dimension in AllocsFit order.
// HBM/latency-bound integer work: no MFMA. Bytes per plan node are the records
// and keys read plus one reason byte (pe_planner_last_bytes).
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

template <int G>
__device__ __forceinline__ int64_t group_sum64(int64_t v) {
    for (int off = G / 2; off > 0; off >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)((uint64_t)v >> 32), off);
        v += (int64_t)((uint64_t)hi << 32 | lo);
    }
    return v;
}

template <int G>
__device__ __forceinline__ bool group_any(bool x, uint32_t lane) {
    const uint64_t m = __ballot(x);
    if (G == 64) return m != 0;
    return ((m >> (lane & ~(uint32_t)(G - 1))) & ((1ull << (G & 63)) - 1)) != 0;
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

struct Acc {
    int64_t cpu = 0, mem = 0, disk = 0;
    bool bad = false, core_dup = false, core_missing = false;
};

// Stage one counted alloc's keys: cores < 64 into the mask, the rest into buf.
template <typename Buf>
__device__ __forceinline__ void take_keys(uint32_t key_off, uint32_t n_keys, const uint64_t* keys, Buf buf,
                                          uint32_t* fill, unsigned long long* cmask, uint64_t node_mask, Acc& acc) {
    if (!n_keys) return;
    const uint32_t base = atomicAdd(fill, n_keys);
    for (uint32_t k = 0; k < n_keys; k++) {
        uint64_t key = keys[key_off + k];
        const uint64_t v = key & kValMask;
        if ((uint32_t)(key >> 60) == K_CORE_USED && v < 64) {
            const unsigned long long bit = 1ull << v;
            const unsigned long long old = atomicOr(cmask, bit);
            acc.core_dup |= (old & bit) != 0;
            acc.core_missing |= (node_mask & bit) == 0;
            key = kHole;
        }
        buf[base + k] = key;
    }
}

// A snapshot alloc: sums, masked cores, keys.
template <typename Buf>
__device__ __forceinline__ void take(const AllocRec& ar, const uint64_t* keys, Buf buf, uint32_t* fill,
                                     unsigned long long* cmask, uint64_t node_mask, Acc& acc) {
    acc.cpu += ar.cpu;
    acc.mem += ar.mem;
    acc.disk += ar.disk;
    acc.bad |= ar.bad_port != 0;
    take_keys(ar.key_off, ar.n_keys, keys, buf, fill, cmask, node_mask, acc);
}

// One plan node as the kernel sees it.
struct PlanNode {
    uint32_t row, place_off, place_cnt, rm_off, rm_cnt;
    bool big;
};

__device__ __forceinline__ PlanNode plan_node(const PlanArgs& a, uint32_t p) {
    PlanNode n;
    const uint32_t row = a.prow[p];
    n.big = row != kNone && (row & kBigRow) != 0;
    n.row = row == kNone ? kNone : row & ~kBigRow;
    n.place_off = a.poff[p];
    n.place_cnt = a.poff[p + 1] - n.place_off;
    n.rm_off = a.rmoff ? a.rmoff[p] : 0;
    n.rm_cnt = a.rmoff ? a.rmoff[p + 1] - n.rm_off : 0;
    return n;
}

template <int G, bool GLOBAL, typename Buf>
__device__ __forceinline__ uint8_t fit_node(const PlanArgs& a, const PlanNode& pn, const NodeRec& nd,
                                            uint32_t lane, Buf buf, uint32_t* fill, unsigned long long* cmask) {
    const uint32_t gl = lane & (G - 1);
    for (uint32_t i = gl; i < nd.n_keys; i += G) buf[i] = a.node_keys[nd.key_off + i];
    if (gl == 0) { *fill = nd.n_keys; *cmask = 0; }
    wave_sync_lds();

    Acc acc;
    const uint32_t* rm = a.rm + pn.rm_off;
    for (uint32_t i = gl; i < nd.alloc_cnt; i += G) {
        const uint32_t q = nd.alloc_off + i;
        const AllocRec ar = a.pool[q];
        if (ar.terminal || (pn.rm_cnt && removed(rm, pn.rm_cnt, q))) continue;
        take(ar, a.pool_keys, buf, fill, cmask, nd.core_mask, acc);
    }
    for (uint32_t c = nd.ext_head; c != kNone;) {   // allocs committed since the last compaction
        const Chunk ch = a.chunks[c];
        for (uint32_t i = gl; i < ch.cnt; i += G) {
            const uint32_t q = ch.off + i;
            const AllocRec ar = a.pool[q];
            if (ar.terminal || (pn.rm_cnt && removed(rm, pn.rm_cnt, q))) continue;
            take(ar, a.pool_keys, buf, fill, cmask, nd.core_mask, acc);
        }
        c = ch.next;
    }
    for (uint32_t i = gl; i < pn.place_cnt; i += G) {
        const PlanAllocRec ar = a.pallocs[pn.place_off + i];
        if (ar.terminal) continue;
        const PlanRes r = a.pres[ar.res];
        acc.cpu += r.cpu;
        acc.mem += r.mem;
        acc.disk += r.disk;
        acc.bad |= ar.bad_port != 0;
        take_keys(ar.key_off, ar.n_keys, a.pkeys, buf, fill, cmask, nd.core_mask, acc);
    }
    if (GLOBAL) wave_sync_global(); else wave_sync_lds();
    const uint32_t k = *fill;
    const int64_t cpu = group_sum64<G>(acc.cpu);
    const int64_t mem = group_sum64<G>(acc.mem);
    const int64_t disk = group_sum64<G>(acc.disk);

    // One pairwise pass: for each staged key, look for an earlier equal key of
    // the same kind (a second holder) and for its AVAIL / NODE twin (kind + 1).
    bool port_hit = false, dev_dup = false;
    const uint32_t trips = (k + G - 1) & ~(uint32_t)(G - 1);
    for (uint32_t i = gl; i < trips; i += G) {
        const bool valid = i < k;
        const uint64_t x = valid ? buf[i] : kHole;
        const uint32_t kx = (uint32_t)(x >> 60);
        const uint64_t vx = x & kValMask;
        if ((kx & 1u) == 0) {
            bool dupe = false, twin = false;
#pragma unroll 4
            for (uint32_t j = 0; j < k; j++) {
                const uint64_t y = buf[j];
                const bool eq = (y & kValMask) == vx;
                const uint32_t ky = (uint32_t)(y >> 60);
                dupe |= eq & (ky == kx) & (j < i);
                twin |= eq & (ky == kx + 1);
            }
            if (kx == K_CORE_USED) { acc.core_dup |= dupe; acc.core_missing |= !twin; }
            else if (kx == K_PORT_USED) port_hit |= dupe | twin;
            else if (kx == K_DEV_USED) dev_dup |= dupe & twin;
        }
    }
    const bool core_dup = group_any<G>(acc.core_dup, lane);
    const bool core_missing = group_any<G>(acc.core_missing, lane);
    const bool bad = group_any<G>(acc.bad, lane);
    port_hit = group_any<G>(port_hit, lane);
    dev_dup = group_any<G>(dev_dup, lane);

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

// Node checks ahead of AllocsFit; returns true when the fit check must run.
__device__ __forceinline__ bool precheck(const PlanArgs& a, const PlanNode& pn, NodeRec* nd, uint8_t* r) {
    if (pn.place_cnt == 0) { *r = PE_PLAN_FIT; return false; }            // evict-only (plan_apply.go:614-616)
    if (pn.row == kNone) { *r = PE_PLAN_NODE_MISSING; return false; }
    *nd = a.nodes[pn.row];
    if (!nd->ready) { *r = PE_PLAN_NODE_NOT_READY; return false; }
    if (!nd->eligible) { *r = PE_PLAN_NODE_INELIGIBLE; return false; }
    return true;
}

template <int G>
__global__ void __launch_bounds__(64 * kWaves) k_plan_eval(PlanArgs a) {
    constexpr int NB = nodes_per_block(G);
    constexpr uint32_t NK = lds_keys(G);
    __shared__ uint64_t keys[NB][NK];
    __shared__ uint32_t fill[NB];
    __shared__ unsigned long long cmask[NB];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t slot = threadIdx.x / G;
    const uint32_t first = blockIdx.x * NB + (threadIdx.x >> 6) * (64 / G);
    if (first >= a.n_plan) return;   // whole wave idle; no workgroup barrier below
    const uint32_t p = blockIdx.x * NB + slot;
    if (p >= a.n_plan) return;       // group-uniform: the group's lanes leave together
    const PlanNode pn = plan_node(a, p);
    NodeRec nd;
    uint8_t r;
    if (pn.big) return;              // k_plan_eval_big writes this node's reason
    if (precheck(a, pn, &nd, &r))
        r = fit_node<G, false>(a, pn, nd, lane, keys[slot], &fill[slot], &cmask[slot]);
    if ((lane & (G - 1)) == 0) a.reason[p] = r;
}

__global__ void __launch_bounds__(64) k_plan_eval_big(PlanArgs a) {
    __shared__ uint32_t fill;
    __shared__ unsigned long long cmask;
    const uint32_t lane = threadIdx.x;
    const BigNode b = a.big[blockIdx.x];
    const PlanNode pn = plan_node(a, b.p);
    NodeRec nd;
    uint8_t r;
    if (precheck(a, pn, &nd, &r))
        r = fit_node<64, true>(a, pn, nd, lane, a.scratch + b.scratch_off, &fill, &cmask);
    if (lane == 0) a.reason[b.p] = r;
}

// pe_planner_commit patch: removed allocs stop counting (terminal byte) and
// the touched nodes get their new records (chain heads, key bounds).
__global__ void __launch_bounds__(256) k_plan_patch(NodeRec* nodes, AllocRec* pool, const uint32_t* dead, uint32_t n_dead,
                                                    const uint32_t* rows, const NodeRec* recs, uint32_t n_rows) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_dead) pool[dead[i]].terminal = 1;
    if (i < n_rows) nodes[rows[i]] = recs[i];
}

// The plan's staging copied from page-locked host memory by the CUs (each
// lane reads 16 B over PCIe per step, many workgroups in flight), instead of
// one copy-engine transfer (PE_PLAN_COPY=kernel).
__global__ void __launch_bounds__(256) k_plan_stage_copy(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         uint64_t n16) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) dst[i] = src[i];
}

}  // namespace pa

hipError_t pe_launch_plan_stage_copy(const void* host_mapped, void* dst, uint64_t bytes, hipStream_t st) {
    const uint64_t n16 = (bytes + 15) / 16;
    if (n16 == 0) return hipSuccess;
    const uint64_t want = (n16 + 255) / 256;
    const uint32_t blocks = (uint32_t)(want < 2048 ? want : 2048);
    hipLaunchKernelGGL(pa::k_plan_stage_copy, dim3(blocks), dim3(256), 0, st, (const uint4*)host_mapped, (uint4*)dst,
                       n16);
    return hipGetLastError();
}

hipError_t pe_launch_plan_patch(pa::NodeRec* nodes, pa::AllocRec* pool, const uint32_t* dead, uint32_t n_dead,
                                const uint32_t* rows, const pa::NodeRec* recs, uint32_t n_rows, hipStream_t st) {
    const uint32_t n = n_dead > n_rows ? n_dead : n_rows;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pa::k_plan_patch, dim3((n + 255) / 256), dim3(256), 0, st, nodes, pool, dead, n_dead, rows, recs,
                       n_rows);
    return hipGetLastError();
}

template <int G>
static void launch_group(const pa::PlanArgs* a, hipStream_t st) {
    const uint32_t blocks = (a->n_plan + pa::nodes_per_block(G) - 1) / pa::nodes_per_block(G);
    hipLaunchKernelGGL(pa::k_plan_eval<G>, dim3(blocks), dim3(64 * pa::kWaves), 0, st, *a);
}

// group: lanes per plan node (4, 8, 16 or 64); the host sized the LDS / scratch
// split with pa::lds_keys(group).
hipError_t pe_launch_plan_eval(const pa::PlanArgs* a, int group, hipStream_t st) {
    if (a->n_plan == 0) return hipSuccess;
    switch (group) {
        case 4: launch_group<4>(a, st); break;
        case 8: launch_group<8>(a, st); break;
        case 64: launch_group<64>(a, st); break;
        default: launch_group<16>(a, st); break;
    }
    if (a->n_big) hipLaunchKernelGGL(pa::k_plan_eval_big, dim3(a->n_big), dim3(64), 0, st, *a);
    return hipGetLastError();
}
