// HIP kernels of the MI355X placement engine (gfx950, wave64).
//
// k_place   — persistent single-workgroup count loop: for each placement it
//             sweeps the visit order from the StaticIterator cursor in chunks
//             of kPlaceBlock positions, evaluates the fused ranking pipeline per
//             node (FeasibilityWrapper verdict from the class table, distinct
//             hosts, BinPack fit + ScoreFit, job anti-affinity, rescheduling
//             penalty, node affinity, spread, ScoreNormalization), reproduces
//             LimitIterator + MaxScoreIterator with ballot prefix counts, and
//             commits the winner (Plan.AppendAlloc) to the HBM SoA before the
//             next placement. One launch runs the whole count loop.
// k_system  — SystemStack sweep: one single-node Select per list entry, every
//             node independent (scheduler_system.go:290-422); grid-stride.
// k_sweep_scores — full-scan scoring sweep with per-block (max, first-3
//             non-positive) reduction records: the bandwidth-bound kernel used
//             for roofline measurement and multi-GPU shards.
#include <hip/hip_runtime.h>
#include "engine_types.h"
#include "gomath_dev.h"

namespace pe {

enum : int { kOption = 0, kFiltered = 1, kExhausted = 2 };

struct NodeEval {
    int status;
    double score;
    uint32_t nscores;
    double parts[PE_MAX_SCORES];
};

__device__ __forceinline__ uint32_t pset_value(const TgTables& t, int p, uint32_t row, uint32_t cls) {
    return t.pset_val_node[p] ? t.pset_val_node[p][row] : t.pset_val_class[p][cls];
}

// Fused per-node pipeline. `spread_tab` holds the per-value spread contribution
// of each property set for the current plan (kMissing value -> -1.0).
template <bool kKeepParts>
__device__ __forceinline__ void eval_node(const NodeSoA& s, const TgTables& t, const Ask& a,
                                          const uint32_t* penalty_bits, double log10,
                                          const double* spread_tab, uint32_t row, NodeEval* out) {
    const uint32_t c = s.cls[row];
    // FeasibilityWrapper: memoised job + task-group checks (host-resolved per class)
    bool ok = t.class_ok[c] != 0;
    if (t.node_ok) ok = ok && t.node_ok[row] != 0;
    // DistinctHostsIterator (feasible.go:569-595)
    if (ok && (a.distinct_job | a.distinct_tg)) {
        if (a.distinct_job && s.coll_job[row] > 0) ok = false;
        if (a.distinct_tg && t.coll_tg[row] > 0) ok = false;
    }
    if (!ok) { out->status = kFiltered; return; }
    // BinPackIterator (rank.go:193-527): network offers, then AllocsFit
    int32_t dyn = 0;
    if (a.tg_dyn > 0 || a.has_task_net) dyn = s.used_dyn[row];
    if (a.tg_dyn > 0) {
        if ((t.alias_ok && !t.alias_ok[row]) || kDynPortCapacity - dyn < 1) { out->status = kExhausted; return; }
        dyn += a.tg_dyn;
    }
    if (a.has_task_net) {
        const int32_t avail = s.avail_mbits[row];
        if (avail < 0 || s.used_mbits[row] + a.task_mbits > avail || kDynPortCapacity - dyn < a.task_dyn) {
            out->status = kExhausted; return;
        }
    }
    const int64_t ucpu = s.used_cpu[row] + a.cpu;
    const int64_t umem = s.used_mem[row] + a.mem;
    const int64_t udisk = s.used_disk[row] + a.disk;
    const int64_t ccpu = s.cap_cpu[row], cmem = s.cap_mem[row];
    if (ccpu < ucpu || cmem < umem || s.cap_disk[row] < udisk) { out->status = kExhausted; return; }
    // Scores in append order, summed left to right.
    const double fit = gm::fit_score(ccpu, cmem, ucpu, umem, a.algo_spread, log10);
    double sum = fit;
    uint32_t k = 1;
    if (kKeepParts) out->parts[0] = fit;
    const uint32_t coll = t.coll_tg[row];
    if (a.anti_aff && coll > 0) {   // JobAntiAffinityIterator (rank.go:588-591)
        const double pen = -1 * (double)(coll + 1) / (double)a.desired_count;
        sum += pen;
        if (kKeepParts) out->parts[k] = pen;
        k++;
    }
    if (penalty_bits && ((penalty_bits[row >> 5] >> (row & 31)) & 1u)) {   // rank.go:632-635
        sum += -1.0;
        if (kKeepParts) out->parts[k] = -1.0;
        k++;
    }
    if (t.class_aff || t.node_aff) {   // NodeAffinityIterator (rank.go:698-725)
        const double aff = t.node_aff ? t.node_aff[row] : t.class_aff[c];
        if (aff != 0.0) {
            sum += aff;
            if (kKeepParts) out->parts[k] = aff;
            k++;
        }
    }
    if (t.n_psets > 0) {   // SpreadIterator (spread.go:110-174)
        double total = 0.0;
        for (int p = 0; p < t.n_psets; p++) {
            const uint32_t v = pset_value(t, p, row, c);
            total += (v == kMissing) ? -1.0 : spread_tab[p * (kMaxValues + 1) + v];
        }
        if (total != 0.0) {
            sum += total;
            if (kKeepParts) out->parts[k] = total;
            k++;
        }
    }
    out->status = kOption;
    out->score = sum / (double)k;   // ScoreNormalizationIterator (rank.go:762-767)
    out->nscores = k;
}

// evenSpreadScoreBoost (spread.go:178-228) / target boost (spread.go:143-164)
// for every value of every property set; one thread per value.
__device__ void build_spread_table(const TgTables& t, double* tab, uint32_t* scratch) {
    const int tid = threadIdx.x;
    for (int p = 0; p < t.n_psets; p++) {
        const int nv = t.pset_nvals[p];
        const uint32_t* cnt = t.pset_counts[p];
        if (t.pset_even[p]) {
            // min / max over values present in the combined use map (count > 0)
            if (tid == 0) {
                uint32_t mn = 0, mx = 0, present = 0;
                for (int v = 0; v < nv; v++) {
                    const uint32_t x = cnt[v];
                    if (x == 0) continue;
                    present++;
                    if (mn == 0 || x < mn) mn = x;
                    if (mx == 0 || x > mx) mx = x;
                }
                scratch[0] = mn; scratch[1] = mx; scratch[2] = present;
            }
            __syncthreads();
            const uint32_t mn = scratch[0], mx = scratch[1], present = scratch[2];
            for (int v = tid; v < nv; v += blockDim.x) {
                const uint32_t cur = cnt[v];
                double b;
                if (present == 0) b = 0.0;
                else {
                    double delta_boost;
                    if (mn == 0) delta_boost = -1.0;
                    else delta_boost = (double)(int)(mn - cur) / (double)mn;
                    if (cur != mn) b = delta_boost;
                    else if (mn == mx) b = -1.0;
                    else if (mn == 0) b = 1.0;
                    else b = (double)(int)(mx - mn) / (double)mn;
                }
                tab[p * (kMaxValues + 1) + v] = b;
            }
            __syncthreads();
        } else {
            for (int v = tid; v < nv; v += blockDim.x) {
                const double desired = t.pset_desired[p][v];
                double b;
                if (desired != desired) b = -1.0;   // no target and no implicit "*"
                else {
                    const double used = (double)(cnt[v] + 1u);
                    b = ((desired - used) / desired) * t.pset_weight_frac[p];
                }
                tab[p * (kMaxValues + 1) + v] = b;
            }
        }
    }
    __syncthreads();
}

template <int BLOCK>
struct PlaceShared {
    double spread_tab[kMaxPsets * (kMaxValues + 1)];
    uint32_t scratch[4];
    uint32_t wave_a[BLOCK / 64];
    uint32_t wave_b[BLOCK / 64];
    double red_score[BLOCK / 64];
    int red_pos[BLOCK / 64];
    // LimitIterator skip list: up to kMaxSkip set-aside options
    double aside_score[kMaxSkip];
    int aside_pos[kMaxSkip];
    int aside_row[kMaxSkip];
    uint32_t aside_nscores[kMaxSkip];
    // loop state
    int stop_j;          // chunk index of the limit-th returned option, or -1
    int done;
};

__device__ __forceinline__ uint32_t lanes_below(uint64_t m, int lane) {
    return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// Exclusive block prefix of a predicate; returns (prefix, total).
template <int BLOCK>
__device__ __forceinline__ uint32_t block_prefix(bool pred, uint32_t* wave_tot, uint32_t* total) {
    constexpr int W = BLOCK / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t m = __ballot(pred);
    if (lane == 0) wave_tot[wid] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < W; w++) {
        const uint32_t x = wave_tot[w];
        before += (w < wid) ? x : 0u;
        tot += x;
    }
    __syncthreads();
    *total = tot;
    return before + lanes_below(m, lane);
}

// argmax over (score desc, pos asc) for candidates; returns winner in lane 0 of wave 0 via LDS
template <int BLOCK>
__device__ __forceinline__ void block_argmax(bool cand, double score, int pos, double* red_score, int* red_pos,
                                             double* best_score, int* best_pos) {
    constexpr int W = BLOCK / 64;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    double s = cand ? score : -__builtin_inf();
    int p = cand ? pos : 0x7FFFFFFF;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double os = __shfl_xor(s, off);
        const int op = __shfl_xor(p, off);
        if (os > s || (os == s && op < p)) { s = os; p = op; }
    }
    if (lane == 0) { red_score[wid] = s; red_pos[wid] = p; }
    __syncthreads();
    double bs = red_score[0];
    int bp = red_pos[0];
#pragma unroll
    for (int w = 1; w < W; w++) {
        const double os = red_score[w];
        const int op = red_pos[w];
        if (os > bs || (os == bs && op < bp)) { bs = os; bp = op; }
    }
    *best_score = bs;
    *best_pos = bp;
    __syncthreads();
}

__device__ __forceinline__ void commit_row(const NodeSoA& s, const TgTables& t, const Ask& a, uint32_t row) {
    s.used_cpu[row] += a.cpu;
    s.used_mem[row] += a.mem;
    s.used_disk[row] += a.disk;
    s.used_mbits[row] += a.commit_mbits;
    s.used_dyn[row] += a.commit_dyn;
    s.coll_job[row] += 1;
    t.coll_tg[row] += 1;
    const uint32_t c = s.cls[row];
    for (int p = 0; p < t.n_psets; p++) {
        const uint32_t v = pset_value(t, p, row, c);
        if (v != kMissing) t.pset_counts[p][v] += 1;
    }
}

// Persistent count loop. One workgroup; see file header.
template <int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_place(SelectArgs A) {
    __shared__ PlaceShared<BLOCK> sh;
    const int tid = threadIdx.x;
    const uint32_t n = A.n_visit;
    uint32_t offset = A.offset % (n ? n : 1);
    uint32_t placed = 0;

    for (uint32_t it = 0; it < A.count; it++) {
        if (A.tg.n_psets > 0) build_spread_table(A.tg, sh.spread_tab, sh.scratch);

        uint32_t r = 0, a = 0;            // returned / set-aside options so far
        double best_score = -__builtin_inf();
        int best_pos = -1;                // relative visit position of the winner
        uint32_t n_filtered = 0, n_exhausted = 0;
        uint32_t consumed = n;
        bool stopped = false;

        for (uint32_t base = 0; base < n; base += BLOCK) {
            const uint32_t j = base + tid;
            const bool valid = j < n;
            NodeEval ev;
            ev.status = kFiltered;
            ev.score = 0.0;
            uint32_t row = 0;
            if (valid) {
                uint32_t pos = offset + j;
                if (pos >= n) pos -= n;
                row = A.perm[pos];
                eval_node<false>(A.soa, A.tg, A.ask, A.penalty_bits, A.log10, sh.spread_tab, row, &ev);
            }
            const bool is_opt = valid && ev.status == kOption;
            const bool is_np = is_opt && ev.score <= 0.0;
            uint32_t np_tot;
            const uint32_t np_before = a + block_prefix<BLOCK>(is_np, sh.wave_a, &np_tot);
            const bool aside = is_np && np_before < (uint32_t)kMaxSkip;
            const bool ret = is_opt && !aside;
            uint32_t ret_tot;
            const uint32_t ret_before = r + block_prefix<BLOCK>(ret, sh.wave_b, &ret_tot);
            // the limit-th returned option ends the pull
            if (tid == 0) sh.stop_j = -1;
            __syncthreads();
            if (ret && ret_before == A.limit - 1u) sh.stop_j = (int)tid;
            __syncthreads();
            const int stop_j = sh.stop_j;
            const bool pulled = valid && (stop_j < 0 || (int)tid <= stop_j);
            // set-aside options actually pulled
            if (aside && pulled) {
                sh.aside_score[np_before] = ev.score;
                sh.aside_pos[np_before] = (int)j;
                sh.aside_row[np_before] = (int)row;
            }
            const bool cand = ret && ret_before < A.limit;
            double cs; int cp;
            block_argmax<BLOCK>(cand, ev.score, (int)j, sh.red_score, sh.red_pos, &cs, &cp);
            if (cp != 0x7FFFFFFF && cs > best_score) { best_score = cs; best_pos = cp; }
            // metrics over pulled positions
            uint32_t f_tot, e_tot;
            block_prefix<BLOCK>(pulled && ev.status == kFiltered, sh.wave_a, &f_tot);
            block_prefix<BLOCK>(pulled && ev.status == kExhausted, sh.wave_b, &e_tot);
            n_filtered += f_tot;
            n_exhausted += e_tot;
            uint32_t aside_pulled;
            block_prefix<BLOCK>(aside && pulled, sh.wave_a, &aside_pulled);
            a += aside_pulled;
            if (stop_j >= 0) {
                consumed = base + (uint32_t)stop_j + 1u;
                r = A.limit;
                stopped = true;
                break;
            }
            r += ret_tot;
        }
        if (!stopped) {
            // source exhausted: skipped options are emitted in order until the limit
            const uint32_t take = min(a, A.limit - r);
            for (uint32_t i = 0; i < take; i++) {
                if (sh.aside_score[i] > best_score) { best_score = sh.aside_score[i]; best_pos = sh.aside_pos[i]; }
            }
        }
        // winner row and its score parts (recomputed by one lane for the record)
        int win_row = -1;
        if (best_pos >= 0) {
            uint32_t pos = offset + (uint32_t)best_pos;
            if (pos >= n) pos -= n;
            win_row = (int)A.perm[pos];
        }
        if (tid == 0) {
            pe_ranked_node& o = A.out[it];
            o.row = win_row;
            o.nodes_evaluated = consumed;
            o.nodes_filtered = n_filtered;
            o.nodes_exhausted = n_exhausted;
            if (win_row >= 0) {
                NodeEval ev;
                eval_node<true>(A.soa, A.tg, A.ask, A.penalty_bits, A.log10, sh.spread_tab, (uint32_t)win_row, &ev);
                o.final_score = ev.score;
                o.n_scores = ev.nscores;
                for (int k = 0; k < PE_MAX_SCORES; k++) o.scores[k] = k < (int)ev.nscores ? ev.parts[k] : 0.0;
            } else {
                o.final_score = 0.0;
                o.n_scores = 0;
                for (int k = 0; k < PE_MAX_SCORES; k++) o.scores[k] = 0.0;
            }
            uint32_t no = offset + (consumed % (n ? n : 1));
            if (no >= n) no -= n;
            o.new_offset = no;
            if (win_row >= 0 && A.commit) commit_row(A.soa, A.tg, A.ask, (uint32_t)win_row);
        }
        if (n) offset = (offset + consumed % n) % n;
        __syncthreads();
        if (win_row < 0) break;   // nil option: failedTGAllocs short-circuit
        placed++;
    }
    if (tid == 0) {
        A.status[0] = placed;
        A.status[1] = offset;
    }
}

// SystemStack: every list entry is an independent single-node Select.
__global__ void __launch_bounds__(256) k_system(SystemArgs A) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t local = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n_list; i += stride) {
        const uint32_t row = A.list[i];
        NodeEval ev;
        eval_node<false>(A.soa, A.tg, A.ask, nullptr, A.log10, nullptr, row, &ev);
        if (ev.status == kOption) {
            A.out_score[i] = ev.score;
            A.out_status[i] = 0;
            commit_row(A.soa, A.tg, A.ask, row);
            local++;
        } else {
            A.out_score[i] = __builtin_nan("");
            A.out_status[i] = (uint8_t)ev.status;
        }
    }
    // one atomic per wave
    for (int off = 32; off > 0; off >>= 1) local += __shfl_xor(local, off);
    if ((threadIdx.x & 63) == 0 && local) atomicAdd(A.placed, local);
}

// Host-side commit of a single placement (pe_commit).
__global__ void k_commit(NodeSoA s, TgTables t, Ask a, uint32_t row) {
    if (threadIdx.x == 0 && blockIdx.x == 0) commit_row(s, t, a, row);
}

}  // namespace pe

// ---- launch wrappers (host) ------------------------------------------------
extern "C" hipError_t pe_launch_place(const pe::SelectArgs* a, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_place<pe::kPlaceBlock>, dim3(1), dim3(pe::kPlaceBlock), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t pe_launch_system(const pe::SystemArgs* a, hipStream_t st) {
    uint32_t blocks = (a->n_list + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_system, dim3(blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}

extern "C" hipError_t pe_launch_commit(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a,
                                       uint32_t row, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_commit, dim3(1), dim3(64), 0, st, *s, *t, *a, row);
    return hipGetLastError();
}
