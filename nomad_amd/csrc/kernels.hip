// HIP kernels of the MI355X placement engine (gfx950, wave64).
//
// k_place<BLOCK, FULL, CORES>  persistent count loop, one workgroup per evaluation.
//   The node SoA in HBM is the snapshot's proposed state and is read-only
//   during the loop; each evaluation keeps the allocs it places in a private
//   LDS overlay (open-addressed hash keyed by node row: cpu/mem/disk/collision/
//   network deltas), so any number of evaluations share one L2-resident table
//   (NumSchedulers workers, nomad/config.go:468). Per placement the workgroup
//   sweeps the visit order from the StaticIterator cursor in chunks of BLOCK
//   positions, runs the fused ranking pipeline per node (FeasibilityWrapper
//   verdict from the class table, distinct_hosts, BinPack fit + ScoreFit, job
//   anti-affinity, rescheduling penalty, node affinity, spread, score
//   normalisation), reproduces LimitIterator + MaxScoreIterator with ballot
//   prefix counts and commits the winner to the overlay
//   (Plan.AppendAlloc). FULL=false: one wave per eval for windowed binpack
//   (limit = ceil(log2 n)); FULL=true: 256 threads per eval for full scans
//   (affinities / spreads: limit = MaxInt32) with per-value spread tables in LDS.
//   With `writeback` the overlay is merged into the HBM SoA at the end (single
//   eval API: the plan persists in the stack).
// k_system              SystemStack: independent single-node Selects, grid-stride.
// k_commit              one Plan.AppendAlloc on the HBM SoA (pe_commit).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstring>
#include "engine_types.h"
#include "gomath_dev.h"
#include "gosort.h"

namespace pe {

enum : int { kOption = 0, kFiltered = 1, kExhausted = 2 };
constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr uint32_t kFoldMaxClasses = 16384;   // class verdict table staged in LDS by a fold

struct NodeEval {
    int status;
    double score;
    uint32_t nscores;
    double parts[PE_MAX_SCORES];
};

// Per-eval LDS overlay of the allocs this eval placed: row -> k placements.
// Every placement of the count loop has the same ask, so the deltas are k * ask.
// Packed form (k == null): one u32 per entry, row << kshift | k, which halves
// the LDS per evaluation and so doubles the evaluations resident per CU.
struct Overlay {
    uint32_t* keys;      // null: no overlay
    uint32_t* k;         // null: packed entries
    uint32_t mask;
    int bits;
    int kshift;
    uint32_t kmask;
};

__device__ __forceinline__ uint32_t ov_hash(const Overlay& o, uint32_t row) {
    return (row * 2654435761u) >> (32 - o.bits);
}

__device__ __forceinline__ uint32_t ov_count(const Overlay& o, uint32_t row) {
    if (!o.keys) return 0;
    uint32_t h = ov_hash(o, row);
    if (!o.k) {
        for (;;) {
            const uint32_t e = o.keys[h];
            if (e == kEmpty) return 0;
            if ((e >> o.kshift) == row) return e & o.kmask;
            h = (h + 1) & o.mask;
        }
    }
    for (;;) {
        const uint32_t key = o.keys[h];
        if (key == row) return o.k[h];
        if (key == kEmpty) return 0;
        h = (h + 1) & o.mask;
    }
}

// Plan.AppendAlloc into the overlay (one lane); returns the row's slot.
__device__ __forceinline__ uint32_t ov_add(const Overlay& o, uint32_t row) {
    uint32_t h = ov_hash(o, row);
    if (!o.k) {
        for (;;) {
            const uint32_t e = o.keys[h];
            if (e == kEmpty) { o.keys[h] = (row << o.kshift) | 1u; return h; }
            if ((e >> o.kshift) == row) { o.keys[h] = e + 1u; return h; }
            h = (h + 1) & o.mask;
        }
    }
    for (;;) {
        const uint32_t key = o.keys[h];
        if (key == row) { o.k[h] += 1; return h; }
        if (key == kEmpty) { o.keys[h] = row; o.k[h] = 1; return h; }
        h = (h + 1) & o.mask;
    }
}

// Slot of `row` in the overlay, or -1 when the row holds no placement.
__device__ __forceinline__ int ov_slot(const Overlay& o, uint32_t row) {
    uint32_t h = ov_hash(o, row);
    if (!o.k) {
        for (;;) {
            const uint32_t e = o.keys[h];
            if (e == kEmpty) return -1;
            if ((e >> o.kshift) == row) return (int)h;
            h = (h + 1) & o.mask;
        }
    }
    for (;;) {
        const uint32_t key = o.keys[h];
        if (key == row) return (int)h;
        if (key == kEmpty) return -1;
        h = (h + 1) & o.mask;
    }
}

__device__ __forceinline__ uint32_t pset_value(const TgTables& t, int p, uint32_t row, uint32_t cls) {
    return t.pset_val_node[p] ? t.pset_val_node[p][row] : t.pset_val_class[p][cls];
}

// The per-node HBM reads of the pipeline, all independent of each other: the
// 64-byte record, the (job, tg) collision count and the folded verdict byte.
struct NodeIn {
    NodeRec r;
    uint32_t coll_tg;
    uint32_t feas;
    uint32_t dev_free;   // free healthy instances per device group (4 x u8), device asks only
};

__device__ __forceinline__ void load_node(const NodeSoA& s, const TgTables& t, uint32_t row, NodeIn& in) {
    in.r = s.rec[row];
    in.coll_tg = t.coll_tg[row];
    in.feas = t.node_feas ? t.node_feas[row] : 1u;
    in.dev_free = t.dev_free ? t.dev_free[row] : 0u;
}

// deviceAllocator.AssignDevice for the task group's requests in order
// (scheduler/device.go:32-131, BinPack rank.go:366-414) on a node's packed
// free counts: per request the best-scoring matching group with enough free
// instances, equal scores -> the later group (the reference walks a map);
// the offer's instances are consumed (AddReserved). Returns false when a
// request cannot be met; *matched = Σ matched weights of requests with
// affinities.
__device__ __forceinline__ bool dev_assign(const Ask& a, const DevClass& dc, uint32_t& free, double* matched,
                                           uint32_t* groups = nullptr) {
    double sum = 0.0;
    if (dc.n_groups == 0) return false;   // "no devices available"
    for (int q = 0; q < kMaxDevReq; q++) {
        if (q >= a.n_dev) break;
        const uint32_t cnt = (uint32_t)a.dev_cnt[q];
        if (cnt == 0) return false;       // "invalid request of zero devices"
        int best = -1;
        double best_score = 0.0;
        for (int g = 0; g < kMaxDevGroups; g++) {
            if (g >= (int)dc.n_groups) break;
            const uint32_t f = (free >> (8 * g)) & 255u;
            if (f < cnt || !((dc.match[q] >> g) & 1u)) continue;
            const double sc = dc.choice[q][g];
            if (best >= 0 && sc < best_score) continue;
            best = g;
            best_score = sc;
        }
        if (best < 0) return false;        // "no devices match request"
        free -= cnt << (8 * best);
        if (groups) groups[q] = (uint32_t)best;
        if ((a.dev_aff >> q) & 1u) sum += dc.matched[q][best];
    }
    *matched = sum;
    return true;
}

// Device state after k further placements of the task group on a node.
__device__ __forceinline__ uint32_t dev_after(const Ask& a, const DevClass& dc, uint32_t free, uint32_t k) {
    for (uint32_t j = 0; j < k; j++) {
        double m;
        dev_assign(a, dc, free, &m);
    }
    return free;
}

// Reserved cores of the (dk+1)-th placement on the row, out of line so that
// the hot pipeline keeps its registers: status 1 when too few cores are free
// ("cores"), 2 when a chosen core is outside the AllocsFit-available set;
// cpu = the cores' CpuShares (SharesPerCore x cores).
struct CoreFit {
    int64_t cpu;
    int32_t status;
};

__device__ __forceinline__ CoreFit core_fit(const uint64_t* rsvable, const uint64_t* used, const uint64_t* avail,
                                         const int64_t* spc, uint32_t cores, uint32_t row, uint32_t dk) {
    CoreFit f{0, 1};
    if (!rsvable) return f;
    uint32_t skip = dk * cores, need = cores;
    uint64_t out = 0, any_av = 0;
#pragma unroll 1
    for (int w = 0; w < 4; w++) {
        any_av |= avail[4 * row + w];
        uint64_t fr = rsvable[4 * row + w] & ~used[4 * row + w];
        const uint32_t c = (uint32_t)__popcll(fr);
        if (skip >= c) { skip -= c; continue; }
        for (; skip; skip--) fr &= fr - 1;
        uint64_t ch = 0;
        for (; fr && need; need--) { ch |= fr & (~fr + 1); fr &= fr - 1; }
        out |= ch & ~avail[4 * row + w];
    }
    if (need) return f;
    f.status = (any_av && out) ? 2 : 0;
    f.cpu = (int64_t)cores * spc[row];
    return f;
}

// CpuShares of one placement on the row: tasks with cores hold SharesPerCore x
// cores (rank.go:461-463).
__device__ __forceinline__ int64_t ask_cpu(const NodeSoA& s, const Ask& a, uint32_t row) {
    return a.cores > 0 ? a.cpu + (int64_t)a.cores * s.core_spc[row] : a.cpu;
}

// Plan.AppendAlloc of k placements on the row: their cores leave the free set.
__device__ __forceinline__ void core_take_rows(const uint64_t* rsvable, uint64_t* used, uint32_t row, uint32_t need) {
#pragma unroll 1
    for (int w = 0; w < 4 && need; w++) {
        uint64_t f = rsvable[4 * row + w] & ~used[4 * row + w], t = 0;
        for (; f && need; need--) { t |= f & (~f + 1); f &= f - 1; }
        used[4 * row + w] |= t;
    }
}

__device__ __forceinline__ void core_take(const NodeSoA& s, const Ask& a, uint32_t row, uint32_t k) {
    if (a.cores > 0 && s.core_rsvable) core_take_rows(s.core_rsvable, s.core_used, row, k * (uint32_t)a.cores);
}

// Inputs of the scoring half of the pipeline (everything after AllocsFit).
// The table lookups (affinity, spread, penalty) are resolved by
// lookup_scores so that their loads issue with the node's own loads; the
// scoring half is then pure arithmetic.
struct ScoreIn {
    int64_t ccpu, cmem, ucpu, umem;   // capacity and proposed use including the ask
    double dev_aff;                   // BinPack device-affinity score (appended when Ask::dev_tw != 0)
    double aff;                       // NodeAffinityIterator score (0 = not appended)
    double spread;                    // SpreadIterator total (0 = not appended)
    uint32_t coll;                    // proposed allocs of (job, tg) on the node
    uint32_t penalty;                 // node in the rescheduling penalty set
};

// Feasibility half of the fused per-node pipeline over base (HBM) + overlay
// (dk placements of this eval): FeasibilityWrapper verdict, distinct_hosts,
// BinPack network offers and AllocsFit. Returns kOption with the scoring
// inputs filled, else kFiltered / kExhausted.
// DistinctPropertyIterator (feasible.go:601-704): the node's value of each
// distinct_property set must exist and be used fewer than `allowed` times.
// `tab` (the eval's per-value table, 0.0 = open) or the HBM counts.
__device__ __forceinline__ bool distinct_ok(const TgTables& t, const double* tab, uint32_t row, uint32_t c) {
    for (int p = t.n_spread; p < t.n_psets; p++) {
        const uint32_t v = pset_value(t, p, row, c);
        if (v == kMissing) return false;
        const bool blocked = tab ? tab[t.pset_tab_off[p] + v] != 0.0 : t.pset_counts[p][v] >= t.pset_allowed[p];
        if (blocked) return false;
    }
    return true;
}

template <bool kCores = true>
__device__ __forceinline__ int status_loaded(const NodeSoA& s, const TgTables& t, const uint8_t* class_ok,
                                             const Ask& a, uint32_t dk, uint32_t row, const NodeIn& in,
                                             ScoreIn* si, const double* ptab = nullptr) {
    const NodeRec& r = in.r;
    const uint32_t c = r.cls;
    // FeasibilityWrapper: memoised job + task-group checks (host-resolved per class)
    bool ok;
    if (t.node_feas) ok = in.feas != 0;
    else {
        ok = class_ok[c] != 0;
        if (t.node_ok) ok = ok && t.node_ok[row] != 0;
    }
    const uint32_t coll = in.coll_tg + dk;
    // DistinctHostsIterator (feasible.go:569-595)
    if (ok && (a.distinct_job | a.distinct_tg)) {
        if (a.distinct_job && s.coll_job[row] + dk > 0) ok = false;
        if (a.distinct_tg && coll > 0) ok = false;
    }
    if (ok && t.n_psets > t.n_spread) ok = distinct_ok(t, ptab, row, c);
    if (!ok) return kFiltered;
    // BinPackIterator (rank.go:193-527): network offers, then AllocsFit.
    // AssignPorts' static ports first (network.go:317-363): the host-built gate
    // (free on the node's address, no placement of the group since)
    if (t.static_gate) {
        const uint32_t gt = t.static_gate[row];
        if (gt == 0u || in.coll_tg + dk + 1u != gt) return kExhausted;
    }
    if (a.tg_dyn > 0 || a.has_task_net) {
        int32_t dyn = r.used_dyn + (int32_t)dk * a.commit_dyn;
        if (a.tg_dyn > 0) {
            if ((t.alias_ok && !t.alias_ok[row]) || kDynPortCapacity - dyn - a.static_dyn < 1) return kExhausted;
            dyn += a.tg_dyn + a.static_dyn;
        }
        if (a.has_task_net) {
            const uint32_t md_lim = t.md ? t.md[row].lim : ~0u;
            if (md_lim != ~0u) {   // a multi-device node: the host's first fit over its devices
                if (in.coll_tg + dk >= md_lim) return kExhausted;
            } else {
                const int32_t avail = r.avail_mbits;
                const int32_t mb = r.used_mbits + (int32_t)dk * a.commit_mbits;
                if (avail < 0 || mb + a.task_mbits > avail || kDynPortCapacity - dyn < a.task_dyn) return kExhausted;
                if (t.task_gate) {   // AssignNetwork's static ports (network.go:419-431), host-built gate
                    const uint32_t gt = t.task_gate[row];
                    if (gt == 0u || in.coll_tg + dk + 1u != gt) return kExhausted;
                }
            }
        }
    }
    si->dev_aff = 0.0;
    if (a.n_dev > 0) {   // devices: this eval's dk earlier placements first consumed their offers
        const DevClass& dc = t.dev_cls[c];
        uint32_t fr = dev_after(a, dc, in.dev_free, dk);
        double m;
        if (!dev_assign(a, dc, fr, &m)) return kExhausted;
        if (a.dev_tw != 0.0) si->dev_aff = m / a.dev_tw;
    }
    int64_t acpu = a.cpu;
    bool core_out = false;
    if (kCores && a.cores > 0) {   // reserved cores (rank.go:437-466), then AllocsFit's Superset check
        const CoreFit f = core_fit(s.core_rsvable, s.core_used, s.core_avail, s.core_spc, (uint32_t)a.cores, row, dk);
        if (f.status == 1) return kExhausted;
        acpu += f.cpu;
        core_out = f.status == 2;
    }
    const int64_t ucpu = r.used_cpu + (int64_t)(dk + 1) * acpu;
    const int64_t umem = r.used_mem + (int64_t)(dk + 1) * a.mem;
    const int64_t udisk = r.used_disk + (int64_t)(dk + 1) * a.disk;
    if (r.cap_cpu < ucpu || core_out || r.cap_mem < umem || r.cap_disk < udisk) return kExhausted;
    si->ccpu = r.cap_cpu;
    si->cmem = r.cap_mem;
    si->ucpu = ucpu;
    si->umem = umem;
    si->coll = coll;
    return kOption;
}

// Table lookups of the scoring half for an option: penalty bit, node affinity,
// spread total (per-property boosts summed in property order, spread.go:145-170).
__device__ __forceinline__ void lookup_scores(const TgTables& t, const uint32_t* penalty_bits,
                                              const double* spread_tab, uint32_t row, uint32_t c, ScoreIn* si) {
    si->penalty = penalty_bits ? (penalty_bits[row >> 5] >> (row & 31)) & 1u : 0u;
    si->aff = (t.class_aff || t.node_aff) ? (t.node_aff ? t.node_aff[row] : t.class_aff[c]) : 0.0;
    double total = 0.0;
    for (int p = 0; p < t.n_spread; p++) {
        const uint32_t v = pset_value(t, p, row, c);
        total += (v == kMissing) ? -1.0 : spread_tab[t.pset_tab_off[p] + v];
    }
    si->spread = total;
}

// Scoring half: scores in append order, summed left to
// right, then ScoreNormalizationIterator.
// The scores before the spread one, summed left to right; k = how many.
template <bool kKeepParts>
__device__ __forceinline__ double score_head(const Ask& a, double log10, const ScoreIn& si, double* parts,
                                             uint32_t& k_out) {
    const uint32_t coll = si.coll;
    const double fit = gm::fit_score(si.ccpu, si.cmem, si.ucpu, si.umem, a.algo_spread, log10);
    double sum = fit;
    uint32_t k = 1;
    if (kKeepParts) parts[0] = fit;
    if (a.dev_tw != 0.0) {   // device affinity (rank.go:518-523)
        sum += si.dev_aff;
        if (kKeepParts) parts[k] = si.dev_aff;
        k++;
    }
    if (a.anti_aff && coll > 0) {   // JobAntiAffinityIterator (rank.go:588-591)
        const double pen = -1 * (double)(coll + 1) / (double)a.desired_count;
        sum += pen;
        if (kKeepParts) parts[k] = pen;
        k++;
    }
    if (si.penalty) {   // NodeReschedulingPenaltyIterator (rank.go:632-635)
        sum += -1.0;
        if (kKeepParts) parts[k] = -1.0;
        k++;
    }
    if (si.aff != 0.0) {   // NodeAffinityIterator (rank.go:698-725)
        sum += si.aff;
        if (kKeepParts) parts[k] = si.aff;
        k++;
    }
    k_out = k;
    return sum;
}

// The normalised score; with kKeepParts the parts go to `parts` (any
// address space: a runtime index into a stack array would live in scratch).
template <bool kKeepParts>
__device__ __forceinline__ double score_into(const Ask& a, double log10, const ScoreIn& si, double* parts,
                                             uint32_t* nscores) {
    uint32_t k;
    double sum = score_head<kKeepParts>(a, log10, si, parts, k);
    if (si.spread != 0.0) {   // SpreadIterator (spread.go:110-174)
        sum += si.spread;
        if (kKeepParts) parts[k] = si.spread;
        k++;
    }
    *nscores = k;
    return sum / (double)k;   // ScoreNormalizationIterator (rank.go:762-767)
}

template <bool kKeepParts>
__device__ __forceinline__ void score_option(const Ask& a, double log10, const ScoreIn& si, NodeEval* out) {
    uint32_t k;
    double sum = score_head<kKeepParts>(a, log10, si, out->parts, k);
    if (si.spread != 0.0) {   // SpreadIterator (spread.go:110-174)
        sum += si.spread;
        if (kKeepParts) out->parts[k] = si.spread;
        k++;
    }
    out->status = kOption;
    out->score = sum / (double)k;   // ScoreNormalizationIterator (rank.go:762-767)
    out->nscores = k;
}

// The whole fused per-node pipeline.
template <bool kKeepParts, bool kCores = true>
__device__ __forceinline__ void eval_loaded(const NodeSoA& s, const TgTables& t, const uint8_t* class_ok,
                                            const Ask& a, uint32_t dk, const uint32_t* penalty_bits,
                                            double log10, const double* spread_tab, uint32_t row,
                                            const NodeIn& in, NodeEval* out) {
    ScoreIn si;
    const int st = status_loaded<kCores>(s, t, class_ok, a, dk, row, in, &si, spread_tab);
    if (st != kOption) { out->status = st; return; }
    lookup_scores(t, penalty_bits, spread_tab, row, in.r.cls, &si);
    score_option<kKeepParts>(a, log10, si, out);
}

template <bool kKeepParts, bool kCores = true>
__device__ __forceinline__ void eval_node(const NodeSoA& s, const TgTables& t, const uint8_t* class_ok,
                                          const Ask& a, const Overlay& ov, const uint32_t* penalty_bits,
                                          double log10, const double* spread_tab, uint32_t row,
                                          NodeEval* out) {
    NodeIn in;
    load_node(s, t, row, in);
    eval_loaded<kKeepParts, kCores>(s, t, class_ok, a, ov_count(ov, row), penalty_bits, log10, spread_tab, row, in,
                            out);
}

// AllocMetric trace (structs.go:9903-9937): for visited rows that passed the
// FeasibilityWrapper, which iterator stopped them and why, with the same state
// the Select saw (HBM SoA, no overlay). Codes: kTr* in engine_types.h; a
// distinct_property failure carries its set index in bits 8-15.
// Options also get their named scores (ScoreNode calls, rank.go:516-522, 591-593,
// 635-637, 704-722, spread.go:170, rank.go:769) as 6 doubles: binpack, devices,
// job-anti-affinity, node-affinity, allocation-spread, normalized-score.
// Row of entry j of record k of a batched trace (TraceSrc).
__device__ __forceinline__ uint32_t trace_row(const TraceSrc& r, uint32_t k, uint32_t j) {
    const uint32_t src = r.rsrc[k];
    if (!(src & kTraceRot)) return r.rows[src + j];
    uint32_t p = (src - kTraceRot) + j;
    if (p >= r.n_list) p -= r.n_list;
    return r.list[p];
}

// Placements of records before k on `row` (the sorted (row, record) pairs).
__device__ __forceinline__ uint32_t trace_dk(const TraceSrc& r, uint32_t row, uint32_t k) {
    const uint64_t key = (uint64_t)row << 32;
    uint32_t lo = 0, hi = r.n_pl;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (r.pl[mid] < key) lo = mid + 1;
        else hi = mid;
    }
    uint32_t d = 0;
    for (; lo < r.n_pl && (uint32_t)(r.pl[lo] >> 32) == row && (uint32_t)r.pl[lo] < k; lo++) d++;
    return d;
}

// Record of entry i of a batched trace: the first k with rec_end[k] > i.
__device__ __forceinline__ uint32_t trace_rec(const TraceSrc& r, uint32_t i) {
    uint32_t lo = 0, hi = r.n_rec;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (r.rec_end[mid] > i) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// dk (TraceSrc): placements of this task group on the row that the state
// lacks (a speculative run's earlier Selects, traced against the run's
// starting state; no distinct_property sets then), applied as status_loaded
// does. In a batched trace record k's spread boosts are spread_tab + k *
// pset_tab_total (k_spread_tables: the record's own use counts).
__global__ void k_trace(NodeSoA s, TgTables t, Ask a, TraceSrc src, uint32_t n, uint32_t* out,
                        const uint32_t* penalty_bits, double log10, const double* spread_tab, double* sc) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t row, dk;
    if (src.rec_end) {
        const uint32_t k = trace_rec(src, i);
        row = trace_row(src, k, i - (k ? src.rec_end[k - 1] : 0u));
        dk = trace_dk(src, row, k);
        if (spread_tab) spread_tab += (size_t)k * t.pset_tab_total;
    } else {
        row = src.rows[i];
        dk = src.dks ? (uint32_t)src.dks[i] : 0u;
    }
    NodeIn in;
    load_node(s, t, row, in);
    NodeRec& r = in.r;
    const uint32_t c = r.cls;
    uint32_t code = kTrOption;
    if ((a.distinct_job && s.coll_job[row] + dk > 0) || (a.distinct_tg && in.coll_tg + dk > 0)) {
        code = kTrDistinctHosts;                                   // feasible.go:569-595
    } else {
        for (int p = t.n_spread; p < t.n_psets && code == kTrOption; p++) {
            const uint32_t v = pset_value(t, p, row, c);
            if (v == kMissing || t.pset_counts[p][v] >= t.pset_allowed[p]) code = kTrDistinctProp | ((uint32_t)p << 8);
        }
    }
    if (code == kTrOption && t.static_gate &&                      // AssignPorts static ports (network.go:317-363)
        (t.static_gate[row] == 0u || in.coll_tg + dk + 1u != t.static_gate[row]))
        code = kTrStaticPort;
    if (dk) {   // the earlier placements' network use
        r.used_dyn += (int32_t)dk * a.commit_dyn;
        r.used_mbits += (int32_t)dk * a.commit_mbits;
    }
    if (code == kTrOption && (a.tg_dyn > 0 || a.has_task_net)) {   // rank.go:231-295
        int32_t dyn = r.used_dyn;
        if (a.tg_dyn > 0) {
            if (t.alias_ok && !t.alias_ok[row]) code = kTrNoAddr;
            else if (kDynPortCapacity - dyn - a.static_dyn < 1) code = kTrDynPorts;
            dyn += a.tg_dyn + a.static_dyn;
        }
        const uint32_t md_lim = (code == kTrOption && a.has_task_net && t.md) ? t.md[row].lim : ~0u;
        if (md_lim != ~0u) {   // a multi-device node: the host's outcome of the first refused placement
            if (in.coll_tg + dk >= md_lim) code = t.md[row].code;
        } else if (code == kTrOption && a.has_task_net) {
            if (r.avail_mbits < 0) code = kTrNoNetworks;
            else if (r.used_mbits + a.task_mbits > r.avail_mbits) code = kTrBandwidth;
            else if (t.task_gate && (t.task_gate[row] == 0u || in.coll_tg + dk + 1u != t.task_gate[row])) code = kTrTaskStatic;
            else if (kDynPortCapacity - dyn < a.task_dyn) code = kTrTaskDyn;
        }
    }
    if (code == kTrOption && a.n_dev > 0) {                         // AssignDevice errors (device.go:32-131)
        const DevClass& dc = t.dev_cls[c];
        uint32_t free = dk ? dev_after(a, dc, in.dev_free, dk) : in.dev_free;
        if (dc.n_groups == 0) code = kTrDevNone;
        for (int q = 0; q < kMaxDevReq && code == kTrOption; q++) {
            if (q >= a.n_dev) break;
            const uint32_t cnt = (uint32_t)a.dev_cnt[q];
            if (cnt == 0) { code = kTrDevZero; break; }
            int best = -1;
            double best_score = 0.0;
            for (int g = 0; g < kMaxDevGroups; g++) {
                if (g >= (int)dc.n_groups) break;
                const uint32_t f = (free >> (8 * g)) & 255u;
                if (f < cnt || !((dc.match[q] >> g) & 1u)) continue;
                const double sc = dc.choice[q][g];
                if (best >= 0 && sc < best_score) continue;
                best = g;
                best_score = sc;
            }
            if (best < 0) { code = kTrDevNoMatch; break; }
            free -= cnt << (8 * best);
        }
    }
    bool core_out = false;
    if (code == kTrOption && a.cores > 0) {                         // reserved cores (rank.go:437-466)
        const CoreFit f = core_fit(s.core_rsvable, s.core_used, s.core_avail, s.core_spc, (uint32_t)a.cores, row, dk);
        if (f.status == 1) code = kTrCores;
        core_out = f.status == 2;
    }
    if (code == kTrOption) {                                        // AllocsFit → Superset order
        const int64_t k1 = (int64_t)dk + 1;
        if (r.cap_cpu < r.used_cpu + k1 * ask_cpu(s, a, row)) code = kTrCpu;
        else if (core_out) code = kTrCores;
        else if (r.cap_mem < r.used_mem + k1 * a.mem) code = kTrMemory;
        else if (r.cap_disk < r.used_disk + k1 * a.disk) code = kTrDisk;
    }
    if (code == kTrOption) {
        ScoreIn si;
        if (dk) {   // status_loaded applies dk itself: the network columns as loaded
            r.used_dyn -= (int32_t)dk * a.commit_dyn;
            r.used_mbits -= (int32_t)dk * a.commit_mbits;
        }
        if (status_loaded(s, t, t.class_ok, a, dk, row, in, &si) != kOption) {
            out[i] = kTrMismatch;
            return;
        }
        lookup_scores(t, penalty_bits, spread_tab, row, c, &si);
        NodeEval ev;
        score_option<true>(a, log10, si, &ev);
        double* o = sc + (size_t)i * 6;
        uint32_t k = 1;
        o[0] = ev.parts[0];
        o[1] = a.dev_tw != 0.0 ? ev.parts[k++] : 0.0;
        o[2] = (a.anti_aff && si.coll > 0) ? ev.parts[k++] : 0.0;
        if (si.penalty) { code |= kTrPenalty; k++; }
        o[3] = si.aff != 0.0 ? ev.parts[k++] : 0.0;
        o[4] = si.spread != 0.0 ? ev.parts[k++] : 0.0;
        o[5] = ev.score;
    }
    out[i] = code;
}

// ScoreMetaData of every record of a speculative run from k_trace's outcomes
// (rows of record k: rec_end[k-1] .. rec_end[k]): one wave per record pushes
// its options' NormScores in visit order into a 5-slot min-heap exactly as
// kheap.ScoreHeap.Push does under container/heap (replace the minimum only
// when strictly greater, heap.Fix, then up(len - 1); lib/kheap/score_heap.go),
// pops them (GetItemsReverse) and writes the NodeScoreMeta items in their
// binary form with the names metrics_outcome gives them
// (structs.go:9976-10018). flags: 1 devices scored, 2 job anti-affinity
// scored, 4 node affinities exist, 8 generic stack.
// A push that does not enter a full heap changes nothing, and the heap's
// minimum only grows. The record's entries are split among the block's waves;
// each wave keeps the top-5 NormScores of its own segment so far and lists the
// entries that enter it: an entry that does not enter its segment's top-5 is
// at or below the minimum of a heap that has seen at least that prefix, so it
// does not enter the record's heap either. Wave 0 then pushes the listed
// entries in order into the heap (held alike in every lane). A segment with
// more entering entries than its list holds sends the record to wave 0's
// sequential pass over every entry.
constexpr uint32_t kTopWaves = 16, kTopCand = 128;
// n_other (or null): per record, its entries that are not options, the first
// kTopOther of them (entry index within the record, code; in no particular
// order) at other_list + k * kTopOther.
constexpr uint32_t kTopOther = 128;
__global__ void __launch_bounds__(1024) k_trace_top(const uint32_t* codes, const double* sc, TraceSrc src,
                                                    uint32_t flags, pe_metric_score* out, uint8_t* n_out,
                                                    uint32_t* n_other, uint2* other_list) {
    __shared__ uint32_t cand_x[kTopWaves][kTopCand];
    __shared__ double cand_v[kTopWaves][kTopCand];
    __shared__ uint32_t cand_n[kTopWaves];
    __shared__ uint32_t overflow, others;
    const uint32_t k = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t nw = blockDim.x >> 6;
    if (k >= src.n_rec) return;   // uniform across the block
    const uint32_t b = k ? src.rec_end[k - 1] : 0u, e = src.rec_end[k];
    if (tid == 0) overflow = others = 0;
    __syncthreads();
    {   // phase 1: the segment's entering entries (and its entries that are not options)
        const uint32_t total = e - b, seg = (total + nw - 1) / nw;
        const uint32_t sb = b + min(total, w * seg), se = b + min(total, (w + 1) * seg);
        double t[5];   // the segment's top-5 so far (values), unsorted; tmin its minimum once full
        uint32_t tl = 0, nc = 0, n_not = 0;
        double tmin = 0.0;
        bool over = false;
        constexpr uint32_t U = 4;
        for (uint32_t c = sb; c < se; c += 64 * U) {
            uint32_t cd[U];
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t x = c + u * 64 + lane;
                cd[u] = x < se ? codes[x] : 0xFFFFFFFFu;
            }
#pragma unroll
            for (uint32_t u = 0; u < U; u++) {
                const uint32_t x = c + u * 64 + lane;
                const bool opt = (cd[u] & 255u) == kTrOption;
                const bool other = x < se && !opt;
                n_not += (uint32_t)__popcll(__ballot(other));
                if (other && other_list) {
                    const uint32_t q = atomicAdd(&others, 1u);
                    if (q < kTopOther) other_list[(size_t)k * kTopOther + q] = make_uint2(x - b, cd[u]);
                }
                const double v = opt ? sc[(size_t)x * 6 + 5] : 0.0;
                uint64_t mask = __ballot(opt && (tl < 5 || v > tmin));
                while (mask) {
                    const uint32_t l = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
                    mask &= mask - 1;
                    const double nv = __shfl(v, (int)l);
                    if (tl < 5) {
                        t[tl++] = nv;   // tl is wave-uniform: a static index after unrolling below
                    } else if (nv > tmin) {
                        bool done = false;   // replace one minimum
#pragma unroll
                        for (int q = 0; q < 5; q++)
                            if (!done && t[q] == tmin) { t[q] = nv; done = true; }
                    } else {
                        continue;
                    }
                    if (tl == 5) {
                        tmin = t[0];
#pragma unroll
                        for (int q = 1; q < 5; q++) tmin = t[q] < tmin ? t[q] : tmin;
                    }
                    if (nc < kTopCand) {
                        if (lane == 0) {
                            cand_x[w][nc] = c + u * 64 + l;
                            cand_v[w][nc] = nv;
                        }
                        nc++;
                    } else {
                        over = true;
                    }
                }
            }
        }
        if (lane == 0) {
            cand_n[w] = nc;
            if (over) atomicOr(&overflow, 1u);
            if (n_not && !other_list) atomicAdd(&others, n_not);
        }
    }
    __syncthreads();
    if (tid == 0 && n_other) n_other[k] = others;
    if (w != 0) return;
    double hn[5];
    uint32_t hi[5];
    uint32_t len = 0;
    auto less = [&](uint32_t x, uint32_t y) { return hn[x] < hn[y]; };
    auto swap_ = [&](uint32_t x, uint32_t y) {
        const double tn = hn[x]; hn[x] = hn[y]; hn[y] = tn;
        const uint32_t ti = hi[x]; hi[x] = hi[y]; hi[y] = ti;
    };
    auto up = [&](uint32_t j) {
        while (j > 0) {
            const uint32_t i = (j - 1) / 2;
            if (!less(j, i)) break;
            swap_(i, j);
            j = i;
        }
    };
    auto down = [&](uint32_t i0, uint32_t n) {
        uint32_t i = i0;
        for (;;) {
            const uint32_t j1 = 2 * i + 1;
            if (j1 >= n) break;
            uint32_t j = j1;
            if (j1 + 1 < n && less(j1 + 1, j1)) j = j1 + 1;
            if (!less(j, i)) break;
            swap_(i, j);
            i = j;
        }
        return i > i0;
    };
    auto push = [&](double norm, uint32_t x) {   // ScoreHeap.Push under container/heap
        if (len < 5) {
            hn[len] = norm;
            hi[len] = x;
            len++;
        } else if (norm > hn[0]) {
            hn[0] = norm;
            hi[0] = x;
            if (!down(0, len)) up(0);
        }
        up(len - 1);
    };
    if (!overflow) {
        for (uint32_t q = 0; q < nw; q++)
            for (uint32_t i = 0; i < cand_n[q]; i++) push(cand_v[q][i], cand_x[q][i]);
    } else {   // every entry in order, 64 at a time (a candidate pass over the whole record)
        for (uint32_t c = b; c < e; c += 64) {
            const uint32_t x = c + lane;
            const bool opt = x < e && (codes[x] & 255u) == kTrOption;
            const double v = opt ? sc[(size_t)x * 6 + 5] : 0.0;
            uint64_t mask = __ballot(opt && (len < 5 || v > hn[0]));
            while (mask) {
                const uint32_t l = (uint32_t)__ffsll((unsigned long long)mask) - 1u;
                mask &= mask - 1;
                push(__shfl(v, (int)l), c + l);
            }
        }
    }
    if (lane != 0) return;
    // GetItemsReverse: heap.Pop until empty, the last popped first
    uint32_t order[5];
    const uint32_t total = len;
    uint32_t at = total;
    while (len > 0) {
        const uint32_t n = len - 1;
        swap_(0, n);
        down(0, n);
        order[--at] = hi[n];
        len--;
    }
    n_out[k] = (uint8_t)total;
    for (uint32_t q = 0; q < total; q++) {
        const uint32_t x = order[q];
        const double* o = sc + (size_t)x * 6;
        pe_metric_score m;
        for (int j = 0; j < PE_MAX_SCORES; j++) { m.scorer[j] = 0; m.score[j] = 0.0; }
        uint32_t ns = 0;
        m.scorer[ns] = PE_SCORER_BINPACK; m.score[ns++] = o[0];
        if (flags & 1u) { m.scorer[ns] = PE_SCORER_DEVICES; m.score[ns++] = o[1]; }
        if (flags & 8u) {   // the SystemStack ranks with BinPack alone (stack.go:277-281)
            if (flags & 2u) { m.scorer[ns] = PE_SCORER_JOB_ANTI_AFFINITY; m.score[ns++] = o[2]; }
            m.scorer[ns] = PE_SCORER_RESCHEDULE_PENALTY;
            m.score[ns++] = (codes[x] & kTrPenalty) ? -1.0 : 0.0;
            if (!(flags & 4u)) { m.scorer[ns] = PE_SCORER_NODE_AFFINITY; m.score[ns++] = 0.0; }
            else if (o[3] != 0.0) { m.scorer[ns] = PE_SCORER_NODE_AFFINITY; m.score[ns++] = o[3]; }
            if (o[4] != 0.0) { m.scorer[ns] = PE_SCORER_ALLOCATION_SPREAD; m.score[ns++] = o[4]; }
        }
        m.row = (int32_t)trace_row(src, k, x - b);
        m.n_scores = ns;
        m.norm = o[5];
        out[(size_t)k * 5 + q] = m;
    }
}

// evenSpreadScoreBoost (spread.go:178-228) / target boost (spread.go:143-164)
// per value of each property set, from the eval's use counts: `counts` in the
// pset_cnt_off layout (an LDS copy, or the loop's own counts), or null to read
// each set's HBM counts. `tab` in the pset_tab_off layout.
template <int BLOCK>
__device__ void build_spread_table(const TgTables& t, const uint32_t* counts, double* tab, uint32_t* scratch) {
    const int tid = threadIdx.x;
    for (int p = 0; p < t.n_psets; p++) {
        const int nv = t.pset_nvals[p];
        const uint32_t* cnt = counts ? counts + t.pset_cnt_off[p] : t.pset_counts[p];
        double* tb = tab + t.pset_tab_off[p];
        if (p >= t.n_spread) {   // distinct_property: 1.0 marks a value at its allowed count
            for (int v = tid; v < nv; v += BLOCK) tb[v] = cnt[v] >= t.pset_allowed[p] ? 1.0 : 0.0;
            continue;
        }
        if (t.pset_even[p]) {
            // min / max / number of the used values (any count of values: a
            // block reduction, the same integers as the reference's map walk)
            uint32_t lmn = 0xFFFFFFFFu, lmx = 0, lpr = 0;
            for (int v = tid; v < nv; v += BLOCK) {
                const uint32_t x = cnt[v];
                if (x == 0) continue;
                lpr++;
                lmn = x < lmn ? x : lmn;
                lmx = x > lmx ? x : lmx;
            }
            for (int off = 32; off > 0; off >>= 1) {
                lmn = min(lmn, (uint32_t)__shfl_xor((int)lmn, off));
                lmx = max(lmx, (uint32_t)__shfl_xor((int)lmx, off));
                lpr += (uint32_t)__shfl_xor((int)lpr, off);
            }
            if (tid == 0) { scratch[0] = 0xFFFFFFFFu; scratch[1] = 0; scratch[2] = 0; }
            __syncthreads();
            if ((tid & 63) == 0) {
                atomicMin(&scratch[0], lmn);
                atomicMax(&scratch[1], lmx);
                atomicAdd(&scratch[2], lpr);
            }
            __syncthreads();
            if (tid == 0 && scratch[2] == 0) { scratch[0] = 0; }   // no used value: min = max = 0
            __syncthreads();
            const uint32_t mn = scratch[0], mx = scratch[1], present = scratch[2];
            for (int v = tid; v < nv; v += BLOCK) {
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
                tb[v] = b;
            }
            __syncthreads();
        } else {
            for (int v = tid; v < nv; v += BLOCK) {
                const double desired = t.pset_desired[p][v];
                double b;
                if (desired != desired) b = -1.0;   // no target and no implicit "*"
                else {
                    const double used = (double)(cnt[v] + 1u);
                    b = ((desired - used) / desired) * t.pset_weight_frac[p];
                }
                tb[v] = b;
            }
        }
    }
    __syncthreads();
}

template <int BLOCK>
struct LoopShared {
    uint32_t scratch[4];
    uint32_t wave_a[BLOCK / 64];
    uint32_t wave_b[BLOCK / 64];
    double red_score[BLOCK / 64];
    int red_pos[BLOCK / 64];
    double aside_score[kMaxSkip];   // LimitIterator skip list
    int aside_pos[kMaxSkip];
    int stop_j;
    SweepRec red_rec[BLOCK / 64];   // full-pass mode: per-wave records
};

template <int BLOCK>
__device__ __forceinline__ void block_sync() {
    if constexpr (BLOCK > 64) __syncthreads();
}

// Ordering point for a single-wave workgroup: one wave's LDS operations execute
// in program order, so a wavefront-scope fence (a compiler barrier, no waits)
// is all the cross-lane hand-off through LDS needs. Unlike __syncthreads it
// does not drain outstanding global stores.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m, int lane) {
    return (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}

// Exclusive block prefix of a predicate; *total = block count.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_prefix(bool pred, uint32_t* wave_tot, uint32_t* total) {
    const int lane = threadIdx.x & 63;
    const uint64_t m = __ballot(pred);
    if constexpr (BLOCK == 64) {
        *total = (uint32_t)__popcll(m);
        return lanes_below(m, lane);
    } else {
        constexpr int W = BLOCK / 64;
        const int wid = threadIdx.x >> 6;
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
}

// first strict maximum: max score, ties -> smallest position
template <int BLOCK>
__device__ __forceinline__ void block_argmax(bool cand, double score, int pos, double* red_score, int* red_pos,
                                             double* best_score, int* best_pos) {
    double s = cand ? score : -__builtin_inf();
    int p = cand ? pos : 0x7FFFFFFF;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double os = __shfl_xor(s, off);
        const int op = __shfl_xor(p, off);
        if (os > s || (os == s && op < p)) { s = os; p = op; }
    }
    if constexpr (BLOCK == 64) {
        *best_score = s;
        *best_pos = p;
    } else {
        constexpr int W = BLOCK / 64;
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
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
}

// Plan.AppendAlloc into the overlay (one lane).
__device__ __forceinline__ void commit_overlay(const NodeSoA& s, const TgTables& t, const Overlay& ov,
                                               uint32_t* counts, uint32_t row) {
    ov_add(ov, row);
    if (t.n_psets > 0) {
        const uint32_t c = s.rec[row].cls;
        for (int p = 0; p < t.n_psets; p++) {
            const uint32_t v = pset_value(t, p, row, c);
            if (v != kMissing) counts[t.pset_cnt_off[p] + v] += 1;
        }
    }
}

// TaskResources device offers of the chosen node (one lane).
__device__ __forceinline__ void record_offers(const NodeSoA& s, const Ask& a, const TgTables& t, uint32_t row,
                                              uint32_t dk, pe_ranked_node* o) {
    o->n_device_offers = 0;
    o->n_preempted = 0;
    if (a.n_dev <= 0) return;
    const DevClass& dc = t.dev_cls[s.rec[row].cls];
    uint32_t fr = dev_after(a, dc, t.dev_free[row], dk);
    double m;
    uint32_t groups[kMaxDevReq];
    if (!dev_assign(a, dc, fr, &m, groups)) return;
    o->n_device_offers = (uint32_t)a.n_dev;
    for (int q = 0; q < kMaxDevReq; q++)
        if (q < a.n_dev) o->device_offer_group[q] = groups[q];
}

// Result records of placement `it` of evaluation e (one lane).
template <bool kCores = true>
__device__ __forceinline__ void emit_placement(const BatchArgs& A, const uint8_t* class_ok, const Overlay& ov,
                                            const double* spread_tab, uint32_t e, uint32_t it, int win_row,
                                            double best_score, uint32_t consumed, uint32_t n_filtered,
                                            uint32_t n_exhausted, uint32_t new_offset) {
    if (A.full_out) {
        pe_ranked_node& o = A.full_out[(size_t)e * A.count + it];
        o.row = win_row;
        o.nodes_evaluated = consumed;
        o.nodes_filtered = n_filtered;
        o.nodes_exhausted = n_exhausted;
        o.new_offset = new_offset;
        o.final_score = 0.0;
        o.n_scores = 0;
        o.n_preempted = 0;
        o.n_device_offers = 0;
        for (int k = 0; k < PE_MAX_SCORES; k++) o.scores[k] = 0.0;
        if (win_row >= 0) {
            NodeEval ev;
            eval_node<true, kCores>(A.soa, A.tg, class_ok, A.ask, ov, A.penalty_bits, A.log10, spread_tab,
                                    (uint32_t)win_row, &ev);
            o.final_score = ev.score;
            o.n_scores = ev.nscores;
            for (int k = 0; k < (int)ev.nscores && k < PE_MAX_SCORES; k++) o.scores[k] = ev.parts[k];
            record_offers(A.soa, A.ask, A.tg, (uint32_t)win_row, ov_count(ov, (uint32_t)win_row), &o);
        }
    }
    if (A.out) {
        pe_placement& o = A.out[(size_t)e * A.count + it];
        o.row = win_row;
        o.nodes_evaluated = consumed;
        o.final_score = win_row >= 0 ? best_score : 0.0;
    }
}

// ---- full-pass reduction records (LimitIterator with limit >= options) -------
__host__ __device__ __forceinline__ void rec_init(SweepRec& r) {
    r.max_score = -__builtin_inff();
    for (int i = 0; i < 4; i++) r.max_rank[i] = 0xFFFFFFFFu;
    for (int i = 0; i < kMaxSkip; i++) { r.np_rank[i] = 0xFFFFFFFFu; r.np_score[i] = 0.0; }
    r.options = r.filtered = r.exhausted = r._pad = 0;
}

// insert x into a sorted list of N ranks (keeps the N smallest); branch-free on indices
template <int N>
__host__ __device__ __forceinline__ void ins_rank(uint32_t (&l)[N], uint32_t x) {
#pragma unroll
    for (int i = 0; i < N; i++) {
        const uint32_t lo = l[i] < x ? l[i] : x, hi = l[i] < x ? x : l[i];
        l[i] = lo;
        x = hi;
    }
}

__host__ __device__ __forceinline__ void ins_np(uint32_t (&rk)[kMaxSkip], double (&sc)[kMaxSkip], uint32_t x, double s) {
#pragma unroll
    for (int i = 0; i < kMaxSkip; i++) {
        if (x < rk[i]) {
            const uint32_t tr = rk[i]; const double ts = sc[i];
            rk[i] = x; sc[i] = s;
            x = tr; s = ts;
        }
    }
}

__device__ __forceinline__ void rec_add(SweepRec& r, uint32_t rank, double score) {
    r.options++;
    if (score > r.max_score) {
        r.max_score = score;
        r.max_rank[0] = rank;
        r.max_rank[1] = r.max_rank[2] = r.max_rank[3] = 0xFFFFFFFFu;
    } else if (score == r.max_score) {
        ins_rank<4>(r.max_rank, rank);
    }
    if (score <= 0.0) ins_np(r.np_rank, r.np_score, rank, score);
}

__host__ __device__ __forceinline__ void rec_merge(SweepRec& a, const SweepRec& b) {
    if (b.max_score > a.max_score) {
        a.max_score = b.max_score;
        for (int i = 0; i < 4; i++) a.max_rank[i] = b.max_rank[i];
    } else if (b.max_score == a.max_score) {
        for (int i = 0; i < 4; i++) ins_rank<4>(a.max_rank, b.max_rank[i]);
    }
    for (int i = 0; i < kMaxSkip; i++) ins_np(a.np_rank, a.np_score, b.np_rank[i], b.np_score[i]);
    a.options += b.options;
    a.filtered += b.filtered;
    a.exhausted += b.exhausted;
}

// Winner rank of a merged record, ~0u = no option.
__device__ __host__ __forceinline__ uint32_t rec_winner(const SweepRec& r) {
    if (r.options == 0) return 0xFFFFFFFFu;
    if (r.max_score > 0.0) return r.max_rank[0];
    for (int i = 0; i < 4; i++) {
        const uint32_t x = r.max_rank[i];
        if (x == 0xFFFFFFFFu) break;
        bool demoted = false;
        for (int k = 0; k < kMaxSkip; k++) demoted = demoted || r.np_rank[k] == x;
        if (!demoted) return x;
    }
    return r.max_rank[0];
}

__device__ __forceinline__ SweepRec rec_shfl_xor(const SweepRec& r, int off) {
    SweepRec o;
    o.max_score = __shfl_xor(r.max_score, off);
#pragma unroll
    for (int i = 0; i < 4; i++) o.max_rank[i] = (uint32_t)__shfl_xor((int)r.max_rank[i], off);
#pragma unroll
    for (int i = 0; i < kMaxSkip; i++) {
        o.np_rank[i] = (uint32_t)__shfl_xor((int)r.np_rank[i], off);
        o.np_score[i] = __shfl_xor(r.np_score[i], off);
    }
    o.options = (uint32_t)__shfl_xor((int)r.options, off);
    o.filtered = (uint32_t)__shfl_xor((int)r.filtered, off);
    o.exhausted = (uint32_t)__shfl_xor((int)r.exhausted, off);
    o._pad = 0;
    return o;
}

// Block reduction of per-thread records; the merge is commutative and
// associative over disjoint row sets, so an xor butterfly inside each wave is
// exact. Thread 0 returns the block's record.
template <int BLOCK>
__device__ __forceinline__ void rec_block_reduce(SweepRec& r, SweepRec* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const SweepRec o = rec_shfl_xor(r, off);
        rec_merge(r, o);
    }
    constexpr int W = BLOCK / 64;
    if constexpr (W > 1) {
        const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
        if (lane == 0) red[wid] = r;
        __syncthreads();
        if (threadIdx.x == 0)
            for (int w = 1; w < W; w++) rec_merge(r, red[w]);
    }
}

// Merge an evaluation's overlay into the HBM SoA (the stack's plan persists).
template <int BLOCK, bool FULL, bool kCores = true>
__device__ void writeback_overlay(const BatchArgs& A, const Overlay& ov, uint32_t H, const uint32_t* counts) {
    for (uint32_t h = threadIdx.x; h < H; h += BLOCK) {
        const uint32_t e = ov.keys[h];
        if (e == kEmpty) continue;
        const uint32_t row = ov.k ? e : e >> ov.kshift;
        const uint32_t k = ov.k ? ov.k[h] : e & ov.kmask;
        NodeRec& r = A.soa.rec[row];
        if (kCores) {
            r.used_cpu += (int64_t)k * ask_cpu(A.soa, A.ask, row);
            core_take(A.soa, A.ask, row, k);
        } else {
            r.used_cpu += (int64_t)k * A.ask.cpu;
        }
        r.used_mem += (int64_t)k * A.ask.mem;
        r.used_disk += (int64_t)k * A.ask.disk;
        r.used_mbits += (int32_t)k * A.ask.commit_mbits;
        r.used_dyn += (int32_t)k * A.ask.commit_dyn;
        A.soa.coll_job[row] += k;
        A.tg.coll_tg[row] += k;
        if (A.ask.n_dev > 0) A.tg.dev_free[row] = dev_after(A.ask, A.tg.dev_cls[r.cls], A.tg.dev_free[row], k);
    }
    if constexpr (FULL) {
        for (int q = 0; q < A.tg.n_psets; q++)
            for (int v = threadIdx.x; v < A.tg.pset_nvals[q]; v += BLOCK)
                A.tg.pset_counts[q][v] = counts[A.tg.pset_cnt_off[q] + v];
    }
}

template <int BLOCK, bool FULL, bool CORES>
__global__ void __launch_bounds__(BLOCK) k_place(BatchArgs A) {
    __shared__ LoopShared<BLOCK> sh;
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
    const int tid = threadIdx.x;
    const uint32_t e = blockIdx.x;
    const uint32_t n = A.n_visit;
    const uint32_t* perm = A.perms + (size_t)e * A.perm_stride;
    const uint8_t* class_ok = A.tg.class_ok + (size_t)e * A.class_ok_stride;

    // carve the overlay (and spread tables) out of dynamic LDS
    const uint32_t H = 1u << A.hash_bits;
    unsigned char* p = dyn_smem;
    double* spread_tab = nullptr;
    uint32_t* counts = nullptr;
    if constexpr (FULL) {
        if (A.pset_g_tab) {   // tables beyond the LDS budget: this evaluation's HBM copy
            spread_tab = A.pset_g_tab + (size_t)e * A.tg.pset_tab_total;
            counts = A.pset_g_cnt + (size_t)e * A.tg.pset_cnt_total;
        } else {
            spread_tab = reinterpret_cast<double*>(p);
            counts = reinterpret_cast<uint32_t*>(p + sizeof(double) * A.tg.pset_tab_total);
            p += A.pset_lds;
        }
    }
    Overlay ov;
    ov.bits = A.hash_bits;
    ov.mask = H - 1;
    ov.keys = reinterpret_cast<uint32_t*>(p); p += 4 * H;
    ov.k = reinterpret_cast<uint32_t*>(p); p += 4 * H;
    for (uint32_t i = tid; i < H; i += BLOCK) ov.keys[i] = kEmpty;
    if constexpr (FULL) {
        for (int q = 0; q < A.tg.n_psets; q++)
            for (int v = tid; v < A.tg.pset_nvals[q]; v += BLOCK) counts[A.tg.pset_cnt_off[q] + v] = A.tg.pset_counts[q][v];
    }
    __syncthreads();

    uint32_t offset = A.offsets ? A.offsets[e] : A.offset0;
    if (n) offset %= n;
    uint32_t placed = 0;

    for (uint32_t it = 0; it < A.count; it++) {
        if constexpr (FULL) {
            if (A.tg.n_psets > 0) build_spread_table<BLOCK>(A.tg, counts, spread_tab, sh.scratch);
        }
        uint32_t r = 0, a = 0;            // returned / set-aside options so far
        double best_score = -__builtin_inf();
        int best_pos = -1;                // relative visit position of the winner
        uint32_t n_filtered = 0, n_exhausted = 0;
        uint32_t consumed = n;
        bool stopped = false;

        if (FULL && A.limit >= n) {
            // A full pass (limit >= every option): no prefix walk,
            // each lane folds its positions into a SweepRec, one block reduction
            // per placement gives the winner and the counters.
            SweepRec rec;
            rec_init(rec);
            for (uint32_t j = tid; j < n; j += BLOCK) {
                uint32_t pos = offset + j;
                if (pos >= n) pos -= n;
                NodeEval ev;
                eval_node<false, CORES>(A.soa, A.tg, class_ok, A.ask, ov, A.penalty_bits, A.log10, spread_tab, perm[pos], &ev);
                if (ev.status == kFiltered) rec.filtered++;
                else if (ev.status == kExhausted) rec.exhausted++;
                else rec_add(rec, j, ev.score);
            }
            rec_block_reduce<BLOCK>(rec, sh.red_rec);
            if (tid == 0) {
                const uint32_t w = rec_winner(rec);
                sh.stop_j = w == 0xFFFFFFFFu ? -1 : (int)w;
                sh.scratch[0] = rec.filtered;
                sh.scratch[1] = rec.exhausted;
                sh.red_score[0] = rec.max_score;   // the winner always scores the maximum
            }
            __syncthreads();
            best_pos = sh.stop_j;
            best_score = sh.red_score[0];
            n_filtered = sh.scratch[0];
            n_exhausted = sh.scratch[1];
            consumed = n;
            stopped = true;   // nothing set aside to append
            __syncthreads();
        }

        for (uint32_t base = 0; base < n && !(FULL && A.limit >= n); base += BLOCK) {
            const uint32_t j = base + tid;
            const bool valid = j < n;
            NodeEval ev;
            ev.status = kFiltered;
            ev.score = 0.0;
            if (valid) {
                uint32_t pos = offset + j;
                if (pos >= n) pos -= n;
                const uint32_t row = perm[pos];
                eval_node<false, CORES>(A.soa, A.tg, class_ok, A.ask, ov, A.penalty_bits, A.log10, spread_tab, row, &ev);
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
            const bool is_stop = ret && ret_before == A.limit - 1u;
            const uint64_t sm = __ballot(is_stop);
            int stop_j;
            if constexpr (BLOCK == 64) {
                stop_j = sm ? (int)__ffsll((long long)sm) - 1 : -1;
            } else {
                if (tid == 0) sh.stop_j = -1;
                __syncthreads();
                if (is_stop) sh.stop_j = tid;
                __syncthreads();
                stop_j = sh.stop_j;
            }
            const bool pulled = valid && (stop_j < 0 || tid <= stop_j);
            if (aside && pulled) {
                sh.aside_score[np_before] = ev.score;
                sh.aside_pos[np_before] = (int)j;
            }
            const bool cand = ret && ret_before < A.limit;
            double cs;
            int cp;
            block_argmax<BLOCK>(cand, ev.score, (int)j, sh.red_score, sh.red_pos, &cs, &cp);
            if (cp != 0x7FFFFFFF && cs > best_score) { best_score = cs; best_pos = cp; }
            uint32_t f_tot, e_tot, a_tot;
            block_prefix<BLOCK>(pulled && ev.status == kFiltered, sh.wave_a, &f_tot);
            block_prefix<BLOCK>(pulled && ev.status == kExhausted, sh.wave_b, &e_tot);
            block_prefix<BLOCK>(aside && pulled, sh.wave_a, &a_tot);
            n_filtered += f_tot;
            n_exhausted += e_tot;
            a += a_tot;
            if (stop_j >= 0) {
                consumed = base + (uint32_t)stop_j + 1u;
                r = A.limit;
                stopped = true;
                break;
            }
            r += ret_tot;
        }
        block_sync<BLOCK>();
        if (!stopped) {
            // source exhausted: set-aside options are emitted in order until the limit
            const uint32_t take = min(a, A.limit - r);
            for (uint32_t i = 0; i < take; i++) {
                if (sh.aside_score[i] > best_score) { best_score = sh.aside_score[i]; best_pos = sh.aside_pos[i]; }
            }
        }
        int win_row = -1;
        if (best_pos >= 0) {
            uint32_t pos = offset + (uint32_t)best_pos;
            if (pos >= n) pos -= n;
            win_row = (int)perm[pos];
        }
        uint32_t no = n ? offset + (consumed % n) : 0u;
        if (no >= n) no -= n;
        if (tid == 0) {
            emit_placement<CORES>(A, class_ok, ov, spread_tab, e, it, win_row, best_score, consumed, n_filtered,
                           n_exhausted, no);
            if (win_row >= 0 && A.commit) commit_overlay(A.soa, A.tg, ov, counts, (uint32_t)win_row);
        }
        offset = no;
        __syncthreads();
        if (win_row < 0) break;   // nil option: failedTGAllocs short-circuit
        placed++;
    }
    if (tid == 0) {
        A.eval_status[2 * e] = placed;
        A.eval_status[2 * e + 1] = offset;
    }
    if (A.writeback) writeback_overlay<BLOCK, FULL, CORES>(A, ov, H, counts);
}

// Windowed count loop (limit < n: no affinities or spreads, so a node's result
// depends only on the snapshot and its own overlay count). One wave per
// evaluation. Each placement pulls ~limit + filtered positions but a wave
// evaluates 64 at a time, so the wave keeps a 128-position ring of evaluated
// visit positions in registers (slot s of lane l = ring index 64 s + l) and
// evaluates a chunk only when the pull runs past the cache. Committing the
// winner changes only that node's overlay count: the cache is cut at the first
// cached position holding the winner's row (only reachable when the visit list
// wraps inside the ring, n < 128). Chunks are aligned to the ring so every lane
// reads its own registers; the LimitIterator / MaxScoreIterator closed form is
// the same ballot logic as k_place.
__global__ void __launch_bounds__(64) k_window(BatchArgs A) {
    __shared__ double aside_score[kMaxSkip];
    __shared__ int aside_pos[kMaxSkip];
    __shared__ pe_placement stage[64];
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
    const int lane = threadIdx.x;
    const uint32_t e = blockIdx.x;
    const uint32_t n = A.n_visit;
    const uint32_t* perm = A.perms + (size_t)e * A.perm_stride;
    const uint8_t* class_ok = A.tg.class_ok + (size_t)e * A.class_ok_stride;
    const uint32_t H = 1u << A.hash_bits;
    Overlay ov;
    ov.bits = A.hash_bits;
    ov.mask = H - 1;
    ov.keys = reinterpret_cast<uint32_t*>(dyn_smem);
    ov.k = A.packed_overlay ? nullptr : ov.keys + H;
    ov.kshift = A.packed_overlay;
    ov.kmask = A.packed_overlay ? (1u << A.packed_overlay) - 1u : 0u;
    for (uint32_t i = lane; i < H; i += 64) ov.keys[i] = kEmpty;
    __syncthreads();

    uint32_t offset = A.offsets ? A.offsets[e] : A.offset0;
    if (n) offset %= n;
    uint32_t placed = 0;
    int st0 = kFiltered, st1 = kFiltered;
    double sc0 = 0.0, sc1 = 0.0;
    uint32_t rw0 = kEmpty, rw1 = kEmpty;
    uint32_t rb = 0;     // ring index of the cursor
    uint32_t have = 0;   // relative positions [0, have) are cached (have <= min(n, 128) at loop top)

    for (uint32_t it = 0; it < A.count; it++) {
        uint32_t r = 0, a = 0;
        double best_score = -__builtin_inf();
        int best_pos = -1;
        uint32_t n_filtered = 0, n_exhausted = 0;
        uint32_t consumed = n;
        bool stopped = false;
        double lbest_s = -__builtin_inf();
        int lbest_p = -1;
        const uint32_t skew = rb & 63u;
        for (uint32_t k = 0; 64u * k < n + skew; k++) {
            const int j = (int)(64u * k + (uint32_t)lane) - (int)skew;   // relative visit position
            const bool valid = j >= 0 && (uint32_t)j < n;
            const bool s1 = (((rb >> 6) + k) & 1u) != 0;
            int st = s1 ? st1 : st0;
            double sc = s1 ? sc1 : sc0;
            const bool need = valid && (uint32_t)j >= have;
            if (__ballot(need)) {
                // The pull ran past the cache: evaluate this chunk and the next
                // one (every position >= have is uncached), all loads in flight
                // before any compute.
                const uint32_t j2 = (uint32_t)(j + 64);
                const bool need2 = j2 < n;
                uint32_t p1 = need ? offset + (uint32_t)j : 0u;
                uint32_t p2 = need2 ? offset + j2 : 0u;
                if (p1 >= n) p1 -= n;
                if (p2 >= n) p2 -= n;
                const uint32_t row1 = perm[p1], row2 = perm[p2];
                NodeIn in1, in2;
                load_node(A.soa, A.tg, row1, in1);
                load_node(A.soa, A.tg, row2, in2);
                const uint32_t dk1 = ov_count(ov, row1), dk2 = ov_count(ov, row2);
                NodeEval e1, e2;
                e1.score = 0.0;
                e2.score = 0.0;
                eval_loaded<false>(A.soa, A.tg, class_ok, A.ask, dk1, A.penalty_bits, A.log10, nullptr, row1, in1,
                                   &e1);
                eval_loaded<false>(A.soa, A.tg, class_ok, A.ask, dk2, A.penalty_bits, A.log10, nullptr, row2, in2,
                                   &e2);
                if (need) {
                    st = e1.status;
                    sc = e1.score;
                    if (s1) { st1 = st; sc1 = sc; rw1 = row1; } else { st0 = st; sc0 = sc; rw0 = row1; }
                }
                if (need2) {
                    if (s1) { st0 = e2.status; sc0 = e2.score; rw0 = row2; }
                    else { st1 = e2.status; sc1 = e2.score; rw1 = row2; }
                }
                have = min(64u * (k + 2) - skew, n);
            }

            const bool is_opt = valid && st == kOption;
            const bool is_np = is_opt && sc <= 0.0;
            uint32_t np_tot;
            const uint32_t np_before = a + block_prefix<64>(is_np, nullptr, &np_tot);
            const bool aside = is_np && np_before < (uint32_t)kMaxSkip;
            const bool ret = is_opt && !aside;
            uint32_t ret_tot;
            const uint32_t ret_before = r + block_prefix<64>(ret, nullptr, &ret_tot);
            const uint64_t sm = __ballot(ret && ret_before == A.limit - 1u);
            const int stop_lane = sm ? (int)__ffsll((long long)sm) - 1 : 64;
            const bool pulled = valid && lane <= stop_lane;
            if (aside && pulled) {
                aside_score[np_before] = sc;
                aside_pos[np_before] = j;
            }
            // lane-local first strict maximum; positions grow with the chunk,
            // so one wave reduction per placement suffices
            if (ret && ret_before < A.limit && sc > lbest_s) { lbest_s = sc; lbest_p = j; }
            if (A.full_out) {
                n_filtered += (uint32_t)__popcll(__ballot(pulled && st == kFiltered));
                n_exhausted += (uint32_t)__popcll(__ballot(pulled && st == kExhausted));
            }
            a += (uint32_t)__popcll(__ballot(aside && pulled));
            if (sm) {
                consumed = 64u * k + (uint32_t)stop_lane - skew + 1u;
                r = A.limit;
                stopped = true;
                break;
            }
            r += ret_tot;
        }
        {
            double cs;
            int cp;
            block_argmax<64>(lbest_p >= 0, lbest_s, lbest_p, nullptr, nullptr, &cs, &cp);
            if (cp != 0x7FFFFFFF) { best_score = cs; best_pos = cp; }
        }
        if (!stopped) {
            const uint32_t take = min(a, A.limit - r);
            for (uint32_t i = 0; i < take; i++) {
                if (aside_score[i] > best_score) { best_score = aside_score[i]; best_pos = aside_pos[i]; }
            }
        }
        int win_row = -1;
        if (best_pos >= 0) {
            if (best_pos + 128 >= (int)have) {
                // still in the ring: positions [have - 128, have) are intact
                const uint32_t idx = (rb + (uint32_t)best_pos) & 127u;
                win_row = __shfl((int)((idx & 64u) ? rw1 : rw0), (int)(idx & 63u));
            } else {
                uint32_t pos = offset + (uint32_t)best_pos;
                if (pos >= n) pos -= n;
                win_row = (int)perm[pos];
            }
        }
        uint32_t no = n ? offset + (consumed % n) : 0u;
        if (no >= n) no -= n;
        if (lane == 0) {
            if (A.full_out)
                emit_placement(A, class_ok, ov, nullptr, e, it, win_row, best_score, consumed, n_filtered,
                               n_exhausted, no);
            pe_placement& o = stage[it & 63u];
            o.row = win_row;
            o.nodes_evaluated = consumed;
            o.final_score = win_row >= 0 ? best_score : 0.0;
            if (win_row >= 0 && A.commit) ov_add(ov, (uint32_t)win_row);
        }
        wave_sync();
        // compact records leave in 1 KB wave stores (possibly straight into
        // mapped host memory, so the transfer overlaps the count loop)
        if (A.out && ((it & 63u) == 63u || win_row < 0 || it + 1 == A.count)) {
            const uint32_t fill = (it & 63u) + 1u;
            if ((uint32_t)lane < fill)
                A.out[(size_t)e * A.count + (it + 1u - fill) + lane] = stage[lane];
        }
        offset = no;
        // slide the cache: a full pass (no stop) leaves the cursor in place but
        // the ring is keyed by unwrapped position, so it restarts empty
        if (stopped) {
            rb = (rb + consumed) & 127u;
            have = have > consumed ? have - consumed : 0u;
        } else {
            have = 0;
        }
        if (win_row >= 0 && A.commit && have) {
            const uint32_t j0 = ((uint32_t)lane - rb) & 127u, j1 = (64u + (uint32_t)lane - rb) & 127u;
            const bool bad0 = j0 < have && rw0 == (uint32_t)win_row;
            const bool bad1 = j1 < have && rw1 == (uint32_t)win_row;
            if (__ballot(bad0 || bad1)) {
                uint32_t cut = min(bad0 ? j0 : 128u, bad1 ? j1 : 128u);
                for (int off = 32; off > 0; off >>= 1) cut = min(cut, (uint32_t)__shfl_xor((int)cut, off));
                if (cut < have) have = cut;
            }
        }
        wave_sync();
        if (win_row < 0) break;
        placed++;
    }
    if (lane == 0) {
        A.eval_status[2 * e] = placed;
        A.eval_status[2 * e + 1] = offset;
    }
    if (A.writeback) writeback_overlay<64, false>(A, ov, H, nullptr);
}

// ---- shared base table ----------------------------------------------------------
__device__ __forceinline__ double encode_eval(const NodeEval& ev) {
    return ev.status == kOption ? ev.score : (ev.status == kFiltered ? -__builtin_inf() : __builtin_inf());
}

// base[row]: the fused pipeline of every row of the snapshot with no placement
// of this launch on it. It does not depend on the visit order, so one pass
// serves every evaluation of a batch. base1 (one placement on the row) is
// computed by a second set of lanes rather than after base in the same lane:
// the pass is one dependent load + evaluate chain per lane, so the two tables
// finish in the time of one; 64-lane workgroups spread it over more CUs. The
// two lanes of one position are neighbours in a wave, so the row's column
// lines are fetched once for both (halves in separate workgroups landed on
// separate XCDs and fetched every line twice).
// With FOLD the launch also carries the FeasibilityWrapper fold (FoldArgs):
// each workgroup pulls the class verdict table from the staging ring into LDS,
// the grid stores node_feas for every row (the later kernels read it), and the
// evaluation reads the verdict from the table (no dependency on another
// workgroup's stores).
constexpr int kBaseBlock = 64;
template <bool FOLD>
__global__ void __launch_bounds__(kBaseBlock) k_base(BatchArgs A) {
    __shared__ uint8_t cls_ok[FOLD ? kFoldMaxClasses : 1];
    const uint32_t stride = gridDim.x * kBaseBlock;
    // the tables straight from the kernel arguments: a local copy of TgTables
    // (its per-set arrays are indexed at run time) lived in scratch, 680 B per
    // lane written and read back by every launch
    const TgTables& tg = A.tg;
    const uint8_t* class_ok = A.tg.class_ok;
    auto fold_ok = [&](uint32_t row, uint32_t c) {
        bool ok = c < A.fold.ncls && cls_ok[c] != 0;
        if (A.fold.node_ok) ok = ok && A.fold.node_ok[row] != 0;
        return ok;
    };
    if (FOLD) {
        const FoldArgs& F = A.fold;
        for (uint32_t c = threadIdx.x; c < F.ncls; c += kBaseBlock) {
            const uint8_t v = F.class_src[c];
            cls_ok[c] = v;
            if (blockIdx.x == 0) F.class_dst[c] = v;
        }
        __syncthreads();
        for (uint32_t row = blockIdx.x * kBaseBlock + threadIdx.x; row < A.soa.n; row += stride)
            F.feas[row] = fold_ok(row, A.soa.rec[row].cls) ? 1 : 0;
        class_ok = cls_ok;
    }
    const uint32_t m = A.base_by_pos ? A.n_visit : A.soa.n;
    const uint32_t sh = A.base1 ? 1u : 0u;
    const uint32_t total = m << sh;
    for (uint32_t t = blockIdx.x * kBaseBlock + threadIdx.x; t < total; t += stride) {
        const uint32_t dk = t & sh;
        const uint32_t j = t >> sh;
        uint32_t row = j;
        if (A.base_by_pos) {
            if (A.perm_src) {
                row = A.perm_src[j];
                if (!dk) A.perm_dst[j] = row;
            } else {
                row = A.perms[j];
            }
        }
        NodeIn in;
        if (FOLD) {   // the verdict from the LDS table: other workgroups are still storing node_feas
            in.r = A.soa.rec[row];
            in.coll_tg = tg.coll_tg[row];
            in.dev_free = tg.dev_free ? tg.dev_free[row] : 0u;
            in.feas = fold_ok(row, in.r.cls) ? 1u : 0u;
        } else {
            load_node(A.soa, tg, row, in);
        }
        NodeEval ev;
        ev.score = 0.0;
        eval_loaded<false, false>(A.soa, tg, class_ok, A.ask, dk, A.penalty_bits, A.log10, nullptr, row, in, &ev);
        (dk ? A.base1 : A.base)[j] = encode_eval(ev);
    }
}

// ---- windowed count loop: phase-static selection ------------------------------
//
// Windowed binpack (limit = ceil(log2 n) < n; no affinity or spread) of one
// evaluation. The value of visit position T (FinalScore, or filtered /
// exhausted) depends only on the row there and on how many of this
// evaluation's placements that row holds. A visit list without repeated rows
// shows a row again only n positions later, and every Select's winner lies
// behind the next Select's start, so once the cursor is at c the values of all
// positions [c, c + n) (one rotation) are fixed: no Select that stops inside
// that window can change them. A *phase* therefore:
//   1. evaluates the n positions in parallel: base[row] (shared, k_base) or the
//      row re-evaluated with its placement count from the LDS overlay;
//   2. scans option / non-positive-option (N) counts into option indices and
//      nb[k] = N options before option k;
//   3. resolves the Select boundaries serially but in O(1) per Select: a Select
//      starting at option i returns every positive option and every N after its
//      third, so it stops at option i + L - 1 + m for the smallest m in {0,1,2}
//      with exactly m N's in [i, i + L - 1 + m], else at i + L + 2
//      (LimitIterator, select.go:35-74);
//   4. finds every Select's winner at once (first strict maximum over its
//      returned options: LDS atomicMax on an order-preserving key, then
//      atomicMin on the option index) and commits the winners to the overlay
//      (distinct rows within a phase, so the inserts are independent).
// The next phase starts after the last stop. A Select that cannot stop inside
// the window ends the phase early; if it is the phase's first one it has seen
// the whole list: the stream is exhausted, set-aside options are appended
// (at most `limit` in total) and the cursor stays (feasible.go:90-107).
// One record of a deferred-record k_chain launch: the full Select result of
// the entry, evaluated on the state the launch started from (the entry's dk =
// placements of the launch on the row before it).
__device__ __forceinline__ void build_emit_rec(const BatchArgs& A, const ChainEmit& m, EmitRec& o) {
    o.row = m.row;
    o.nodes_evaluated = m.consumed;
    o.nodes_filtered = m.filtered;
    o.nodes_exhausted = m.exhausted;
    o.new_offset = m.new_offset;
    o.final_score = 0.0;
    o.n_scores = 0;
    o.n_device_offers = 0;
    o.flags = 0;
    for (int q = 0; q < PE_MAX_SCORES; q++) o.scores[q] = 0.0;
    for (int q = 0; q < PE_MAX_DEVICE_REQ; q++) o.device_offer_group[q] = 0;
    if (m.row < 0) return;
    const uint32_t row = (uint32_t)m.row;
    if (A.fused_parts && m.dk == 0 && m.pos != PE_NONE && A.ask.n_dev == 0) {
        // the row's first-phase evaluation (its state at the launch's start)
        const uint32_t np = A.fused_nparts[m.pos];
        o.final_score = m.score;
        o.n_scores = np;
        for (int q = 0; q < PE_MAX_SCORES; q++)
            if (q < (int)np) o.scores[q] = A.fused_parts[(size_t)m.pos * PE_MAX_SCORES + q];
        return;
    }
    NodeIn in;
    load_node(A.soa, A.tg, row, in);
    NodeEval ev;
    ev.score = 0.0;
    eval_loaded<true, false>(A.soa, A.tg, A.tg.class_ok, A.ask, m.dk, A.penalty_bits, A.log10, nullptr, row, in, &ev);
    o.final_score = ev.score;
    o.n_scores = ev.nscores;
    for (int q = 0; q < PE_MAX_SCORES; q++) if (q < (int)ev.nscores) o.scores[q] = ev.parts[q];
    if (A.ask.n_dev > 0) {
        const DevClass& dc = A.tg.dev_cls[A.soa.rec[row].cls];
        uint32_t fr = dev_after(A.ask, dc, A.tg.dev_free[row], m.dk);
        double mm;
        uint32_t groups[kMaxDevReq];
        if (dev_assign(A.ask, dc, fr, &mm, groups)) {
            o.n_device_offers = (uint32_t)A.ask.n_dev;
            for (int q = 0; q < kMaxDevReq; q++)
                if (q < A.ask.n_dev) o.device_offer_group[q] = (uint16_t)groups[q];
        }
    }
}

constexpr int kChainBlock = 1024;
constexpr int kChainItems = 16;                               // positions per lane of the largest shape
constexpr uint32_t kChainMaxN = kChainBlock * kChainItems;   // positions per phase held in registers (largest shape)
constexpr int kChainMaxSel = 1024;                            // Selects resolved per phase
constexpr uint32_t kChainMaxRedo = 2048;                      // rows re-evaluated per phase (<= placements per launch)

enum : int { kPhaseMore = 0, kPhaseCount = 1, kPhaseExhausted = 2, kPhaseStall = 3, kPhaseRetry = 4 };
constexpr uint32_t kChainStalled = 0x80000000u;   // eval_status cursor flag: continue with the lazy loop
constexpr int kSegE = 21;                 // entry offsets into a segment: a Select spans <= limit + 3 options
constexpr uint32_t kSegLen = 256;         // options per segment of the boundary walk
constexpr uint32_t kMaxChainLimit = kSegE - 3;
constexpr uint16_t kNxFail = 0xFFFF;      // the Select starting at this option cannot stop in the window
constexpr uint32_t kExFail = 0xFF;
// k_chain error flags (eval_status cursor word, beside kChainStalled): an
// index the shape's arrays do not cover. The kernel stops the evaluation
// instead of storing out of bounds and the host fails the call.
constexpr uint32_t kChainError = 0x40000000u;

// Per-instantiation shape of k_chain: ITEMS visit positions per lane, so one
// phase covers kMaxN = 1024 * ITEMS positions. Every array and loop bound below
// derives from it, including the wave-0 tile scan (kScanPer tiles per lane,
// at least one: a shape with fewer than 64 tiles still scans all of them).
template <int ITEMS>
struct ChainShape {
    static constexpr int kItems = ITEMS;
    static constexpr uint32_t kMaxN = (uint32_t)kChainBlock * ITEMS;
    static constexpr int kTiles = (int)(kMaxN / 64);
    static constexpr int kSegs = (int)((kMaxN + kSegLen - 1) / kSegLen);
    static constexpr int kScanPer = (kTiles + 63) / 64;
    static_assert(kScanPer * 64 >= kTiles, "the tile scan covers every tile");
    static_assert(kMaxN <= kChainMaxN, "the host sizes scratch for the largest shape");
    static_assert(kMaxN % 32 == 0, "position bitmaps");
};

template <int ITEMS>
struct ChainShared {
    using Shp = ChainShape<ITEMS>;
    uint32_t tile_o[Shp::kTiles], tile_n[Shp::kTiles];    // per 64-position tile counts, then exclusive offsets
    uint32_t sel_b[kChainMaxSel];                          // option index of each Select's stop
    uint32_t sel_end[kChainMaxSel];                        // its visit position (relative to the phase start)
    unsigned long long sel_max[kChainMaxSel];              // order-preserving key of the max returned score,
                                                           // then the winner's FinalScore bits
    uint32_t sel_arg[kChainMaxSel];                        // option index of the first maximum
    uint32_t sel_row[kChainMaxSel];                        // the winner's row
    uint32_t sel_f[kChainMaxSel], sel_x[kChainMaxSel];     // filtered / exhausted positions (metrics)
    uint32_t seg_tab[Shp::kSegs][kSegE];                  // per segment and entry offset: count | exit << 16
    uint16_t seg_entry[Shp::kSegs], seg_base[Shp::kSegs];
    uint2 redo[kChainMaxRedo];                             // (row, placements) to re-evaluate; then the value
    uint16_t sel_pos[kChainMaxSel];                        // the winner's visit position (relative)
    // visit positions (mod n) whose row holds >= 1 / >= 2 placements of this
    // launch: later phases find their values without probing the overlay
    uint32_t bm1[Shp::kMaxN / 32], bm2[Shp::kMaxN / 32];
    double aside_v[kMaxSkip];
    uint32_t aside_row[kMaxSkip];
    uint32_t tot_o, tot_n, nsel, mode, n_redo, n_seg, slow, n_emit, n_ov;
    uint32_t err;                                          // a bounds guard tripped (kChainError)
};

__device__ __forceinline__ unsigned long long order_key(double x) {
    const unsigned long long b = (unsigned long long)gm::f2u(x);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}

__device__ __forceinline__ uint32_t wrap_pos(uint32_t x, uint32_t n) {
    if (x < n) return x;
    x -= n;
    return x < n ? x : x % n;
}

// Plan.AppendAlloc into the overlay from many threads at once; the rows are
// distinct, so no two threads race on one key.
__device__ __forceinline__ uint32_t ov_add_atomic(const Overlay& o, uint32_t row) {
    uint32_t h = ov_hash(o, row);
    if (!o.k) {
        const uint32_t fresh = (row << o.kshift) | 1u;
        for (;;) {
            uint32_t e = o.keys[h];
            if (e == kEmpty) {
                e = atomicCAS(&o.keys[h], kEmpty, fresh);
                if (e == kEmpty) return h;
            }
            if ((e >> o.kshift) == row) { atomicAdd(&o.keys[h], 1u); return h; }
            h = (h + 1) & o.mask;
        }
    }
    for (;;) {
        uint32_t key = o.keys[h];
        if (key == kEmpty) {
            key = atomicCAS(&o.keys[h], kEmpty, row);
            if (key == kEmpty) { atomicAdd(&o.k[h], 1u); return h; }
        }
        if (key == row) { atomicAdd(&o.k[h], 1u); return h; }
        h = (h + 1) & o.mask;
    }
}

// first index s in [0, cnt) with a[s] >= x (a ascending; cnt if none)
__device__ __forceinline__ uint32_t lower_bound_lds(const uint32_t* a, uint32_t cnt, uint32_t x) {
    uint32_t lo = 0, hi = cnt;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (a[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Register state per position q of a thread: option index (14 bits) and, until
// the Select ids are known, the N-option prefix (14 bits); afterwards the
// Select id (10 bits) in the high half.
constexpr uint32_t kIdxBits = 14, kIdxMask = (1u << kIdxBits) - 1u;

// Optional step profile (PE_CHAIN_PROF): thread 0 accumulates shader clocks
// per step into A.prof[phase * 8 + step] (phases 0..3, the last one
// accumulating the rest); marks follow the block barriers. Step 0 of phase 0
// includes the kernel's start and the overlay initialisation.
#define PE_PROF_MARK(k)                                                   \
    do {                                                                  \
        if (A.prof && tid == 0) {                                         \
            const uint64_t now_ = __builtin_readcyclecounter();           \
            A.prof[prof_ph * 8 + (k)] += now_ - prof_t;                   \
            prof_t = now_;                                                \
        }                                                                 \
    } while (0)


// The chain's rare heavy paths out of line: inlined, the table and ask fields
// they read were hoisted to the kernel's start and held (spilled) for its
// whole run.
__device__ __noinline__ void chain_emit_full(const BatchArgs& A, Overlay ov, uint32_t e, uint32_t it, int win_row,
                                             double score, uint32_t consumed, uint32_t f, uint32_t x, uint32_t next_off) {
    emit_placement<false>(A, A.tg.class_ok, ov, nullptr, e, it, win_row, score, consumed, f, x, next_off);
}

// The FUSED first phase's evaluation of visit position p: its value, and its
// score parts into A.fused_parts (the records of winners without an earlier
// placement of the launch copy them)
__device__ __noinline__ double chain_eval_parts(const BatchArgs& A, uint32_t row, uint32_t p) {
    NodeIn in;
    load_node(A.soa, A.tg, row, in);
    NodeEval ev;
    ev.score = 0.0;
    eval_loaded<true, false>(A.soa, A.tg, A.tg.class_ok, A.ask, 0u, A.penalty_bits, A.log10, nullptr, row, in, &ev);
    if (ev.status == kOption) {
        A.fused_nparts[p] = (uint8_t)ev.nscores;
        for (int q = 0; q < PE_MAX_SCORES; q++) A.fused_parts[(size_t)p * PE_MAX_SCORES + q] = ev.parts[q];
    }
    return encode_eval(ev);
}

// value of (row, placements) re-evaluated: the k_base pipeline with dk placements
__device__ __noinline__ double chain_reeval(const BatchArgs& A, uint32_t row, uint32_t dk) {
    NodeIn in;
    load_node(A.soa, A.tg, row, in);
    NodeEval ev;
    ev.score = 0.0;
    eval_loaded<false, false>(A.soa, A.tg, A.tg.class_ok, A.ask, dk, A.penalty_bits, A.log10, nullptr, row, in, &ev);
    return encode_eval(ev);
}

// Step 5 of k_chain (out of line: its loads would otherwise raise the whole
// kernel's register pressure).
template <class Sh>
__device__ __noinline__ void chain_walk(Sh& sh, const uint16_t* nb, const double* vs, const uint32_t* perm,
                                        uint32_t cur, uint32_t n, uint32_t nsel, int tid) {
    for (uint32_t s = (uint32_t)tid; s < nsel; s += kChainBlock) {
        const uint32_t p0 = s ? (uint32_t)nb[sh.sel_b[s - 1]] + 1u : 0u;
        const uint32_t p1 = nb[sh.sel_b[s]];
        uint32_t n_aside = 0, f = 0, x = 0;
        int bp = -1;
        double best = 0.0;
        for (uint32_t pb = p0; pb <= p1; pb += 8u) {
            double y[8];
#pragma unroll
            for (int k = 0; k < 8; k++) y[k] = vs[min(pb + (uint32_t)k, p1)];   // one round of loads
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (pb + (uint32_t)k > p1) break;
                const double yk = y[k];
                if (yk == -__builtin_inf()) { f++; continue; }
                if (yk == __builtin_inf()) { x++; continue; }
                if (yk <= 0.0 && n_aside < (uint32_t)kMaxSkip) { n_aside++; continue; }
                if (bp < 0 || yk > best) { best = yk; bp = (int)(pb + (uint32_t)k); }
            }
        }
        if (bp < 0) {   // every Select returns at least one option past its set-aside ones
            sh.err = 1u;
            bp = (int)p1;
        }
        sh.sel_end[s] = p1;
        sh.sel_pos[s] = (uint16_t)bp;
        sh.sel_max[s] = (unsigned long long)gm::f2u(best);
        sh.sel_row[s] = perm[wrap_pos(cur + (uint32_t)bp, n)];
        sh.sel_f[s] = f;
        sh.sel_x[s] = x;
    }
}

// Row patches (pe_update_nodes): payload = rows[n] then n rows of `words`
// 4-byte words each, read from the mapped staging; dst row r gets its row.
__global__ void __launch_bounds__(256) k_scatter_rows(uint32_t* dst, uint32_t words, const uint32_t* payload,
                                                      uint32_t n) {
    const uint64_t total = (uint64_t)n * words;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += stride) {
        const uint32_t i = (uint32_t)(t / words), w = (uint32_t)(t % words);
        dst[(uint64_t)payload[i] * words + w] = payload[n + t];
    }
}

// Per-node count arrays from a sorted sparse list (key = row << 5 | array,
// value = count): each thread owns one row, zeroes it in every array and
// writes the row's entries found by binary search. A deferred ResetPlan (R.rec)
// rides along: its arrays are disjoint from the counts.
// `first` / `stride`: this thread's first index and the launch's thread count.
__device__ __forceinline__ void counts_apply(const CountDsts& D, uint32_t nd, uint32_t n, const uint2* ents,
                                             uint32_t m, const ResetArgs& R, uint32_t first, uint32_t stride) {
    if (R.rec) {
        for (uint32_t i = first; i < R.n; i += stride) {
            R.rec[i] = R.base_rec[i];
            R.dev_free[i] = R.dev_free_base[i];
        }
        for (uint32_t i = first; i < R.m; i += stride) R.preempted[i] = 0;
        for (uint32_t i = first; i < R.keys; i += stride) R.pcount[i] = 0;
    }
    for (uint32_t row = first; row < n; row += stride) {
        uint32_t lo = 0, hi = m;
        const uint32_t k0 = row << 5;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ents[mid].x < k0) lo = mid + 1;
            else hi = mid;
        }
        for (uint32_t d = 0; d < nd; d++) {
            if (!D.d[d]) continue;
            uint32_t v = 0;
            if (lo < m && ents[lo].x == (k0 | d)) v = ents[lo++].y;
            D.d[d][row] = v;
        }
    }
}

// FUSED (short lists of one evaluation, BatchArgs::fused): no k_base, k_emit
// or k_emit_writeback launch; the kernel carries the fold (FoldArgs), evaluates
// its first phase's positions itself (storing them as the base table of the
// later phases, whose rows with placements are re-evaluated: no base1), builds
// the records into the mapped output, writes the placements back and raises
// done_flag[0].
constexpr uint32_t kFusedMaxClasses = 4096;
template <int ITEMS, bool FUSED>
__global__ void __launch_bounds__(kChainBlock) k_chain(BatchArgs A, uint32_t n_evals) {
    using Shp = ChainShape<ITEMS>;
    static_assert(Shp::kMaxN <= (1u << kIdxBits), "option index packing");
    static_assert(kChainMaxSel <= (1 << (32 - 2 * kIdxBits + kIdxBits)), "select id packing");
    __shared__ ChainShared<ITEMS> sh;
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn_smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t n = A.n_visit;
    // positions per phase: one rotation, or its first Shp::kMaxN positions on a
    // longer list (every Select of the phase still stops inside the window)
    const uint32_t Wfull = n < Shp::kMaxN ? n : Shp::kMaxN;
    const uint32_t L = A.limit;
    const uint32_t H = 1u << A.hash_bits;
    // A in the kernel-argument segment, for the out-of-line helpers (taking the
    // parameter's address would copy the whole struct to scratch)
    const BatchArgs& Ak = *(const BatchArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    Overlay ov;
    ov.bits = A.hash_bits;
    ov.mask = H - 1;
    ov.keys = reinterpret_cast<uint32_t*>(dyn_smem);
    ov.k = A.packed_overlay ? nullptr : ov.keys + H;
    ov.kshift = A.packed_overlay;
    ov.kmask = A.packed_overlay ? (1u << A.packed_overlay) - 1u : 0u;
    uint16_t* nb = reinterpret_cast<uint16_t*>(ov.keys + (A.packed_overlay ? H : 2 * H));   // [n + 2]
    uint16_t* nx = nb + ((Wfull + 2 + 1) & ~1u);   // [W + 2]: next Select start per option, then Select id per option

    uint64_t prof_t = A.prof ? __builtin_readcyclecounter() : 0;
    int prof_ph = 0;   // profile slot group: phase (capped at 3)
    if (FUSED && A.counts.nd) {
        // SetJob's collision counts (and the deferred ResetPlan copy) carried
        // by this launch instead of a k_counts launch of their own
        const CountArgs& C = A.counts;
        counts_apply(C.D, C.nd, C.n, C.ents, C.m, C.R, (uint32_t)tid, kChainBlock);
        __syncthreads();
    }
    if (FUSED && A.fold.feas) {
        // the FeasibilityWrapper fold of every row, before any evaluation
        __shared__ uint8_t fcls[FUSED ? kFusedMaxClasses : 1];
        const FoldArgs& F = A.fold;
        for (uint32_t c = tid; c < F.ncls; c += kChainBlock) {
            const uint8_t v = F.class_src[c];
            fcls[c] = v;
            F.class_dst[c] = v;
        }
        __syncthreads();
        for (uint32_t row = tid; row < A.soa.n; row += kChainBlock) {
            const uint32_t c = A.soa.rec[row].cls;
            bool ok = c < F.ncls && fcls[c] != 0;
            if (F.node_ok) ok = ok && F.node_ok[row] != 0;
            F.feas[row] = ok ? 1 : 0;
        }
        __syncthreads();
    }
    for (uint32_t e = blockIdx.x; e < n_evals; e += gridDim.x) {
        const uint32_t* __restrict__ perm = A.perms + (size_t)e * A.perm_stride;
        double* __restrict__ vs = A.chain_vs + (size_t)blockIdx.x * kChainMaxN;   // values by relative position
        for (uint32_t i = tid; i < H; i += kChainBlock) {
            ov.keys[i] = kEmpty;
            if (ov.k) ov.k[i] = 0;
        }
        for (uint32_t i = tid; i < Shp::kMaxN / 32; i += kChainBlock) {
            sh.bm1[i] = 0;
            sh.bm2[i] = 0;
        }
        if (tid == 0) {
            sh.slow = n > Shp::kMaxN ? 1u : 0u;   // the position bitmaps cover one window of the list
            sh.n_emit = 0;
            sh.err = 0;
        }
        uint32_t cur = wrap_pos(A.offsets ? A.offsets[e] : A.offset0, n);
        uint32_t placed = 0;
        bool stalled = false;
        bool done = n == 0 || A.count == 0;
        uint32_t pos_used = 0;      // visit positions the resolved Selects consumed so far
        bool force_full = false;    // a shortened window held no whole Select: use the full one
        if (n == 0 && A.count && tid == 0 && A.out) {
            pe_placement& o = A.out[(size_t)e * A.count];
            o.row = -1; o.nodes_evaluated = 0; o.final_score = 0.0;
        }
        __syncthreads();
        while (!done) {
            PE_PROF_MARK(0);
            // positions of this phase: the full window, or after the first
            // phase what the remaining Selects need at the observed positions
            // per Select with a margin (the per-position steps scale with it)
            uint32_t W = Wfull;
            if (placed && !force_full) {
                const uint64_t need = (uint64_t)(A.count - placed) * pos_used * 3u / (2u * placed) + 1024u;
                if (need < W) W = (uint32_t)((need + kChainBlock - 1) / kChainBlock * kChainBlock);
                if (W > Wfull) W = Wfull;
            }
            force_full = false;
            // items a lane holds this phase (wave-uniform): the rest lie past the window
            const int qn = (int)((W + kChainBlock - 1) / kChainBlock);
            // 1. values of the window [cur, cur + n): base (no placement of this
            //    launch on the row), base1 (one), or queued for re-evaluation
            if (tid == 0) sh.n_redo = 0;
            // rows holding placements of this launch: one (base1) from the
            // position bitmaps, two or more re-evaluated (ov_count)
            const bool use_bm = placed && sh.slow == 0;
            uint32_t optmask = 0, nmask = 0, redo_mask = 0;   // bit q: option / non-positive option / re-evaluate
            {
                // rows are read only where the value needs them: every position
                // without the bitmaps (overlay probes) or for a row-indexed base,
                // else none (the first phase reads base, later ones base / base1
                // by position and re-evaluate the bitmaps' rows from the list)
                const bool rows_all = !A.base_by_pos || (placed && !use_bm);
                uint32_t row[ITEMS];
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                    row[q] = rows_all && j < W ? perm[wrap_pos(cur + j, n)] : 0u;
                }
                uint32_t one_mask = 0;
                if (placed) {
#pragma unroll
                    for (int q = 0; q < ITEMS; q++) {
                        if (q >= qn) break;
                        const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                        if (j < W) {
                            uint32_t b1 = 1, b2 = 1;
                            if (use_bm) {
                                const uint32_t p = wrap_pos(cur + j, n), bit = 1u << (p & 31);
                                b1 = sh.bm1[p >> 5] & bit;
                                b2 = sh.bm2[p >> 5] & bit;
                                if (b1 && (b2 || !A.base1)) redo_mask |= 1u << q;
                                else if (b1) one_mask |= 1u << q;
                            } else {
                                const uint32_t dk = ov_count(ov, row[q]);
                                if (dk == 1u && A.base1) one_mask |= 1u << q;
                                else if (dk) redo_mask |= 1u << q;
                            }
                        }
                    }
                }
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                    if (j < W && !((redo_mask >> q) & 1u)) {
                        double v;
                        if (FUSED && !placed) {
                            // the first phase evaluates its positions (and
                            // stores the visit order when it came staged)
                            const uint32_t p = wrap_pos(cur + j, n);
                            uint32_t r;
                            if (A.perm_src) {
                                r = A.perm_src[p];
                                A.perm_dst[p] = r;
                            } else {
                                r = perm[p];
                            }
                            v = A.fused_parts ? chain_eval_parts(Ak, r, p) : chain_reeval(Ak, r, 0u);
                            A.base[p] = v;
                        } else {
                            const double* src = ((one_mask >> q) & 1u) ? A.base1 : A.base;
                            v = src[A.base_by_pos ? wrap_pos(cur + j, n) : row[q]];
                        }
                        vs[j] = v;   // read back by the Select walks of step 5 (after the barriers)
                        const bool is_o = v > -__builtin_inf() && v < __builtin_inf();
                        optmask |= (uint32_t)is_o << q;
                        nmask |= (uint32_t)(is_o && v <= 0.0) << q;
                    }
                }
            }
            if (__syncthreads_or(redo_mask != 0)) {
                // rows with placements of this launch the tables do not cover:
                // evaluated in parallel, the value stored at its window position
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    if ((redo_mask >> q) & 1u) {
                        const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                        const uint32_t r = perm[wrap_pos(cur + j, n)];
                        const uint32_t slot = atomicAdd(&sh.n_redo, 1u);
                        if (slot < kChainMaxRedo) sh.redo[slot] = make_uint2(r, ov_count(ov, r) | (j << 18));
                        else sh.err = 1u;
                    }
                }
                __syncthreads();
                const uint32_t nr = min(sh.n_redo, kChainMaxRedo);
                for (uint32_t w = tid; w < nr; w += kChainBlock) {
                    const uint2 rd = sh.redo[w];
                    vs[rd.y >> 18] = chain_reeval(Ak, rd.x, rd.y & 0x3FFFFu);
                }
                __syncthreads();
                if (sh.err) break;
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    if ((redo_mask >> q) & 1u) {
                        const double v = vs[q * kChainBlock + tid];
                        const bool is_o = v > -__builtin_inf() && v < __builtin_inf();
                        optmask |= (uint32_t)is_o << q;
                        nmask |= (uint32_t)(is_o && v <= 0.0) << q;
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < ITEMS; q++) {
                if (q >= qn) break;
                const uint64_t bo = __ballot((optmask >> q) & 1u), bn = __ballot((nmask >> q) & 1u);
                if (lane == 0 && q * kChainBlock < (int)W) {
                    sh.tile_o[q * (kChainBlock / 64) + wave] = (uint32_t)__popcll(bo);
                    sh.tile_n[q * (kChainBlock / 64) + wave] = (uint32_t)__popcll(bn);
                }
            }
            for (uint32_t s = tid; s < kChainMaxSel; s += kChainBlock) {
                sh.sel_max[s] = 0ull;
                sh.sel_arg[s] = kEmpty;
                sh.sel_f[s] = 0;
                sh.sel_x[s] = 0;
            }
            __syncthreads();
            PE_PROF_MARK(1);
            // 2. exclusive scan of the tile counts (wave 0)
            const uint32_t ntiles = (W + 63) / 64;
            if (wave == 0) {
                constexpr int PER = Shp::kScanPer;
                uint32_t so = 0, sn = 0, lo[PER], ln[PER];
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const uint32_t t = (uint32_t)(lane * PER + k);
                    lo[k] = t < ntiles ? sh.tile_o[t] : 0u;
                    ln[k] = t < ntiles ? sh.tile_n[t] : 0u;
                    so += lo[k];
                    sn += ln[k];
                }
                uint32_t io = so, in_ = sn;   // inclusive wave scan
#pragma unroll
                for (int off = 1; off < 64; off <<= 1) {
                    const uint32_t xo = (uint32_t)__shfl_up((int)io, off), xn = (uint32_t)__shfl_up((int)in_, off);
                    if (lane >= off) { io += xo; in_ += xn; }
                }
                uint32_t eo = io - so, en = in_ - sn;
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const uint32_t t = (uint32_t)(lane * PER + k);
                    if (t < ntiles) { sh.tile_o[t] = eo; sh.tile_n[t] = en; }
                    eo += lo[k];
                    en += ln[k];
                }
                if (lane == 63) { sh.tot_o = io; sh.tot_n = in_; }
            }
            __syncthreads();
            PE_PROF_MARK(2);
            // 3. option index and N prefix of every option; nb[k] = N options before option k
            uint32_t pk[ITEMS];
#pragma unroll
            for (int q = 0; q < ITEMS; q++) {
                if (q >= qn) break;
                const uint64_t bo = __ballot((optmask >> q) & 1u), bn = __ballot((nmask >> q) & 1u);
                const uint32_t t = (uint32_t)(q * (kChainBlock / 64) + wave);
                const bool live = (uint32_t)(q * kChainBlock) < W;
                const uint32_t k = (live ? sh.tile_o[t] : 0u) + lanes_below(bo, lane);
                const uint32_t nbk = (live ? sh.tile_n[t] : 0u) + lanes_below(bn, lane);
                pk[q] = (k & kIdxMask) | ((nbk & kIdxMask) << kIdxBits);
                if ((optmask >> q) & 1u) {
                    if (k < W) nb[k] = (uint16_t)nbk;
                    else sh.err = 1u;   // an option index past the window: the scan is wrong
                }
            }
            const uint32_t tot_o = sh.tot_o, tot_n = sh.tot_n;
            if (tid == 0) {
                if (tot_o <= W) nb[tot_o] = (uint16_t)tot_n;
                else sh.err = 1u;
            }
            __syncthreads();
            if (sh.err) break;   // stop the evaluation before any index built on the scan is used
            PE_PROF_MARK(3);
            // 4. Select boundaries. A Select starting at option i stops at option
            //    i + L - 1 + m for the smallest m in {0, 1, 2} with exactly m N's
            //    in [i, i + L - 1 + m], else at i + L + 2 (its third N is set aside
            //    and every later option returned). 4a: the next start nx[i] of every
            //    option in parallel; 4b: per 64-option segment and entry offset the
            //    Selects inside and the exit offset; 4c: one lane walks the
            //    segments; 4d: the Selects are written out in parallel.
            if (tot_n == 0) {
                // no non-positive option in the window: every Select returns
                // exactly L options (m = 0 above), so Select s stops at option
                // (s + 1) L - 1; nb takes the options' positions at once
#pragma unroll
                for (int q = 0; q < ITEMS; q++)
                    if (q < qn && ((optmask >> q) & 1u)) nb[pk[q] & kIdxMask] = (uint16_t)(q * kChainBlock + tid);
                if (tid == 0) {
                    const uint32_t want = min(A.count - placed, (uint32_t)kChainMaxSel);
                    const uint32_t fit = tot_o / L;
                    uint32_t ns = fit < want ? fit : want;
                    int fmode = kPhaseMore;
                    if (ns == 0 && W < Wfull) fmode = kPhaseRetry;
                    else if (ns == 0 && W < n) fmode = kPhaseStall;
                    else if (ns == 0) { fmode = kPhaseExhausted; ns = tot_o ? 1u : 0u; if (ns) sh.sel_b[0] = tot_o - 1; }
                    else if (ns == A.count - placed) fmode = kPhaseCount;
                    sh.nsel = ns;
                    sh.mode = (uint32_t)fmode;
                    sh.n_seg = 0;
                }
                __syncthreads();
                if (sh.mode == (uint32_t)kPhaseMore || sh.mode == (uint32_t)kPhaseCount)
                    for (uint32_t sel = tid; sel < sh.nsel; sel += kChainBlock) sh.sel_b[sel] = (sel + 1) * L - 1;
                __syncthreads();
            } else {
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    if ((optmask >> q) & 1u) {
                        const uint32_t i = pk[q] & kIdxMask;
                        const uint32_t a0 = pk[q] >> kIdxBits;
                        uint32_t nxt = kNxFail;
                        if (i + L - 1 < tot_o) {
                            if (nb[min(i + L, tot_o)] - a0 == 0) nxt = i + L;
                            else if (i + L < tot_o) {
                                if (nb[i + L + 1] - a0 == 1) nxt = i + L + 1;
                                else if (i + L + 1 < tot_o) {
                                    if (nb[i + L + 2] - a0 == 2) nxt = i + L + 2;
                                    else if (i + L + 2 < tot_o) nxt = i + L + 3;
                                }
                            }
                        }
                        nx[i] = (uint16_t)nxt;
                    }
                }
                if (tid == 0) nx[tot_o] = kNxFail;
                __syncthreads();
                // nb is free from here on: the relative position of every option
#pragma unroll
                for (int q = 0; q < ITEMS; q++)
                    if (q < qn && ((optmask >> q) & 1u)) nb[pk[q] & kIdxMask] = (uint16_t)(q * kChainBlock + tid);
                const uint32_t n_seg = (tot_o + kSegLen - 1) / kSegLen;
                const uint32_t E = L + 3;
                for (uint32_t t = tid; t < n_seg * E; t += kChainBlock) {
                    const uint32_t g = t / E, o = t - g * E;
                    const uint32_t end = kSegLen * (g + 1);
                    uint32_t i = kSegLen * g + o, cnt = 0, ex = kExFail;
                    for (;;) {
                        if (i >= end) { ex = i - end; break; }
                        if (i >= tot_o) break;
                        const uint32_t x = nx[i];
                        if (x == kNxFail) break;
                        cnt++;
                        i = x;
                    }
                    sh.seg_tab[g][o] = cnt | (ex << 16);
                }
                __syncthreads();
                if (tid == 0) {
                    const uint32_t want = min(A.count - placed, (uint32_t)kChainMaxSel);
                    uint32_t total = 0, o = 0, used = 0;
                    for (uint32_t g = 0; g < n_seg; g++) {
                        const uint32_t te = sh.seg_tab[g][o], cnt = te & 0xFFFFu, ex = te >> 16;
                        sh.seg_entry[g] = (uint16_t)o;
                        sh.seg_base[g] = (uint16_t)total;
                        used = g + 1;
                        if (total + cnt >= want) { total = want; break; }
                        total += cnt;
                        if (ex == kExFail) break;
                        o = ex;
                    }
                    int mode = kPhaseMore;
                    uint32_t ns = total;
                    if (ns == 0 && W < Wfull) {
                        // the shortened window held no whole Select: again with the full one
                        mode = kPhaseRetry;
                        used = 0;
                    } else if (ns == 0 && W < n) {
                        // a Select needs more than the window: the lazy loop goes on from here
                        mode = kPhaseStall;
                        used = 0;
                    } else if (ns == 0) {
                        // the first Select saw the whole list without reaching the limit
                        mode = kPhaseExhausted;
                        ns = tot_o ? 1u : 0u;
                        if (ns) sh.sel_b[0] = tot_o - 1;
                        used = 0;
                    } else if (ns == A.count - placed) {
                        mode = kPhaseCount;
                    }
                    sh.nsel = ns;
                    sh.mode = (uint32_t)mode;
                    sh.n_seg = used;
                }
                __syncthreads();
                {
                    const uint32_t ns = sh.nsel, used = sh.n_seg;
                    for (uint32_t g = tid; g < used; g += kChainBlock) {
                        uint32_t i = kSegLen * g + sh.seg_entry[g], sel = sh.seg_base[g];
                        while (sel < ns && i < kSegLen * (g + 1)) {
                            const uint32_t x = nx[i];
                            sh.sel_b[sel++] = x - 1u;
                            i = x;
                        }
                    }
                }
                __syncthreads();
            }
            const uint32_t nsel = sh.nsel;
            const int mode = (int)sh.mode;
            if (mode == kPhaseStall) {
                stalled = true;
                break;
            }
            if (mode == kPhaseRetry) {
                force_full = true;
                continue;
            }
            PE_PROF_MARK(4);
            if (mode != kPhaseExhausted) {
                // 5. one thread per Select walks its positions (previous stop + 1
                //    .. its stop) in the scratch copy of the values: the first
                //    kMaxSkip non-positive options are set aside, MaxScoreIterator
                //    keeps the first strict maximum of the rest (select.go:79-116);
                //    filtered / exhausted positions are the Select's metrics
                chain_walk(sh, nb, vs, perm, cur, n, nsel, tid);
            } else {
                // the one Select of an exhausted stream: every option of the
                // window (atomics over one key), its first kMaxSkip N's set aside
                uint32_t retmask = 0;
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    if ((optmask >> q) & 1u) {
                        const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                        const double vq = vs[j];
                        const uint32_t nrank = pk[q] >> kIdxBits;   // N options before this one
                        const bool aside = ((nmask >> q) & 1u) && nrank < (uint32_t)kMaxSkip;
                        if (!aside) {
                            retmask |= 1u << q;
                            atomicMax(&sh.sel_max[0], order_key(vq));
                        } else {
                            sh.aside_v[nrank] = vq;
                            sh.aside_row[nrank] = perm[wrap_pos(cur + j, n)];
                        }
                    }
                }
                __syncthreads();
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                    if (((retmask >> q) & 1u) &&
                        order_key(vs[j]) == sh.sel_max[0])
                        atomicMin(&sh.sel_arg[0], pk[q] & kIdxMask);
                }
                if (A.full_out || A.emit) {
#pragma unroll
                    for (int q = 0; q < ITEMS; q++) {
                        if (q >= qn) break;
                        const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                        if (j < W && !((optmask >> q) & 1u))
                            atomicAdd(vs[j] == -__builtin_inf()
                                          ? &sh.sel_f[0] : &sh.sel_x[0], 1u);
                    }
                }
                __syncthreads();
#pragma unroll
                for (int q = 0; q < ITEMS; q++) {
                    if (q >= qn) break;
                    const uint32_t j = (uint32_t)(q * kChainBlock + tid);
                    if (((retmask >> q) & 1u) && sh.sel_arg[0] == (pk[q] & kIdxMask)) {
                        sh.sel_row[0] = perm[wrap_pos(cur + j, n)];
                        sh.sel_max[0] = (unsigned long long)gm::f2u(vs[j]);
                    }
                }
            }
            __syncthreads();
            if (sh.err) break;
            PE_PROF_MARK(5);
            // 6. emit the winners and commit them (Plan.AppendAlloc), one Select per thread
            if (mode != kPhaseExhausted) {
                for (uint32_t s = tid; s < nsel; s += kChainBlock) {
                    const uint32_t start = s ? sh.sel_end[s - 1] + 1u : 0u;
                    const uint32_t consumed = sh.sel_end[s] - start + 1u;
                    const int win_row = (int)sh.sel_row[s];
                    const double score = gm::u2f(sh.sel_max[s]);
                    const uint32_t it = placed + s;
                    const uint32_t next_off = wrap_pos(cur + sh.sel_end[s] + 1u, n);
                    if (it >= A.count) {   // nsel <= count - placed by construction
                        sh.err = 1u;
                        continue;
                    }
                    if (A.emit) {
                        ChainEmit& m = A.emit[it];
                        m.row = win_row;
                        m.pos = wrap_pos(cur + sh.sel_pos[s], n);
                        m.dk = ov_count(ov, (uint32_t)win_row);
                        m.consumed = consumed;
                        m.filtered = sh.sel_f[s];
                        m.exhausted = sh.sel_x[s];
                        m.new_offset = next_off;
                        m.score = score;
                    } else if (A.full_out) {
                        chain_emit_full(Ak, ov, e, it, win_row, score, consumed, sh.sel_f[s], sh.sel_x[s], next_off);
                    }
                    if (A.out) {
                        pe_placement& o = A.out[(size_t)e * A.count + it];
                        o.row = win_row;
                        o.nodes_evaluated = consumed;
                        o.final_score = score;
                    }
                }
                __syncthreads();   // the records read the overlay before the commits
                if (A.commit) {
                    for (uint32_t s = tid; s < nsel; s += kChainBlock) {
                        ov_add_atomic(ov, sh.sel_row[s]);
                        if (n <= Shp::kMaxN) {   // the bitmaps cover lists of one window only
                            const uint32_t p = wrap_pos(cur + sh.sel_pos[s], n), bit = 1u << (p & 31);
                            if (atomicOr(&sh.bm1[p >> 5], bit) & bit) atomicOr(&sh.bm2[p >> 5], bit);
                        }
                    }
                }
                if (tid == 0) sh.n_emit = placed + nsel;
                placed += nsel;
                pos_used += sh.sel_end[nsel - 1] + 1u;
                cur = wrap_pos(cur + sh.sel_end[nsel - 1] + 1u, n);
                done = mode == kPhaseCount;
            } else {
                // exhausted stream: returned options in order, then set-aside ones
                // until the limit (select.go:35-74); the cursor stays
                if (tid == 0) {
                    const uint32_t a = min(tot_n, (uint32_t)kMaxSkip);
                    const uint32_t r = tot_o - a;
                    double best = -__builtin_inf();
                    int win_row = -1;
                    if (nsel && r) { best = gm::u2f(sh.sel_max[0]); win_row = (int)sh.sel_row[0]; }
                    const uint32_t take = min(a, L > r ? L - r : 0u);
                    for (uint32_t k = 0; k < take; k++)
                        if (sh.aside_v[k] > best) { best = sh.aside_v[k]; win_row = (int)sh.aside_row[k]; }
                    if (A.emit) {
                        ChainEmit& m = A.emit[placed];
                        m.row = win_row;
                        m.pos = PE_NONE;
                        m.dk = win_row >= 0 ? ov_count(ov, (uint32_t)win_row) : 0u;
                        m.consumed = n;
                        m.filtered = sh.sel_f[0];
                        m.exhausted = sh.sel_x[0];
                        m.new_offset = cur;
                        m.score = best;
                    } else if (A.full_out) {
                        chain_emit_full(Ak, ov, e, placed, win_row, best, n, sh.sel_f[0], sh.sel_x[0], cur);
                    }
                    sh.n_emit = placed + 1;
                    sh.slow = 1;   // the winner's position is not tracked: later phases probe the overlay
                    if (A.out) {
                        pe_placement& o = A.out[(size_t)e * A.count + placed];
                        o.row = win_row;
                        o.nodes_evaluated = n;
                        o.final_score = win_row >= 0 ? best : 0.0;
                    }
                    if (win_row >= 0 && A.commit) ov_add(ov, (uint32_t)win_row);
                    sh.mode = win_row >= 0 ? 1u : 0u;
                }
                __syncthreads();
                if (sh.mode) placed++;
                else done = true;   // nil option: failedTGAllocs short-circuit
                if (placed >= A.count) done = true;
            }
            __syncthreads();
            PE_PROF_MARK(6);
            prof_ph = prof_ph < 3 ? prof_ph + 1 : 3;
        }
        __syncthreads();
        if (tid == 0) {
            A.eval_status[2 * e] = placed;
            A.eval_status[2 * e + 1] = cur | (stalled ? kChainStalled : 0u) | (sh.err ? kChainError : 0u);
        }
        if (FUSED) {
            // the records, on the state the launch started from, then the
            // placements into HBM, then the completion word
            __syncthreads();
            const uint32_t ne = min(sh.n_emit, A.count);
            for (uint32_t i = tid; i < ne; i += kChainBlock) build_emit_rec(Ak, A.emit[i], A.emit_out[i]);
            __syncthreads();
            if (A.writeback) writeback_overlay<kChainBlock, false, false>(A, ov, H, nullptr);
            __syncthreads();
            if (tid == 0 && A.done_flag) {
                __threadfence_system();
                __hip_atomic_store(A.done_flag, A.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else if (A.emit) {
            // records and the HBM writeback are k_emit's: dump the overlay
            if (tid == 0) sh.n_ov = 0;
            __syncthreads();
            for (uint32_t h = tid; h < H; h += kChainBlock) {
                const uint32_t key = ov.keys[h];
                if (key == kEmpty) continue;
                const uint32_t r = ov.k ? key : key >> ov.kshift;
                const uint32_t kk = ov.k ? ov.k[h] : key & ov.kmask;
                const uint32_t slot = atomicAdd(&sh.n_ov, 1u);
                if (slot < A.count) A.emit_ov[slot] = make_uint2(r, kk);   // overlay rows <= placements
                else sh.err = 1u;
            }
            __syncthreads();
            if (tid == 0) {
                A.emit_n[0] = min(sh.n_emit, A.count);
                A.emit_n[1] = A.writeback ? min(sh.n_ov, A.count) : 0u;
                if (sh.err) A.eval_status[2 * e + 1] |= kChainError;
            }
        } else if (A.writeback) {
            writeback_overlay<kChainBlock, false, false>(A, ov, H, nullptr);   // no cores on the chain path
        }
        __syncthreads();
    }
}

constexpr uint32_t kEmitBlock = 64;

// Records of a single-evaluation k_chain launch (A.emit): the full Select
// result of every entry, evaluated on the state the launch started from (the
// entry's dk = placements on the row before it); k_emit_writeback then
// writes the launch's placements back to the HBM SoA.
__global__ void __launch_bounds__(kEmitBlock) k_emit(BatchArgs A) {
    // records are built in LDS and stored to the (host-mapped) output as one
    // contiguous run per workgroup: 8-byte coalesced stores of compact records
    // instead of every lane writing its own record field by field over the
    // bus; small workgroups spread the bus writes over more CUs
    __shared__ EmitRec recs[kEmitBlock];
    const uint32_t i = blockIdx.x * kEmitBlock + threadIdx.x;
    const uint32_t n_emit = min(A.emit_n[0], A.count);
    if (i < n_emit) build_emit_rec(A, A.emit[i], recs[threadIdx.x]);
    __syncthreads();
    {
        const uint32_t first = blockIdx.x * kEmitBlock;
        const uint32_t cnt = n_emit > first ? min(kEmitBlock, n_emit - first) : 0u;
        constexpr uint32_t W = sizeof(EmitRec) / 8;
        const uint2* src = reinterpret_cast<const uint2*>(recs);
        uint2* dst = reinterpret_cast<uint2*>(A.emit_out + first);
        for (uint32_t w = threadIdx.x; w < cnt * W; w += kEmitBlock) dst[w] = src[w];
    }
    if (!A.done_flag) return;
    __syncthreads();
    // every workgroup raises its own completion word once its records are out:
    // the spinning host checks them all (no ticket atomic round trip and one
    // system fence per workgroup instead of two)
    if (threadIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(A.done_flag + blockIdx.x, A.done_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The launch's placements written back to the HBM SoA, one overlay entry
// (row, placements) per thread; runs after k_emit on the stream (the records
// read the state the launch started from), off the host's critical path.
__global__ void __launch_bounds__(256) k_emit_writeback(BatchArgs A) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x;
    if (x >= A.emit_n[1]) return;
    const uint2 e = A.emit_ov[x];
    NodeRec& r = A.soa.rec[e.x];
    r.used_cpu += (int64_t)e.y * ask_cpu(A.soa, A.ask, e.x);
    core_take(A.soa, A.ask, e.x, e.y);
    r.used_mem += (int64_t)e.y * A.ask.mem;
    r.used_disk += (int64_t)e.y * A.ask.disk;
    r.used_mbits += (int32_t)e.y * A.ask.commit_mbits;
    r.used_dyn += (int32_t)e.y * A.ask.commit_dyn;
    A.soa.coll_job[e.x] += e.y;
    A.tg.coll_tg[e.x] += e.y;
    if (A.ask.n_dev > 0) A.tg.dev_free[e.x] = dev_after(A.ask, A.tg.dev_cls[r.cls], A.tg.dev_free[e.x], e.y);
}

// The placed count of a 256-lane workgroup, one atomic per workgroup into one
// of kPlacedSlots counters (the host sums them): same-address atomics from
// every wave serialise at one L2 channel (32k of them at 6.4M rows cost more
// than the evaluation).
__device__ __forceinline__ void add_placed(uint32_t local, uint32_t* slots) {
    __shared__ uint32_t red[4];
    for (int off = 32; off > 0; off >>= 1) local += __shfl_xor(local, off);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = local;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t x = red[0] + red[1] + red[2] + red[3];
        if (x) atomicAdd(&slots[blockIdx.x % kPlacedSlots], x);
    }
}

// SystemStack: every list entry is an independent single-node Select.
__global__ void __launch_bounds__(256) k_system(SystemArgs A) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t local = 0;
    Overlay none;
    none.keys = nullptr;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < A.n_list; i += stride) {
        const uint32_t row = A.list[i];
        NodeEval ev;
        eval_node<false>(A.soa, A.tg, A.tg.class_ok, A.ask, none, nullptr, A.log10, nullptr, row, &ev);
        if (ev.status == kOption) {
            A.out_score[i] = ev.score;
            A.out_status[i] = 0;
            local++;
            if (!A.commit) continue;
            // Plan.AppendAlloc: rows are unique in the list, so no races
            NodeRec& r = A.soa.rec[row];
            r.used_cpu += ask_cpu(A.soa, A.ask, row);
            core_take(A.soa, A.ask, row, 1);
            r.used_mem += A.ask.mem;
            r.used_disk += A.ask.disk;
            r.used_mbits += A.ask.commit_mbits;
            r.used_dyn += A.ask.commit_dyn;
            A.soa.coll_job[row] += 1;
            A.tg.coll_tg[row] += 1;
            if (A.ask.n_dev > 0) A.tg.dev_free[row] = dev_after(A.ask, A.tg.dev_cls[r.cls], A.tg.dev_free[row], 1);
        } else {
            A.out_score[i] = __builtin_nan("");
            A.out_status[i] = (uint8_t)ev.status;
        }
    }
    if (A.placed) add_placed(local, A.placed);
}

// k_system in row order, phase one: every row of the list evaluated (and
// committed) with coalesced accesses; the outcome lands in res[row].
__device__ __forceinline__ uint64_t sys_box(int status, double score) {
    if (status == kOption) return (uint64_t)__double_as_longlong(score);
    return 0x7FF8000000000000ull | (uint64_t)status;   // a quiet NaN carrying the outcome
}

__global__ void __launch_bounds__(256) k_system_rows(SystemArgs A) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t local = 0;
    Overlay none;
    none.keys = nullptr;
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < A.n_rows; row += stride) {
        const uint32_t pos = A.rank_of[row];
        if (pos == 0xFFFFFFFFu) continue;
        NodeEval ev;
        eval_node<false>(A.soa, A.tg, A.tg.class_ok, A.ask, none, nullptr, A.log10, nullptr, row, &ev);
        if (A.n_list) {   // the outcome at the row's list position (scattered stores, nothing waits on them)
            A.out_score[pos] = ev.status == kOption ? ev.score : __builtin_nan("");
            A.out_status[pos] = (uint8_t)ev.status;
        } else {
            A.res[row] = sys_box(ev.status, ev.score);
        }
        if (ev.status != kOption) continue;
        local++;
        if (!A.commit) continue;
        NodeRec& r = A.soa.rec[row];
        r.used_cpu += ask_cpu(A.soa, A.ask, row);
        core_take(A.soa, A.ask, row, 1);
        r.used_mem += A.ask.mem;
        r.used_disk += A.ask.disk;
        r.used_mbits += A.ask.commit_mbits;
        r.used_dyn += A.ask.commit_dyn;
        A.soa.coll_job[row] += 1;
        A.tg.coll_tg[row] += 1;
        if (A.ask.n_dev > 0) A.tg.dev_free[row] = dev_after(A.ask, A.tg.dev_cls[r.cls], A.tg.dev_free[row], 1);
    }
    if (A.placed) add_placed(local, A.placed);
}

// Phase two of the row-order pass: the outcomes back in list order. Reads the
// list coalesced and res[list[pos]] (8 B per row, L2 / MALL resident), writes
// FinalScore and the outcome coalesced; random 8-byte stores into the outputs
// would cost a 64-byte line write each.
__global__ void __launch_bounds__(256) k_system_gather(const uint32_t* list, uint32_t n_list, const uint64_t* res,
                                                      double* out_score, uint8_t* out_status) {
    const uint32_t pos = blockIdx.x * 256 + threadIdx.x;
    if (pos >= n_list) return;
    const uint64_t v = res[list[pos]];
    const bool boxed = (v & 0xFFFFFFFFFFFFFFF0ull) == 0x7FF8000000000000ull;
    out_score[pos] = boxed ? __builtin_nan("") : __longlong_as_double((long long)v);
    out_status[pos] = boxed ? (uint8_t)(v & 15u) : (uint8_t)kOption;
}

// rank_of[row] = position of row in the list (rows absent: PE_NONE, set by the caller's memset)
__global__ void __launch_bounds__(256) k_rank_of(const uint32_t* list, uint32_t n_list, uint32_t* rank_of) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n_list) rank_of[list[i]] = i;
}

// Outcome census of one Select pass over the visit list on the HBM state
// (no overlay): counts[0] options, [1] filtered, [2] exhausted. With no option
// the Select is nil after pulling every node, which the count loop's
// preemption retry uses instead of a windowed scan of the whole list.
// kParts: also the score parts of each option (k_ploop's plain winner records).
template <bool kParts>
__global__ void __launch_bounds__(256) k_census(BatchArgs A, uint32_t* counts, uint8_t* status, double* score,
                                                double* parts, uint8_t* nparts) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t c[3] = {0, 0, 0};
    Overlay none;
    none.keys = nullptr;
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < A.n_visit; j += stride) {
        NodeEval ev;
        eval_node<kParts>(A.soa, A.tg, A.tg.class_ok, A.ask, none, A.penalty_bits, A.log10, nullptr, A.perms[j], &ev);
        c[ev.status]++;
        if (status) {   // per-position outcomes for a parallel Select (k_evict_resolve)
            status[j] = (uint8_t)ev.status;
            score[j] = ev.status == kOption ? ev.score : 0.0;
        }
        if (kParts && ev.status == kOption) {
            nparts[j] = (uint8_t)ev.nscores;
            for (int k = 0; k < PE_MAX_SCORES; k++) parts[(size_t)j * PE_MAX_SCORES + k] = ev.parts[k];
        }
    }
    // one atomic per workgroup and counter (not per wave): fewer same-address
    // atomics queueing at one L2 channel
    __shared__ uint32_t red[3][4];
    for (int k = 0; k < 3; k++) {
        uint32_t x = c[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
        if ((threadIdx.x & 63) == 0) red[k][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const uint32_t x = red[threadIdx.x][0] + red[threadIdx.x][1] + red[threadIdx.x][2] + red[threadIdx.x][3];
        if (x) atomicAdd(&counts[threadIdx.x], x);
    }
}

// Host-driven Plan.AppendAlloc on the HBM SoA (pe_commit). `offers`: the
// device offers of the Select that chose the node (one byte per request), or
// ~0u to assign them on the current state.
template <bool kCores = true>
__device__ __forceinline__ void commit_row(const NodeSoA& s, const TgTables& t, const Ask& a, uint32_t row,
                                           uint32_t offers) {
    // Every load before the first store: the counters share types with the
    // record's fields, so a load placed after a store is issued only once the
    // store's own load has returned, one HBM round trip per field.
    NodeRec& r = s.rec[row];
    const int64_t cpu = r.used_cpu, mem = r.used_mem, disk = r.used_disk;
    const int32_t mbits = r.used_mbits, dyn = r.used_dyn;
    const uint32_t c = r.cls, cj = s.coll_job[row], ct = t.coll_tg[row];
    const uint32_t fr0 = a.n_dev > 0 ? t.dev_free[row] : 0u;
    const int64_t ac = kCores ? ask_cpu(s, a, row) : a.cpu;
    uint32_t fr = fr0;
    if (a.n_dev > 0) {
        if (offers == 0xFFFFFFFFu) {
            fr = dev_after(a, t.dev_cls[c], fr0, 1);
        } else {
            for (int q = 0; q < kMaxDevReq && q < a.n_dev; q++) {
                const uint32_t g = (offers >> (8 * q)) & 255u, f = (fr >> (8 * g)) & 255u;
                const uint32_t cnt = (uint32_t)a.dev_cnt[q];
                fr -= (cnt < f ? cnt : f) << (8 * g);
            }
        }
    }
    r.used_cpu = cpu + ac;
    r.used_mem = mem + a.mem;
    r.used_disk = disk + a.disk;
    r.used_mbits = mbits + a.commit_mbits;
    r.used_dyn = dyn + a.commit_dyn;
    s.coll_job[row] = cj + 1u;
    t.coll_tg[row] = ct + 1u;
    if (a.n_dev > 0) t.dev_free[row] = fr;
    if (kCores) core_take(s, a, row, 1);
    for (int p = 0; p < t.n_psets; p++) {
        const uint32_t v = pset_value(t, p, row, c);
        if (v != kMissing) t.pset_counts[p][v] += 1;
    }
}

__global__ void k_commit(NodeSoA s, TgTables t, Ask a, uint32_t row, uint32_t offers) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    commit_row(s, t, a, row, offers);
}

// Plan.AppendAlloc of distinct rows chosen on the host (SystemScheduler
// placements resolved against distinct_property counts): commit_row per
// thread, the shared property-set counts by atomics.
__global__ void __launch_bounds__(256) k_commit_rows(NodeSoA s, TgTables t, Ask a, const uint32_t* rows, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = rows[i];
    NodeRec& r = s.rec[row];
    r.used_cpu += ask_cpu(s, a, row);
    core_take(s, a, row, 1);
    r.used_mem += a.mem;
    r.used_disk += a.disk;
    r.used_mbits += a.commit_mbits;
    r.used_dyn += a.commit_dyn;
    s.coll_job[row] += 1;
    t.coll_tg[row] += 1;
    if (a.n_dev > 0) t.dev_free[row] = dev_after(a, t.dev_cls[r.cls], t.dev_free[row], 1);
    for (int p = 0; p < t.n_psets; p++) {
        const uint32_t v = pset_value(t, p, row, r.cls);
        if (v != kMissing) atomicAdd(&t.pset_counts[p][v], 1u);
    }
}

// Replay (sign +1) of a speculative loop's confirmed placements after a
// rollback to its checkpoint, or removal (sign -1) of its unconfirmed ones
// (pe_commit / pe_select, engine.cpp): one thread per placement, every update
// an integer atomic add, so repeated rows sum exactly as the sequential
// commit_row calls would. Each offer was assigned on the state that already
// held every earlier placement, so no free count underflows and the packed u8
// subtractions never borrow. Removal is only used without device asks.
__global__ void __launch_bounds__(256) k_apply_commits(NodeSoA s, TgTables t, Ask a, const uint32_t* rows,
                                                      const uint32_t* offers, uint32_t n, int sign) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t row = rows[i];
    NodeRec& r = s.rec[row];
    const unsigned long long s64 = (unsigned long long)(long long)sign;
    const unsigned int s32 = (unsigned int)sign;
    atomicAdd(reinterpret_cast<unsigned long long*>(&r.used_cpu), (unsigned long long)a.cpu * s64);
    atomicAdd(reinterpret_cast<unsigned long long*>(&r.used_mem), (unsigned long long)a.mem * s64);
    atomicAdd(reinterpret_cast<unsigned long long*>(&r.used_disk), (unsigned long long)a.disk * s64);
    atomicAdd(reinterpret_cast<unsigned int*>(&r.used_mbits), (unsigned int)a.commit_mbits * s32);
    atomicAdd(reinterpret_cast<unsigned int*>(&r.used_dyn), (unsigned int)a.commit_dyn * s32);
    atomicAdd(&s.coll_job[row], s32);
    atomicAdd(&t.coll_tg[row], s32);
    const uint32_t c = r.cls;
    if (a.n_dev > 0 && sign > 0) {
        const uint32_t o = offers[i];
        uint32_t sub = 0;
        for (int q = 0; q < kMaxDevReq && q < a.n_dev; q++) sub += (uint32_t)a.dev_cnt[q] << (8 * ((o >> (8 * q)) & 255u));
        atomicSub(&t.dev_free[row], sub);
    }
    for (int p = 0; p < t.n_psets; p++) {
        const uint32_t v = pset_value(t, p, row, c);
        if (v != kMissing) atomicAdd(&t.pset_counts[p][v], s32);
    }
}

// One pass of the scoring sweep over rows [row_begin, row_end), one tile of
// BLOCK rows per workgroup iteration (grid-stride), 64 rows per wave. Every
// lane streams its row (64-byte record, collision count, verdict, visit rank),
// runs the feasibility half and resolves the score-table lookups of an option.
// Options go to a wave-private LDS ring (kQueue entries); whenever it holds 64
// the wave runs the fp64 scoring half (two software Pow) on a full wave, so
// the scoring is dense and no workgroup barrier sits in the loop. PF: the next
// tile's loads are issued before the current tile is evaluated, so HBM
// streaming overlaps the scoring. Per-lane SweepRec records, reduced per
// workgroup at the end. Rows outside the visit list are dropped.
//
// AUX: the node's verdict, affinity index and spread values come folded in one
// u32 per node (k_fold_aux) and resolve against LDS copies of the affinity
// values and the spread boosts, so an option costs no dependent table load.
// The grid's last workgroup to finish merges every workgroup's record into
// *A.merged (a shard's one record: the all-gather then moves 80 bytes per
// rank). Each workgroup's record store is released by its arrival count; the
// last one acquires them all (the records cross XCDs: agent scope).
template <int BLOCK>
__device__ __forceinline__ void sweep_last_merge(const SweepArgs& A, SweepRec* red) {
    __shared__ uint32_t last;
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(A.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (!last) return;   // workgroup-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    SweepRec r;
    rec_init(r);
    for (uint32_t i = threadIdx.x; i < gridDim.x; i += BLOCK) rec_merge(r, A.recs[i]);
    rec_block_reduce<BLOCK>(r, red);
    if (threadIdx.x == 0) {
        *A.merged = r;
        __hip_atomic_store(A.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int BLOCK, bool PF, int PROBE = 0, bool AUX = false, bool MERGE = false>
__device__ __forceinline__ void sweep_block(const SweepArgs& A) {
    constexpr int W = BLOCK / 64;
    constexpr uint32_t kQueue = 128;
    __shared__ SweepRec red[W];
    __shared__ ScoreIn q[W][kQueue];
    __shared__ uint32_t q_rank[W][kQueue];
    __shared__ double aff_lds[AUX ? kAuxValues : 1];
    __shared__ double sp_lds[AUX ? kAuxPsets : 1][AUX ? kAuxValues : 1];
    SweepRec r;
    rec_init(r);
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    if (AUX) {
        for (int i = tid; i < kAuxValues; i += BLOCK) aff_lds[i] = A.aff_vals[i];
        for (int p = 0; p < A.tg.n_psets; p++)
            for (int i = tid; i < kAuxValues; i += BLOCK)
                sp_lds[p][i] = i < A.tg.pset_nvals[p] ? A.spread_tab[A.tg.pset_tab_off[p] + i] : 0.0;
        __syncthreads();
    }
    const uint32_t n = A.n_visit;
    const uint32_t stride = gridDim.x * BLOCK;
    ScoreIn* wq = q[wid];
    uint32_t* wr = q_rank[wid];
    uint32_t head = 0, qn = 0;   // wave-uniform ring state
    auto score_from = [&](uint32_t at) {
        const uint32_t i = (at + (uint32_t)lane) & (kQueue - 1);
        NodeEval ev;
        if (PROBE == 2) ev.score = wq[i].aff + wq[i].spread;
        else score_option<false>(A.ask, A.log10, wq[i], &ev);
        rec_add(r, wr[i], ev.score);
    };
    NodeIn nx;
    uint32_t npos = kEmpty, naux = 0;
    auto fetch = [&](uint32_t t) {
        const uint32_t row = t + (uint32_t)tid;
        npos = kEmpty;
        if (row < A.row_end && row >= t) {
            npos = A.rank_of[row];
            if (AUX) {
                nx.r = A.soa.rec[row];
                nx.coll_tg = A.tg.coll_tg[row];
                nx.dev_free = A.tg.dev_free ? A.tg.dev_free[row] : 0u;
                naux = A.node_aux[row];
                nx.feas = naux >> 31;
            } else {
                load_node(A.soa, A.tg, row, nx);
            }
        }
    };
    uint32_t tile = A.row_begin + blockIdx.x * BLOCK;
    if (PF) fetch(tile);
    for (; tile < A.row_end; tile += stride) {
        NodeIn in;
        uint32_t pos, aux;
        if (PF) {
            in = nx;
            pos = npos;
            aux = naux;
            const uint32_t nt = tile + stride;
            if (nt > tile && nt < A.row_end) fetch(nt);
        } else {
            fetch(tile);
            in = nx;
            pos = npos;
            aux = naux;
        }
        const uint32_t row = tile + (uint32_t)tid;
        bool opt = false;
        uint32_t rank = 0;
        ScoreIn si;
        if (pos != kEmpty) {
            const int st = status_loaded(A.soa, A.tg, A.tg.class_ok, A.ask, 0u, row, in, &si);
            if (st == kFiltered) r.filtered++;
            else if (st == kExhausted) r.exhausted++;
            else {
                opt = true;
                rank = pos >= A.offset ? pos - A.offset : pos + n - A.offset;
                if (PROBE == 1) {
                    si.aff = si.spread = 0.0;
                    si.penalty = 0;
                } else if (AUX) {
                    si.penalty = A.penalty_bits ? (A.penalty_bits[row >> 5] >> (row & 31)) & 1u : 0u;
                    si.aff = aff_lds[aux & 255u];
                    double total = 0.0;
                    for (int p = 0; p < A.tg.n_psets; p++) {
                        const uint32_t v = (aux >> (8 + 8 * p)) & 255u;
                        total += (v == kAuxMissing) ? -1.0 : sp_lds[p][v];
                    }
                    si.spread = total;
                } else {
                    lookup_scores(A.tg, A.penalty_bits, A.spread_tab, row, in.r.cls, &si);
                }
            }
        }
        const uint64_t m = __ballot(opt);
        if (opt) {
            const uint32_t i = (head + qn + lanes_below(m, lane)) & (kQueue - 1);
            wq[i] = si;
            wr[i] = rank;
        }
        qn += (uint32_t)__popcll(m);
        if (qn >= 64) {   // LDS ops of one wave complete in order: the ring is visible
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
            __builtin_amdgcn_wave_barrier();
            score_from(head);
            head = (head + 64) & (kQueue - 1);
            qn -= 64;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if ((uint32_t)lane < qn) score_from(head);
    rec_block_reduce<BLOCK>(r, red);
    if (threadIdx.x == 0) A.recs[blockIdx.x] = r;
    if (MERGE) sweep_last_merge<BLOCK>(A, red);
}

template <int BLOCK, bool PF, int PROBE = 0, bool AUX = false, bool MERGE = false>
__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(AUX ? 4 : 5))) k_sweep(SweepArgs A) {
    sweep_block<BLOCK, PF, PROBE, AUX, MERGE>(A);
}

// Bound probes for the sweep (PE_SWEEP_VARIANT 5 / 6): 5 streams exactly the
// sweep's bytes with trivial arithmetic; 6 runs the scoring arithmetic on
// register-synthesised inputs without touching memory.
template <int BLOCK, int MODE>
__global__ void __launch_bounds__(BLOCK) k_sweep_probe(SweepArgs A) {
    __shared__ SweepRec red[BLOCK / 64];
    SweepRec r;
    rec_init(r);
    const uint32_t stride = gridDim.x * BLOCK;
    uint64_t acc = 0;
    for (uint32_t row = A.row_begin + blockIdx.x * BLOCK + threadIdx.x; row < A.row_end; row += stride) {
        if (MODE == 5) {
            NodeIn in;
            load_node(A.soa, A.tg, row, in);
            acc += (uint64_t)in.r.cap_cpu + (uint64_t)in.r.used_mem + (uint64_t)in.r.cap_disk + in.r.cls + in.coll_tg +
                   in.feas + A.rank_of[row] + (uint64_t)in.r.used_cpu + (uint64_t)in.r.cap_mem +
                   (uint64_t)in.r.used_disk + (uint64_t)in.r.avail_mbits;
        } else {
            NodeIn in;
            in.r.cap_cpu = 4000 + (row & 1023);
            in.r.cap_mem = 8192 + (row & 2047);
            in.r.cap_disk = 100000;
            in.r.used_cpu = row & 511;
            in.r.used_mem = row & 255;
            in.r.used_disk = 0;
            in.r.cls = row & 7;
            in.r.avail_mbits = -1;
            in.r.used_mbits = 0;
            in.r.used_dyn = 0;
            in.coll_tg = 0;
            in.feas = (row & 3) == 0;
            TgTables t = A.tg;
            t.node_feas = &A.tg.class_ok[0];   // unused: in.feas drives the verdict
            NodeEval ev;
            ev.score = 0.0;
            eval_loaded<false>(A.soa, t, A.tg.class_ok, A.ask, 0u, nullptr, A.log10, A.spread_tab, row, in, &ev);
            if (ev.status == kOption) rec_add(r, row, ev.score);
        }
    }
    r.filtered += (uint32_t)acc;
    rec_block_reduce<BLOCK>(r, red);
    if (threadIdx.x == 0) A.recs[blockIdx.x] = r;
}

// Merge the per-workgroup records (one 512-thread workgroup: a few records per
// thread, so the dependent load chain stays short).
__global__ void __launch_bounds__(512) k_sweep_merge(const SweepRec* recs, uint32_t count, SweepRec* out) {
    __shared__ SweepRec red[8];
    SweepRec r;
    rec_init(r);
    for (uint32_t i = threadIdx.x; i < count; i += 512) rec_merge(r, recs[i]);
    rec_block_reduce<512>(r, red);
    if (threadIdx.x == 0) *out = r;
}

// Spread contribution table in HBM for the sweep path (same code as the
// persistent loop's LDS table, so both paths are bit-identical).
// The spread boost tables of every record of a speculative run (spec_metrics):
// record k's use counts are the run's starting counts (t.pset_counts, the
// checkpoint) plus the earlier records' placements (`delta`: n_rec x
// pset_cnt_total, host-built, completed here in place); one block per record,
// its table at tab + k * pset_tab_total. Spread sets only.
__global__ void __launch_bounds__(256) k_spread_tables(TgTables t, uint32_t* delta, double* tab) {
    __shared__ uint32_t scratch[4];
    const uint32_t k = blockIdx.x;
    uint32_t* cnt = delta + (size_t)k * t.pset_cnt_total;
    for (int p = 0; p < t.n_psets; p++)
        for (int v = threadIdx.x; v < t.pset_nvals[p]; v += 256) cnt[t.pset_cnt_off[p] + v] += t.pset_counts[p][v];
    __syncthreads();
    build_spread_table<256>(t, cnt, tab + (size_t)k * t.pset_tab_total, scratch);
}

__global__ void __launch_bounds__(256) k_spread_table(TgTables t, double* tab) {
    __shared__ uint32_t counts[kLdsPsetValues];
    __shared__ uint32_t scratch[4];
    const bool lds = t.pset_cnt_total <= (uint32_t)kLdsPsetValues;   // else the HBM counts
    if (lds)
        for (int p = 0; p < t.n_psets; p++)
            for (int v = threadIdx.x; v < t.pset_nvals[p]; v += 256) counts[t.pset_cnt_off[p] + v] = t.pset_counts[p][v];
    __syncthreads();
    build_spread_table<256>(t, lds ? counts : nullptr, tab, scratch);
}

// Score parts of the winner straight into its record (eval_node<true> with
// the parts in the record, not in a stack array, which would live in scratch).
__device__ __forceinline__ void record_winner(const SweepArgs& A, uint32_t row, pe_ranked_node* o) {
    NodeIn in;
    load_node(A.soa, A.tg, row, in);
    ScoreIn si;
    (void)status_loaded(A.soa, A.tg, A.tg.class_ok, A.ask, 0u, row, in, &si, A.spread_tab);
    lookup_scores(A.tg, A.penalty_bits, A.spread_tab, row, in.r.cls, &si);
    for (int k = 0; k < PE_MAX_SCORES; k++) o->scores[k] = 0.0;
    uint32_t ns;
    o->final_score = score_into<true>(A.ask, A.log10, si, o->scores, &ns);
    o->n_scores = ns;
}

// Score parts of one node (the winner's RankedNode record).
__global__ void k_node_record(SweepArgs A, uint32_t row, pe_ranked_node* out) {
    if (threadIdx.x != 0) return;
    record_winner(A, row, out);
    record_offers(A.soa, A.ask, A.tg, row, 0u, out);
}

// One placement of the device-resident full-pass count loop (pe_place on long
// lists), after this placement's k_sweep: thread 0 merges the per-block
// SweepRecs (k_sweep_merge), resolves the Select result (sweep_finish +
// k_node_record) and commits the winner (k_commit with the record's device
// offers); then the workgroup rebuilds the spread table for the next
// placement from the updated counts (k_spread_table). state[0]: a nil Select
// ended the loop (later steps do nothing); state[1]: placements so far.
__device__ __forceinline__ void step_block(const SweepArgs& A, uint32_t nrecs, const uint32_t* visit, uint32_t n,
                                           uint32_t offset, pe_ranked_node* out, uint32_t* state) {
    __shared__ uint32_t counts[kLdsPsetValues];
    __shared__ uint32_t scratch[4];
    __shared__ SweepRec red[4];
    __shared__ uint32_t go;
    if (state[0]) return;   // every thread reads the flag before thread 0 may set it
    SweepRec rec;
    rec_init(rec);
    for (uint32_t i = threadIdx.x; i < nrecs; i += 256) rec_merge(rec, A.recs[i]);
    rec_block_reduce<256>(rec, red);
    if (threadIdx.x == 0) {
        go = 0;
        {
            pe_ranked_node* o = out + state[1];
            pe_ranked_node z = {};
            *o = z;
            o->row = -1;
            o->nodes_evaluated = n;            // a full pass pulls every node
            o->nodes_filtered = rec.filtered;
            o->nodes_exhausted = rec.exhausted;
            o->new_offset = offset;            // and leaves the cursor where it is
            const uint32_t rank = rec_winner(rec);
            if (rank == kEmpty) {
                state[0] = 1;
            } else {
                uint32_t pos = offset + rank;
                if (pos >= n) pos -= n;
                const uint32_t row = visit[pos];
                o->row = (int32_t)row;
                record_winner(A, row, o);
                record_offers(A.soa, A.ask, A.tg, row, 0u, o);
                uint32_t offers = 0xFFFFFFFFu;
                if (o->n_device_offers) {
                    offers = 0;
                    for (uint32_t q = 0; q < o->n_device_offers && q < 4; q++)
                        offers |= (o->device_offer_group[q] & 255u) << (8 * q);
                }
                commit_row(A.soa, A.tg, A.ask, row, offers);
                state[1] += 1;
                go = A.spread_tab != nullptr;
            }
        }
    }
    __syncthreads();
    if (!go) return;   // workgroup-uniform
    const TgTables& t = A.tg;
    const bool lds = t.pset_cnt_total <= (uint32_t)kLdsPsetValues;   // else the HBM counts
    if (lds)
        for (int p = 0; p < t.n_psets; p++)
            for (int v = threadIdx.x; v < t.pset_nvals[p]; v += 256) counts[t.pset_cnt_off[p] + v] = t.pset_counts[p][v];
    __syncthreads();
    build_spread_table<256>(t, lds ? counts : nullptr, const_cast<double*>(A.spread_tab), scratch);
}

__global__ void __launch_bounds__(256) k_sweep_step(SweepArgs A, uint32_t nrecs, const uint32_t* visit, uint32_t n,
                                                    uint32_t offset, pe_ranked_node* out, uint32_t* state) {
    step_block(A, nrecs, visit, n, offset, out, state);
}

// The whole full-pass count loop in one workgroup, for lists whose options
// fit LDS. A commit changes only the committed node's own inputs (use,
// collisions, devices, distinct_hosts) and the spread boosts (one value per
// property value), and a node that is filtered or exhausted stays so while
// the loop only adds allocations. So the workgroup evaluates the list once
// and keeps one LDS entry per option: its visit position, status, the sum of
// its scores before the spread one (score_head: binpack, device affinity,
// anti-affinity, penalty, affinity, summed left to right) and its spread
// property values. A placement then reads 16 bytes of LDS per option, adds
// the spread boost and normalises exactly as score_option does. The maximum
// is found on approximate scores (sum x 1/k, within 2^-52 relative of
// sum / k): only the options within a 2^-48 margin of a wave's maximum take
// the exact quotient, and (max score, earliest rank) is reduced over those;
// a non-positive maximum takes the exact LimitIterator skip record instead
// (rec_add / rec_winner). Two lanes of wave 0 then
// load the winner once and evaluate it side by side: lane 0 as it stands
// (dk = 0: the placement's record, parts written straight into it), lane 1
// with the placement added (dk = 1: the option's new entry, as the overlay
// chain does); lane 0 commits to the SoA and, for target spreads, refreshes
// the one boost per property whose count moved (even spreads rebuild the
// table). One launch for the whole loop; results equal `count` x (k_sweep +
// k_sweep_step). More options than entries: state[5] = 1 before any commit
// and the host runs the multi-workgroup loop instead. The arguments come
// through a device buffer: the TgTables arrays are indexed by property at
// run time, which would copy a by-value argument to scratch.
}  // namespace pe
// ROCm device library wave reduction (DPP), also behind __reduce_max_sync
extern "C" __device__ __attribute__((const)) double __ockl_wfred_max_f64(double);
namespace pe {

constexpr int kFullThreads = 1024;
constexpr int kFullWaves = kFullThreads / 64;
constexpr int kFullPer = 9;                               // entries per thread
constexpr uint32_t kFullCap = kFullThreads * kFullPer;    // LDS entries (16 B each)

__device__ __forceinline__ double readlane_f64(double x, int l) {
    const unsigned long long u = __double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

template <int NP>   // spread properties scored (A.spread_tab ? n_psets : 0), at most kAuxPsets
__global__ void __launch_bounds__(kFullThreads) k_fullpass_lds(const SweepArgs* __restrict__ Ap, const uint32_t* visit,
                                                               uint32_t n, uint32_t count, pe_ranked_node* out,
                                                               uint32_t* state, unsigned long long* prof) {
    const SweepArgs& A = *Ap;
    extern __shared__ double ent_sum[];                                    // [kFullCap] score_head sums
    uint32_t* ent_meta = reinterpret_cast<uint32_t*>(ent_sum + kFullCap);   // status | k << 2 | spread values
    uint32_t* ent_pos = ent_meta + kFullCap;                                // visit position
    // the pset_tab_off / pset_cnt_off layout of at most kAuxPsets sets of < kAuxValues values
    __shared__ double tab[kAuxPsets * (kAuxValues + 1)];
    __shared__ double desired[kAuxPsets * kAuxValues];
    __shared__ uint32_t counts[kAuxPsets * kAuxValues];
    __shared__ double aff_lds[kAuxValues];
    __shared__ double red_s[kFullWaves];
    __shared__ uint32_t red_r[kFullWaves];
    __shared__ uint32_t red_f[kFullWaves], red_e[kFullWaves];
    __shared__ SweepRec red[kFullWaves];
    __shared__ uint32_t scratch[4];
    __shared__ uint32_t sh_nf, sh_ne, sh_stop, sh_win, sh_m;
    __shared__ double parts1[PE_MAX_SCORES];   // lane 1's parts (unused)
    __shared__ double rcp_k[8];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const TgTables& t = A.tg;
    constexpr int np = NP;
    const uint32_t off = A.offset;
    bool any_even = false;
    for (int p = 0; p < np; p++) any_even = any_even || t.pset_even[p];
    for (int i = tid; i < kAuxValues; i += kFullThreads) aff_lds[i] = A.aff_vals[i];
    if (tid < 8) rcp_k[tid] = tid ? 1.0 / (double)tid : 0.0;
    if (tid == 0) sh_m = 0;
    for (int p = 0; p < np; p++)
        for (int v = tid; v < t.pset_nvals[p]; v += kFullThreads) {
            counts[t.pset_cnt_off[p] + v] = t.pset_counts[p][v];
            desired[t.pset_cnt_off[p] + v] = t.pset_even[p] ? 0.0 : t.pset_desired[p][v];
        }
    __syncthreads();
    if (np) build_spread_table<kFullThreads>(t, counts, tab, scratch);
    auto spread_of = [&](uint32_t meta) __attribute__((always_inline)) -> double {   // lookup_scores' total
        double sp = 0.0;
#pragma unroll
        for (int p = 0; p < np; p++) {
            const uint32_t v = (meta >> (8 + 8 * p)) & 255u;
            sp += (v == kAuxMissing) ? -1.0 : tab[t.pset_tab_off[p] + v];
        }
        return sp;
    };
    auto load = [&](uint32_t row, NodeIn& in) __attribute__((always_inline)) -> uint32_t {   // the sweep's AUX fetch
        in.r = A.soa.rec[row];
        in.coll_tg = t.coll_tg[row];
        in.dev_free = t.dev_free ? t.dev_free[row] : 0u;
        const uint32_t aux = A.node_aux[row];
        in.feas = aux >> 31;
        return aux;
    };
    // status and score_head of a loaded node with dk placements of this loop
    // added; with a `parts` pointer the parts are written there
    auto head = [&](uint32_t row, const NodeIn& in, uint32_t aux, uint32_t dk, double* parts, double* sum,
                    uint32_t* kk) __attribute__((always_inline)) -> int {
        ScoreIn si;
        const int st = status_loaded(A.soa, t, t.class_ok, A.ask, dk, row, in, &si);
        *kk = 0;
        *sum = 0.0;
        if (st == kOption) {
            si.penalty = A.penalty_bits ? (A.penalty_bits[row >> 5] >> (row & 31)) & 1u : 0u;
            si.aff = aff_lds[aux & 255u];
            si.spread = 0.0;
            *sum = parts ? score_head<true>(A.ask, A.log10, si, parts, *kk)
                         : score_head<false>(A.ask, A.log10, si, nullptr, *kk);
        }
        return st;
    };
    // the final score of an entry (score_option's tail)
    auto final_sum = [&](uint32_t e, uint32_t* kk_out) __attribute__((always_inline)) -> double {
        const uint32_t meta = ent_meta[e];
        double sum = ent_sum[e];
        const double sp = spread_of(meta);
        uint32_t kk = (meta >> 2) & 7u;
        if (sp != 0.0) { sum += sp; kk++; }
        *kk_out = kk;
        return sum;
    };
    uint32_t nf = 0, ne = 0;
    for (uint32_t pos = tid; pos < n; pos += kFullThreads) {
        const uint32_t row = visit[pos];
        NodeIn in;
        const uint32_t aux = load(row, in);
        double s;
        uint32_t kk;
        const int st = head(row, in, aux, 0u, nullptr, &s, &kk);
        nf += st == kFiltered;
        ne += st == kExhausted;
        if (st == kOption) {
            const uint32_t e = atomicAdd(&sh_m, 1u);
            if (e < kFullCap) {
                ent_sum[e] = s;
                ent_meta[e] = (uint32_t)st | (kk << 2) | (aux & 0x00FFFF00u);
                ent_pos[e] = pos;
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        nf += (uint32_t)__shfl_xor((int)nf, o);
        ne += (uint32_t)__shfl_xor((int)ne, o);
    }
    if (lane == 0) { red_f[wid] = nf; red_e[wid] = ne; }
    __syncthreads();
    const uint32_t m = sh_m;
    if (m > kFullCap) {   // uniform: nothing committed yet, the host takes the other loop
        if (tid == 0) state[5] = 1;
        return;
    }
    if (tid == 0) {
        uint32_t a = 0, b = 0;
        for (int w = 0; w < kFullWaves; w++) { a += red_f[w]; b += red_e[w]; }
        sh_nf = a;
        sh_ne = b;
        sh_stop = 0;
    }
    __syncthreads();
    auto rank_of_pos = [&](uint32_t pos) __attribute__((always_inline)) -> uint32_t {
        return pos >= off ? pos - off : pos + n - off;
    };
    __shared__ unsigned long long sh_wprof[4];   // PE_FULL_PROF: the winner lane's load / score / record+commit
    if (prof && tid < 4) sh_wprof[tid] = 0;
    unsigned long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tl = prof ? wall_clock64() : 0;
    auto mark = [&](int i) __attribute__((always_inline)) {
        if (prof && tid == 0) {
            const unsigned long long x = wall_clock64();
            tp[i] += x - tl;
            tl = x;
        }
    };
    for (uint32_t it = 0; it < count; it++) {
        double ap[kFullPer];
        double amax = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < kFullPer; j++) {
            const uint32_t e = (uint32_t)tid + (uint32_t)j * kFullThreads;
            ap[j] = -__builtin_inff();
            if (e < m) {
                uint32_t kk;
                const double sum = final_sum(e, &kk);
                if ((ent_meta[e] & 3u) == (uint32_t)kOption) ap[j] = sum * rcp_k[kk];
            }
            amax = ap[j] > amax ? ap[j] : amax;
        }
        mark(4);
        amax = __ockl_wfred_max_f64(amax);
        mark(5);
        const double cut = amax - (__builtin_fabs(amax) * 0x1p-48 + 0x1p-1000);
        double best = -__builtin_inff();
        uint32_t best_rank = 0xFFFFFFFFu;
#pragma unroll
        for (int j = 0; j < kFullPer; j++) {
            const bool near = ap[j] >= cut && ap[j] != -__builtin_inff();   // options only
            if (__ballot(near)) {
                if (near) {
                    const uint32_t e = (uint32_t)tid + (uint32_t)j * kFullThreads;
                    uint32_t kk;
                    const double sc = final_sum(e, &kk) / (double)kk;
                    const uint32_t rk = rank_of_pos(ent_pos[e]);
                    if (sc > best || (sc == best && rk < best_rank)) { best = sc; best_rank = rk; }
                }
            }
        }
        mark(6);
        {   // the wave's (max, earliest rank) over its few candidate lanes
            uint64_t cand = __ballot(best_rank != 0xFFFFFFFFu);
            double wb = -__builtin_inff();
            uint32_t wr = 0xFFFFFFFFu;
            while (cand) {
                const int l = __builtin_ctzll(cand);
                cand &= cand - 1;
                const double b = readlane_f64(best, l);
                const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)best_rank, l);
                if (b > wb || (b == wb && r < wr)) { wb = b; wr = r; }
            }
            best = wb;
            best_rank = wr;
        }
        mark(7);
        if (lane == 0) { red_s[wid] = best; red_r[wid] = best_rank; }
        // Each wave's lanes 0-1 look their wave's candidate row up now (the
        // winner is one of the waves' candidates): the dependent visit load
        // overlaps the barrier and the resolve, and the winning wave loads its
        // candidate's node straight after. (Loading the whole node here keeps
        // ~20 more VGPRs live across the barrier: they spill.)
        const uint32_t my_rank = best_rank;   // wave-uniform
        uint32_t c_row = 0;
        if (lane < 2 && my_rank != 0xFFFFFFFFu) {
            uint32_t pos = off + my_rank;
            if (pos >= n) pos -= n;
            c_row = visit[pos];
        }
        __syncthreads();
        mark(0);
        // every wave resolves the block's winner itself (no second barrier):
        // the maximum score, then the earliest rank among the waves holding it
        best = lane < kFullWaves ? red_s[lane] : -__builtin_inff();
        best_rank = lane < kFullWaves ? red_r[lane] : 0xFFFFFFFFu;
        best = __ockl_wfred_max_f64(best);
        uint32_t win = __ockl_wfred_min_u32(lane < kFullWaves && red_s[lane] == best ? best_rank : 0xFFFFFFFFu);
        if (win != 0xFFFFFFFFu && !(best > 0.0)) {   // every option non-positive: the skip rule decides (rare)
            SweepRec r;
            rec_init(r);
            for (uint32_t e = tid; e < m; e += kFullThreads) {
                if ((ent_meta[e] & 3u) != (uint32_t)kOption) continue;
                uint32_t kk;
                const double sum = final_sum(e, &kk);
                rec_add(r, rank_of_pos(ent_pos[e]), sum / (double)kk);
            }
            rec_block_reduce<kFullThreads>(r, red);
            if (tid == 0) sh_win = rec_winner(r);
            __syncthreads();
            win = sh_win;
        }
        mark(1);
        pe_ranked_node* o = out + it;
        // the wave whose candidate won evaluates it; when the skip rule picked
        // a rank no wave held (every option non-positive), wave 0 loads it
        bool mine = win != 0xFFFFFFFFu && my_rank == win;
        if (win != 0xFFFFFFFFu && wid == 0 &&
            __ballot(lane < kFullWaves && red_r[lane] == win) == 0) {   // wave-uniform
            mine = true;
            if (lane < 2) {
                uint32_t pos = off + win;
                if (pos >= n) pos -= n;
                c_row = visit[pos];
            }
        }
        if (wid == 0 && win == 0xFFFFFFFFu) {
            if (lane == 0) {
                o->row = -1;
                o->nodes_evaluated = n;            // a full pass pulls every node
                o->nodes_filtered = sh_nf;
                o->nodes_exhausted = sh_ne;
                o->new_offset = off;
                state[0] = 1;
                sh_stop = 1;
            }
        } else if (mine && lane < 2) {
            const uint32_t row = c_row;
            const unsigned long long w0 = prof ? wall_clock64() : 0;
            NodeIn in;
            const uint32_t aux = load(row, in);
            if (prof) {   // the load's latency alone
                __builtin_amdgcn_s_waitcnt(0);
                if (lane == 0) sh_wprof[0] += wall_clock64() - w0;
            }
            const unsigned long long w1 = prof ? wall_clock64() : 0;
            double s;
            uint32_t kk;
            const int st = head(row, in, aux, (uint32_t)lane, lane == 0 ? o->scores : parts1, &s, &kk);
            if (prof && lane == 0) sh_wprof[1] += wall_clock64() - w1;
            const unsigned long long w2 = prof ? wall_clock64() : 0;
            const int st1 = __shfl(st, 1);
            const uint32_t meta0 = (aux & 0x00FFFF00u);   // spread values: the entry's
            if (lane == 1) {
                sh_win = (uint32_t)st | (kk << 2) | meta0;
                parts1[0] = s;
            } else {           // the placement's record, then the commit
                const double sp = spread_of(meta0);
                if (sp != 0.0) {   // SpreadIterator (spread.go:110-174)
                    s += sp;
                    o->scores[kk] = sp;
                    kk++;
                }
                o->row = (int32_t)row;
                o->final_score = s / (double)kk;   // ScoreNormalizationIterator (rank.go:762-767)
                o->n_scores = kk;
                o->nodes_evaluated = n;            // a full pass pulls every node
                o->nodes_filtered = sh_nf;
                o->nodes_exhausted = sh_ne;
                o->new_offset = off;               // and leaves the cursor where it is
                record_offers(A.soa, A.ask, t, row, 0u, o);
                uint32_t offers = 0xFFFFFFFFu;
                if (o->n_device_offers) {
                    offers = 0;
                    for (uint32_t q = 0; q < o->n_device_offers && q < 4; q++)
                        offers |= (o->device_offer_group[q] & 255u) << (8 * q);
                }
                const bool fast = A.ask.n_dev == 0 && A.ask.cores == 0 && np == t.n_psets;
                if (fast) {   // commit_row from the loaded values: stores only
                    NodeRec& r = A.soa.rec[row];
                    r.used_cpu = in.r.used_cpu + A.ask.cpu;
                    r.used_mem = in.r.used_mem + A.ask.mem;
                    r.used_disk = in.r.used_disk + A.ask.disk;
                    r.used_mbits = in.r.used_mbits + A.ask.commit_mbits;
                    r.used_dyn = in.r.used_dyn + A.ask.commit_dyn;
                    A.soa.coll_job[row] += 1;
                    t.coll_tg[row] = in.coll_tg + 1;
                } else {
                    commit_row(A.soa, t, A.ask, row, offers);
                }
#pragma unroll
                for (int p = 0; p < np; p++) {
                    const uint32_t v = (meta0 >> (8 + 8 * p)) & 255u;
                    if (v == kAuxMissing) continue;
                    const uint32_t c = ++counts[t.pset_cnt_off[p] + v];
                    if (fast) t.pset_counts[p][v] = c;
                    if (!t.pset_even[p]) {       // build_spread_table's target boost of this value
                        const double d = desired[t.pset_cnt_off[p] + v];
                        tab[t.pset_tab_off[p] + v] = d != d ? -1.0 : ((d - (double)(c + 1u)) / d) *
                                                                     t.pset_weight_frac[p];
                    }
                }
                state[1] = it + 1;
                sh_nf += st1 == kFiltered;
                sh_ne += st1 == kExhausted;
                if (prof) sh_wprof[2] += wall_clock64() - w2;
            }
        }
        mark(2);
        __syncthreads();
        if (sh_stop) break;
        if (win != 0xFFFFFFFFu) {   // the winner's entry with this placement added
            uint32_t pos = off + win;
            if (pos >= n) pos -= n;
#pragma unroll
            for (int j = 0; j < kFullPer; j++) {
                const uint32_t e = (uint32_t)tid + (uint32_t)j * kFullThreads;
                if (e < m && ent_pos[e] == pos) {
                    ent_sum[e] = parts1[0];
                    ent_meta[e] = sh_win;
                }
            }
        }
        if (any_even) build_spread_table<kFullThreads>(t, counts, tab, scratch);
        __syncthreads();
        mark(3);
    }
    if (prof && tid == 0)
        for (int i = 0; i < 8; i++) prof[i] = tp[i];
    if (prof && tid == 0)
        for (int i = 0; i < 3; i++) prof[8 + i] = sh_wprof[i];
    // the HBM table the next Select starts from
    for (int p = 0; p < np; p++)
        for (int v = tid; v < t.pset_nvals[p]; v += kFullThreads)
            const_cast<double*>(A.spread_tab)[t.pset_tab_off[p] + v] = tab[t.pset_tab_off[p] + v];
}

// The full-pass loop with a service wave (C3's shape: target spreads, no
// device asks or reserved cores). Waves 0-14 hold the options (kSvcPer per
// lane) and run each placement's approximate and exact passes as
// k_fullpass_lds does; wave 15 serves the winners one placement behind. The
// build gives every option its entry with one more placement of the loop as
// well (next sum / meta), so at the resolve thread 0 swaps the winner's next
// entry in and updates its spread boost, and the next placement's passes start
// at once. Meanwhile the service wave loads the winner, writes its record
// (lane 0, dk = 0), evaluates the entry two placements on (lane 1, dk = 2:
// the next entry the winner swaps in) and commits it. The next placement's
// barrier waits for the service, so a winner's next entry is in place before
// it can win again. Results equal k_fullpass_lds. More options than kSvcCap:
// state[5] = 1 before any commit (the host runs k_fullpass_lds instead).
constexpr int kSvcEntryWaves = kFullWaves - 1;
constexpr int kSvcEntryLanes = kSvcEntryWaves * 64;
constexpr int kSvcPer = 4;
constexpr uint32_t kSvcCap = (uint32_t)kSvcEntryLanes * kSvcPer;   // 3840 options, 32 B of LDS each

// LEAN (the host checks): no distinct_hosts, no network asks or static ports,
// no devices, no reserved cores, no distinct_property, no multi-device record:
// an option of the build stays feasible, and the service's evaluation with dk
// placements added is AllocsFit's three comparisons and the scores
// (status_loaded + score_head reduced to the branches such an ask takes).
template <int NP, bool LEAN>
__global__ void __launch_bounds__(kFullThreads) k_fullpass_svc(const SweepArgs* __restrict__ Ap, const uint32_t* visit,
                                                               uint32_t n, uint32_t count, pe_ranked_node* out,
                                                               uint32_t* state) {
    const SweepArgs& A = *Ap;
    extern __shared__ double svc_sum[];                                      // [kSvcCap] score_head sums
    double* next_sum = svc_sum + kSvcCap;                                     // ... with one more placement
    uint32_t* ent_meta = reinterpret_cast<uint32_t*>(next_sum + kSvcCap);     // status | k << 2 | spread values
    uint32_t* next_meta = ent_meta + kSvcCap;
    uint32_t* ent_rank = next_meta + kSvcCap;                                 // visit rank (LimitIterator order)
    uint32_t* ent_row = ent_rank + kSvcCap;
    __shared__ double tab[kAuxPsets * (kAuxValues + 1)];
    __shared__ double desired[kAuxPsets * kAuxValues];
    __shared__ uint32_t counts[kAuxPsets * kAuxValues];
    __shared__ double aff_lds[kAuxValues];
    __shared__ double red_s[kFullWaves];
    __shared__ uint32_t red_r[kFullWaves], red_e[kFullWaves], red_f[kFullWaves], red_x[kFullWaves];
    __shared__ SweepRec red[kFullWaves];
    __shared__ uint32_t scratch[4];
    __shared__ uint32_t sh_nf, sh_ne, sh_stop, sh_win, sh_win_e, sh_m;
    __shared__ uint32_t pend_on, pend_e, pend_nf, pend_ne, pend_it;   // the winner the service wave serves next
    __shared__ double pend_sp;                                        // its spread score at its placement
    __shared__ double parts1[PE_MAX_SCORES];                          // lane 1's parts (unused)
    __shared__ double rcp_k[8];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const TgTables& t = A.tg;
    constexpr int np = NP;
    const uint32_t off = A.offset;
    for (int i = tid; i < kAuxValues; i += kFullThreads) aff_lds[i] = A.aff_vals[i];
    if (tid < 8) rcp_k[tid] = tid ? 1.0 / (double)tid : 0.0;
    if (tid == 0) { sh_m = 0; pend_on = 0; }
    for (int p = 0; p < np; p++)
        for (int v = tid; v < t.pset_nvals[p]; v += kFullThreads) {
            counts[t.pset_cnt_off[p] + v] = t.pset_counts[p][v];
            desired[t.pset_cnt_off[p] + v] = t.pset_desired[p][v];   // target spreads only (the host checks)
        }
    __syncthreads();
    if (np) build_spread_table<kFullThreads>(t, counts, tab, scratch);
    auto spread_of = [&](uint32_t meta) __attribute__((always_inline)) -> double {   // lookup_scores' total
        double sp = 0.0;
#pragma unroll
        for (int p = 0; p < np; p++) {
            const uint32_t v = (meta >> (8 + 8 * p)) & 255u;
            sp += (v == kAuxMissing) ? -1.0 : tab[t.pset_tab_off[p] + v];
        }
        return sp;
    };
    auto load = [&](uint32_t row, NodeIn& in) __attribute__((always_inline)) -> uint32_t {   // the sweep's AUX fetch
        in.r = A.soa.rec[row];
        in.coll_tg = t.coll_tg[row];
        in.dev_free = t.dev_free ? t.dev_free[row] : 0u;
        const uint32_t aux = A.node_aux[row];
        in.feas = aux >> 31;
        return aux;
    };
    // status and score_head of a loaded node with dk placements of this loop
    // added; with a `parts` pointer the parts are written there
    auto head = [&](uint32_t row, const NodeIn& in, uint32_t aux, uint32_t dk, double* parts, double* sum,
                    uint32_t* kk) __attribute__((always_inline)) -> int {
        ScoreIn si;
        const int st = status_loaded(A.soa, t, t.class_ok, A.ask, dk, row, in, &si);
        *kk = 0;
        *sum = 0.0;
        if (st == kOption) {
            si.penalty = A.penalty_bits ? (A.penalty_bits[row >> 5] >> (row & 31)) & 1u : 0u;
            si.aff = aff_lds[aux & 255u];
            si.spread = 0.0;
            *sum = parts ? score_head<true>(A.ask, A.log10, si, parts, *kk)
                         : score_head<false>(A.ask, A.log10, si, nullptr, *kk);
        }
        return st;
    };
    auto final_sum = [&](uint32_t e, uint32_t* kk_out) __attribute__((always_inline)) -> double {
        const uint32_t meta = ent_meta[e];
        double sum = svc_sum[e];
        const double sp = spread_of(meta);
        uint32_t kk = (meta >> 2) & 7u;
        if (sp != 0.0) { sum += sp; kk++; }
        *kk_out = kk;
        return sum;
    };
    auto rank_of_pos = [&](uint32_t pos) __attribute__((always_inline)) -> uint32_t {
        return pos >= off ? pos - off : pos + n - off;
    };
    // build: every option's entry now and with one more placement of the loop
    uint32_t nf = 0, ne = 0;
    for (uint32_t pos = tid; pos < n; pos += kFullThreads) {
        const uint32_t row = visit[pos];
        NodeIn in;
        const uint32_t aux = load(row, in);
        double s;
        uint32_t kk;
        const int st = head(row, in, aux, 0u, nullptr, &s, &kk);
        nf += st == kFiltered;
        ne += st == kExhausted;
        if (st == kOption) {
            const uint32_t e = atomicAdd(&sh_m, 1u);
            if (e < kSvcCap) {
                svc_sum[e] = s;
                ent_meta[e] = (uint32_t)st | (kk << 2) | (aux & 0x00FFFF00u);
                ent_rank[e] = rank_of_pos(pos);
                ent_row[e] = row;
                double s1;
                uint32_t k1;
                const int st1 = head(row, in, aux, 1u, nullptr, &s1, &k1);
                next_sum[e] = s1;
                next_meta[e] = (uint32_t)st1 | (k1 << 2) | (aux & 0x00FFFF00u);
            }
        }
    }
    for (int o = 32; o > 0; o >>= 1) {
        nf += (uint32_t)__shfl_xor((int)nf, o);
        ne += (uint32_t)__shfl_xor((int)ne, o);
    }
    if (lane == 0) { red_f[wid] = nf; red_x[wid] = ne; }
    __syncthreads();
    const uint32_t m = sh_m;
    if (m > kSvcCap) {   // uniform: nothing committed yet, the host takes the other loop
        if (tid == 0) state[5] = 1;
        return;
    }
    if (tid == 0) {
        uint32_t a = 0, b = 0;
        for (int w = 0; w < kFullWaves; w++) { a += red_f[w]; b += red_x[w]; }
        sh_nf = a;
        sh_ne = b;
        sh_stop = 0;
    }
    __syncthreads();
    // the service of one winner (lanes 0 and 1 of wave 15): its record (lane
    // 0: the placement's state, dk = 0), its entry two placements on (lane 1,
    // dk = 2: what it swaps in when it wins again), the commit (lane 0)
    auto serve = [&]() __attribute__((always_inline)) {
        const uint32_t e = pend_e, row = ent_row[e];
        pe_ranked_node* o = out + pend_it;
        NodeIn in;
        const uint32_t aux = load(row, in);
        double s;
        uint32_t kk;
        // both lanes take the parts-keeping path (lockstep, no divergence)
        int st;
        if (LEAN) {
            const uint32_t dk = lane == 0 ? 0u : 2u;
            const NodeRec& r = in.r;
            const int64_t ucpu = r.used_cpu + (int64_t)(dk + 1) * A.ask.cpu;
            const int64_t umem = r.used_mem + (int64_t)(dk + 1) * A.ask.mem;
            const int64_t udisk = r.used_disk + (int64_t)(dk + 1) * A.ask.disk;
            s = 0.0;
            kk = 0;
            if (r.cap_cpu < ucpu || r.cap_mem < umem || r.cap_disk < udisk) {   // AllocsFit
                st = kExhausted;
            } else {
                ScoreIn si;
                si.ccpu = r.cap_cpu;
                si.cmem = r.cap_mem;
                si.ucpu = ucpu;
                si.umem = umem;
                si.dev_aff = 0.0;
                si.coll = in.coll_tg + dk;
                si.penalty = A.penalty_bits ? (A.penalty_bits[row >> 5] >> (row & 31)) & 1u : 0u;
                si.aff = aff_lds[aux & 255u];
                si.spread = 0.0;
                s = score_head<true>(A.ask, A.log10, si, lane == 0 ? o->scores : parts1, kk);
                st = kOption;
            }
        } else {
            st = head(row, in, aux, lane == 0 ? 0u : 2u, lane == 0 ? o->scores : parts1, &s, &kk);
        }
        if (lane == 1) {
            next_sum[e] = s;
            next_meta[e] = (uint32_t)st | (kk << 2) | (aux & 0x00FFFF00u);
        } else {
            const double sp = pend_sp;
            if (sp != 0.0) {   // SpreadIterator (spread.go:110-174)
                s += sp;
                o->scores[kk] = sp;
                kk++;
            }
            o->row = (int32_t)row;
            o->final_score = s / (double)kk;   // ScoreNormalizationIterator (rank.go:762-767)
            o->n_scores = kk;
            o->nodes_evaluated = n;            // a full pass pulls every node
            o->nodes_filtered = pend_nf;
            o->nodes_exhausted = pend_ne;
            o->new_offset = off;               // and leaves the cursor where it is
            record_offers(A.soa, A.ask, t, row, 0u, o);
            NodeRec& r = A.soa.rec[row];       // commit_row from the loaded values: stores only
            r.used_cpu = in.r.used_cpu + A.ask.cpu;
            r.used_mem = in.r.used_mem + A.ask.mem;
            r.used_disk = in.r.used_disk + A.ask.disk;
            r.used_mbits = in.r.used_mbits + A.ask.commit_mbits;
            r.used_dyn = in.r.used_dyn + A.ask.commit_dyn;
            A.soa.coll_job[row] += 1;
            t.coll_tg[row] = in.coll_tg + 1;
            pend_on = 0;   // thread 0 sets the next one after the barrier
        }
    };
    for (uint32_t it = 0; it < count; it++) {
        if (wid < kSvcEntryWaves) {
            double ap[kSvcPer];
            double amax = -__builtin_inff();
#pragma unroll
            for (int j = 0; j < kSvcPer; j++) {
                const uint32_t e = (uint32_t)tid + (uint32_t)j * kSvcEntryLanes;
                ap[j] = -__builtin_inff();
                if (e < m) {
                    uint32_t kk;
                    const double sum = final_sum(e, &kk);
                    if ((ent_meta[e] & 3u) == (uint32_t)kOption) ap[j] = sum * rcp_k[kk];
                }
                amax = ap[j] > amax ? ap[j] : amax;
            }
            amax = __ockl_wfred_max_f64(amax);
            const double cut = amax - (__builtin_fabs(amax) * 0x1p-48 + 0x1p-1000);
            double best = -__builtin_inff();
            uint32_t best_rank = 0xFFFFFFFFu, best_e = 0xFFFFFFFFu;
#pragma unroll
            for (int j = 0; j < kSvcPer; j++) {
                const bool near = ap[j] >= cut && ap[j] != -__builtin_inff();   // options only
                if (__ballot(near)) {
                    if (near) {
                        const uint32_t e = (uint32_t)tid + (uint32_t)j * kSvcEntryLanes;
                        uint32_t kk;
                        const double sc = final_sum(e, &kk) / (double)kk;
                        const uint32_t rk = ent_rank[e];
                        if (sc > best || (sc == best && rk < best_rank)) { best = sc; best_rank = rk; best_e = e; }
                    }
                }
            }
            {   // the wave's (max, earliest rank) over its few candidate lanes
                uint64_t cand = __ballot(best_rank != 0xFFFFFFFFu);
                double wb = -__builtin_inff();
                uint32_t wr = 0xFFFFFFFFu, we = 0xFFFFFFFFu;
                while (cand) {
                    const int l = __builtin_ctzll(cand);
                    cand &= cand - 1;
                    const double b = readlane_f64(best, l);
                    const uint32_t r = (uint32_t)__builtin_amdgcn_readlane((int)best_rank, l);
                    if (b > wb || (b == wb && r < wr)) {
                        wb = b;
                        wr = r;
                        we = (uint32_t)__builtin_amdgcn_readlane((int)best_e, l);
                    }
                }
                if (lane == 0) { red_s[wid] = wb; red_r[wid] = wr; red_e[wid] = we; }
            }
        } else {
            if (pend_on && lane < 2) serve();
            if (lane == 0) { red_s[wid] = -__builtin_inff(); red_r[wid] = 0xFFFFFFFFu; }
        }
        __syncthreads();
        // every thread resolves the block's winner (max score, then the
        // earliest rank among the waves holding it)
        double best = lane < kFullWaves ? red_s[lane] : -__builtin_inff();
        best = __ockl_wfred_max_f64(best);
        uint32_t win = __ockl_wfred_min_u32(lane < kFullWaves && red_s[lane] == best ? red_r[lane] : 0xFFFFFFFFu);
        bool skip_rule = false;
        if (win != 0xFFFFFFFFu && !(best > 0.0)) {   // every option non-positive: the skip rule decides (rare)
            skip_rule = true;
            SweepRec r;
            rec_init(r);
            for (uint32_t e = tid; e < m; e += kFullThreads) {
                if ((ent_meta[e] & 3u) != (uint32_t)kOption) continue;
                uint32_t kk;
                const double sum = final_sum(e, &kk);
                rec_add(r, ent_rank[e], sum / (double)kk);
            }
            rec_block_reduce<kFullThreads>(r, red);
            if (tid == 0) sh_win = rec_winner(r);
            __syncthreads();
            win = sh_win;
            if (win != 0xFFFFFFFFu) {
                for (uint32_t e = tid; e < m; e += kFullThreads)
                    if (ent_rank[e] == win) sh_win_e = e;
            }
            __syncthreads();
        }
        if (tid == 0) {
            pe_ranked_node* o = out + it;
            if (win == 0xFFFFFFFFu) {
                o->row = -1;
                o->nodes_evaluated = n;            // a full pass pulls every node
                o->nodes_filtered = sh_nf;
                o->nodes_exhausted = sh_ne;
                o->new_offset = off;
                state[0] = 1;
                sh_stop = 1;
            } else {
                uint32_t e = sh_win_e;
                if (!skip_rule)
                    for (int w = 0; w < kFullWaves; w++)
                        if (red_s[w] == best && red_r[w] == win) { e = red_e[w]; break; }
                const uint32_t meta0 = ent_meta[e];
                pend_e = e;
                pend_it = it;
                pend_nf = sh_nf;
                pend_ne = sh_ne;
                pend_sp = spread_of(meta0);   // the boost this placement saw
                pend_on = 1;
                // the winner's entry with this placement added
                svc_sum[e] = next_sum[e];
                ent_meta[e] = next_meta[e];
                const uint32_t st1 = next_meta[e] & 3u;
                sh_nf += st1 == (uint32_t)kFiltered;
                sh_ne += st1 == (uint32_t)kExhausted;
#pragma unroll
                for (int p = 0; p < np; p++) {   // the target boost of the winner's value (build_spread_table)
                    const uint32_t v = (meta0 >> (8 + 8 * p)) & 255u;
                    if (v == kAuxMissing) continue;
                    const uint32_t c = ++counts[t.pset_cnt_off[p] + v];
                    t.pset_counts[p][v] = c;
                    const double d = desired[t.pset_cnt_off[p] + v];
                    tab[t.pset_tab_off[p] + v] = d != d ? -1.0 : ((d - (double)(c + 1u)) / d) * t.pset_weight_frac[p];
                }
                state[1] = it + 1;
            }
        }
        __syncthreads();
        if (sh_stop) break;
    }
    if (wid == kSvcEntryWaves && pend_on && lane < 2) serve();   // the last winner
    // the HBM table the next Select starts from
    for (int p = 0; p < np; p++)
        for (int v = tid; v < t.pset_nvals[p]; v += kFullThreads)
            const_cast<double*>(A.spread_tab)[t.pset_tab_off[p] + v] = tab[t.pset_tab_off[p] + v];
}

// Grid-wide barrier of the persistent count loop (every workgroup resident;
// the host launches at most one per CU). Stores of the whole workgroup are
// released at agent scope before the arrival and acquired after it, so rows
// committed by workgroup 0 on one XCD are seen by the sweeps on the others
// (MI355X_MICROARCH.md, inter-workgroup visibility). The wait is bounded: on
// timeout the workgroup sets state[4] and every workgroup leaves the loop.
__device__ __forceinline__ bool grid_sync(uint32_t* state, uint32_t nblocks, uint32_t* gen) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __syncthreads();
    __shared__ uint32_t ok;
    if (threadIdx.x == 0) {
        ok = 1;
        const uint32_t g = *gen;
        const uint32_t arrived = __hip_atomic_fetch_add(&state[2], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
        if (arrived == nblocks) {
            __hip_atomic_store(&state[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&state[3], g + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            uint32_t spins = 0;
            while (__hip_atomic_load(&state[3], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g) {
                if (++spins > (1u << 20) ||
                    __hip_atomic_load(&state[4], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    __hip_atomic_store(&state[4], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        *gen = g + 1;
    }
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    return ok != 0;
}

// Persistent full-pass count loop: every placement is sweep_block on all
// workgroups, a grid barrier, step_block on workgroup 0 (merge, record,
// commit, next spread table), a grid barrier. state: [0] stopped, [1] placed,
// [2] barrier arrivals, [3] barrier generation, [4] barrier timeout.
template <bool AUX>
__global__ void __launch_bounds__(256) k_sweep_loop(SweepArgs A, uint32_t count, const uint32_t* visit, uint32_t n,
                                                    uint32_t offset, pe_ranked_node* out, uint32_t* state) {
    __shared__ uint32_t gen;
    __shared__ uint32_t stop;
    if (threadIdx.x == 0) gen = __hip_atomic_load(&state[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    for (uint32_t k = 0; k < count; k++) {
        sweep_block<256, false, 0, AUX>(A);
        if (!grid_sync(state, gridDim.x, &gen)) return;
        if (blockIdx.x == 0) step_block(A, gridDim.x, visit, n, offset, out, state);
        if (!grid_sync(state, gridDim.x, &gen)) return;
        if (threadIdx.x == 0) stop = __hip_atomic_load(&state[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        if (stop) return;
    }
}

// node_feas[row] = class_ok[cls] && node_ok[row]: one verdict byte per node so
// the count loop issues a single dependent round trip per node.
// Host -> device upload as a kernel: the source is page-locked mapped host
// memory read directly over the bus (a DMA copy costs more setup per call than
// the whole transfer of these small per-evaluation arrays).
__global__ void __launch_bounds__(256) k_upload(unsigned char* dst, const unsigned char* src, size_t bytes) {
    const size_t n16 = bytes / 16;
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
        reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
    for (size_t i = n16 * 16 + (size_t)blockIdx.x * 256 + threadIdx.x; i < bytes; i += stride) dst[i] = src[i];
}

// Per-node count arrays from a sorted sparse list (key = row << 5 | array,
// value = count): each thread owns one row, zeroes it in every array and
// writes the row's entries found by binary search. A deferred ResetPlan (R.rec)
// rides in the same launch: its arrays are disjoint from the counts.
__global__ void __launch_bounds__(256) k_counts(CountDsts D, uint32_t nd, uint32_t n, const uint2* ents, uint32_t m,
                                                ResetArgs R) {
    counts_apply(D, nd, n, ents, m, R, blockIdx.x * 256 + threadIdx.x, gridDim.x * 256);
}

// ResetPlan in one launch: the proposed state back to the snapshot (node
// records, device free counts), no plan preemptions.
__global__ void __launch_bounds__(256) k_reset_plan(NodeRec* rec, const NodeRec* base_rec, uint32_t* dev_free,
                                                   const uint32_t* dev_free_base, uint32_t n, uint8_t* preempted,
                                                   uint32_t m, uint32_t* pcount, uint32_t keys) {
    const uint32_t stride = gridDim.x * 256;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        rec[i] = base_rec[i];
        dev_free[i] = dev_free_base[i];
    }
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < m; i += stride) preempted[i] = 0;
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < keys; i += stride) pcount[i] = 0;
}

__global__ void __launch_bounds__(256) k_fold_feas(NodeSoA s, const uint8_t* class_ok, const uint8_t* node_ok,
                                                   uint8_t* feas) {
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < s.n; row += gridDim.x * blockDim.x) {
        bool ok = class_ok[s.rec[row].cls] != 0;
        if (node_ok) ok = ok && node_ok[row] != 0;
        feas[row] = ok ? 1 : 0;
    }
}

// k_fold_feas with the class table read from the page-locked staging ring:
// every workgroup pulls the (small) table over the bus into LDS, workgroup 0
// also stores it to its device copy for the later kernels; saves the
// separate upload launch.
__global__ void __launch_bounds__(256) k_fold_feas_staged(NodeSoA s, const uint8_t* class_src, uint8_t* class_dst,
                                                          uint32_t ncls, const uint8_t* node_ok, uint8_t* feas) {
    __shared__ uint8_t cls_ok[kFoldMaxClasses];
    for (uint32_t c = threadIdx.x; c < ncls; c += blockDim.x) {
        const uint8_t v = class_src[c];
        cls_ok[c] = v;
        if (blockIdx.x == 0) class_dst[c] = v;
    }
    __syncthreads();
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < s.n; row += gridDim.x * blockDim.x) {
        const uint32_t c = s.rec[row].cls;
        bool ok = c < ncls && cls_ok[c] != 0;
        if (node_ok) ok = ok && node_ok[row] != 0;
        feas[row] = ok ? 1 : 0;
    }
}

// node_aux[row] (SweepArgs): verdict bit, affinity index (per class, or per
// node when the affinities escape the class), spread values of the first
// kAuxPsets properties. Built once per (job, task group) tables.
__global__ void __launch_bounds__(256) k_fold_aux(NodeSoA s, TgTables t, const uint8_t* aff_idx_class,
                                                  const uint8_t* aff_idx_node, uint32_t* aux) {
    for (uint32_t row = blockIdx.x * blockDim.x + threadIdx.x; row < s.n; row += gridDim.x * blockDim.x) {
        const uint32_t c = s.rec[row].cls;
        bool ok = t.class_ok[c] != 0;
        if (t.node_ok) ok = ok && t.node_ok[row] != 0;
        uint32_t x = ok ? 1u << 31 : 0u;
        x |= aff_idx_node ? aff_idx_node[row] : (aff_idx_class ? aff_idx_class[c] : 0u);
        for (int p = 0; p < t.n_psets && p < kAuxPsets; p++) {
            const uint32_t v = pset_value(t, p, row, c);
            x |= (v == kMissing ? kAuxMissing : v) << (8 + 8 * p);
        }
        aux[row] = x;
    }
}

// Static port gate of a task group (status_loaded): blocked rows stay 0, the
// others hold the group's collision count + 1 at build time.
__global__ void __launch_bounds__(256) k_static_gate(const uint8_t* blocked, const uint32_t* coll_tg, uint32_t* gate,
                                                     uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) gate[i] = blocked[i] ? 0u : coll_tg[i] + 1u;
}

// Multi-device gates (TgTables::md): the host wrote the admitted placement
// count in `lim` (kMdUnbounded: no limit); the rows get the group's collision
// count at build time added (saturating below ~0u, which marks other rows).
__global__ void __launch_bounds__(256) k_md_gate(MdNet* md, const uint32_t* coll_tg, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    MdNet& m = md[i];
    if (m.lim == ~0u) return;
    const uint32_t c = coll_tg[i];
    m.coll = c;
    const uint64_t lim = (uint64_t)c + m.lim;
    m.lim = (m.lim == kMdUnbounded || lim >= (uint64_t)kMdUnbounded) ? kMdUnbounded : (uint32_t)lim;
}

#include "evict.inc"

}  // namespace pe

// ---- launch wrappers (host) ------------------------------------------------
hipError_t pe_launch_static_gate(const uint8_t* blocked, const uint32_t* coll_tg, uint32_t* gate, uint32_t n,
                                 hipStream_t st);
size_t pe_place_lds_bytes(bool full, int hash_bits, bool packed, size_t pset_bytes) {
    size_t b = (size_t)(packed ? 4u : 8u) * ((size_t)1 << hash_bits);
    if (full) b += pset_bytes;
    return b;
}

hipError_t pe_launch_place(const pe::BatchArgs* a, uint32_t n_evals, bool full, hipStream_t st) {
    if (full && a->packed_overlay) return hipErrorInvalidValue;   // packed entries: windowed kernel only
    const size_t lds = pe_place_lds_bytes(full, a->hash_bits, a->packed_overlay != 0, a->pset_lds);
    if (full) {
        // few evaluations: 1024-lane workgroups keep more rows in flight per pass
        // reserved cores are a separate instantiation (their code costs the others registers)
        const bool cores = a->ask.cores > 0;
        if (n_evals <= 64) {
            if (cores) hipLaunchKernelGGL((pe::k_place<1024, true, true>), dim3(n_evals), dim3(1024), lds, st, *a);
            else hipLaunchKernelGGL((pe::k_place<1024, true, false>), dim3(n_evals), dim3(1024), lds, st, *a);
        } else {
            if (cores) hipLaunchKernelGGL((pe::k_place<256, true, true>), dim3(n_evals), dim3(256), lds, st, *a);
            else hipLaunchKernelGGL((pe::k_place<256, true, false>), dim3(n_evals), dim3(256), lds, st, *a);
        }
    } else {
        hipLaunchKernelGGL(pe::k_window, dim3(n_evals), dim3(64), lds, st, *a);
    }
    return hipGetLastError();
}

// Phase-static windowed loop: k_base over the snapshot, then k_chain with a
// persistent grid of at most `max_blocks` workgroups (one evaluation each at a time).
uint32_t pe_chain_max_n() { return pe::kChainMaxN; }
uint32_t pe_emit_grid(uint32_t count) { return count ? (count + pe::kEmitBlock - 1) / pe::kEmitBlock : 1u; }
uint32_t pe_chain_max_limit() { return pe::kMaxChainLimit; }

size_t pe_chain_lds_bytes(int hash_bits, bool packed, uint32_t n) {
    if (n > pe::kChainMaxN) n = pe::kChainMaxN;   // nb / nx cover one window
    return (size_t)(packed ? 4u : 8u) * ((size_t)1 << hash_bits) + 4u * (((size_t)n + 3u) & ~(size_t)1);
}

int pe_chain_blocks_per_cu(size_t lds) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pe::k_chain<pe::kChainItems, false>, pe::kChainBlock, lds) !=
            hipSuccess || nb <= 0)
        nb = 1;
    return nb;
}

// Shape of a launch: the fewest positions per lane that hold one window of
// the list. PE_CHAIN_ITEMS=4 / 16 asks for a larger shape (tests run every
// shape on the same list); a smaller one than the list needs is never used.
static int chain_items(uint32_t n_visit) {
    int items = n_visit > pe::kChainBlock * 4u ? 16 : (n_visit > pe::kChainBlock ? 4 : 1);
    if (const char* e = std::getenv("PE_CHAIN_ITEMS")) {
        const int forced = std::atoi(e);
        if (forced > items) items = forced >= 16 ? 16 : 4;
    }
    return items;
}

int pe_chain_shape(uint32_t n_visit) { return chain_items(n_visit); }

// Largest list / count / class table a fused launch (BatchArgs::fused) takes.
uint32_t pe_chain_fused_max_n() { return pe::kChainBlock * 4u; }
uint32_t pe_chain_fused_max_count() { return 256u; }
uint32_t pe_chain_fused_max_classes() { return pe::kFusedMaxClasses; }

// split (or null): five events recorded before k_base and after k_base,
// k_chain, k_emit and k_emit_writeback (per-kernel device time, PE_KERNEL_SPLIT)
hipError_t pe_launch_chain(const pe::BatchArgs* a, uint32_t n_evals, uint32_t max_blocks, hipStream_t st,
                           hipEvent_t* split) {
    if (!a->base || !a->chain_vs || (a->n_visit > pe::kChainMaxN && n_evals != 1) || a->class_ok_stride ||
        a->limit > pe::kMaxChainLimit || a->count >= (1u << 18))   // redo entries pack count | position << 18
        return hipErrorInvalidValue;
    if (a->base_by_pos && n_evals != 1) return hipErrorInvalidValue;
    if (a->perm_src && (!a->base_by_pos || !a->perm_dst)) return hipErrorInvalidValue;
    if (a->fold.feas && (!a->fold.class_src || !a->fold.class_dst || a->fold.ncls > pe::kFoldMaxClasses))
        return hipErrorInvalidValue;
    const size_t lds = pe_chain_lds_bytes(a->hash_bits, a->packed_overlay != 0, a->n_visit);
    uint32_t grid = n_evals < max_blocks ? n_evals : max_blocks;
    if (grid == 0) grid = 1;
    const int items = chain_items(a->n_visit);
    if (a->fused) {
        // one launch: fold, first-phase values, chain, records, writeback
        if (n_evals != 1 || !a->base_by_pos || a->base1 || !a->emit || !a->emit_out || items > 4 ||
            a->count > pe_chain_fused_max_count() || (a->fold.feas && a->fold.ncls > pe::kFusedMaxClasses))
            return hipErrorInvalidValue;
        if (split) for (int k = 0; k < 2; k++) (void)hipEventRecord(split[k], st);
        if (items == 1) hipLaunchKernelGGL((pe::k_chain<1, true>), dim3(1), dim3(pe::kChainBlock), lds, st, *a, 1u);
        else hipLaunchKernelGGL((pe::k_chain<4, true>), dim3(1), dim3(pe::kChainBlock), lds, st, *a, 1u);
        if (split) for (int k = 2; k < 5; k++) (void)hipEventRecord(split[k], st);
        return hipGetLastError();
    }
    const uint32_t m = a->base_by_pos ? a->n_visit : a->soa.n;
    uint32_t blocks = ((a->base1 ? 2u * m : m) + pe::kBaseBlock - 1) / pe::kBaseBlock;
    if (blocks > 8192) blocks = 8192;
    if (blocks == 0) blocks = 1;
    if (split) (void)hipEventRecord(split[0], st);
    if (a->fold.feas) hipLaunchKernelGGL(pe::k_base<true>, dim3(blocks), dim3(pe::kBaseBlock), 0, st, *a);
    else hipLaunchKernelGGL(pe::k_base<false>, dim3(blocks), dim3(pe::kBaseBlock), 0, st, *a);
    if (split) (void)hipEventRecord(split[1], st);
    switch (items) {
    case 1: hipLaunchKernelGGL((pe::k_chain<1, false>), dim3(grid), dim3(pe::kChainBlock), lds, st, *a, n_evals); break;
    case 4: hipLaunchKernelGGL((pe::k_chain<4, false>), dim3(grid), dim3(pe::kChainBlock), lds, st, *a, n_evals); break;
    default:
        hipLaunchKernelGGL((pe::k_chain<pe::kChainItems, false>), dim3(grid), dim3(pe::kChainBlock), lds, st, *a,
                           n_evals);
    }
    if (split) (void)hipEventRecord(split[2], st);
    if (a->emit) {
        if (n_evals != 1 || !a->emit_out || !a->emit_ov || !a->emit_n) return hipErrorInvalidValue;
        hipLaunchKernelGGL(pe::k_emit, dim3(pe_emit_grid(a->count)), dim3(pe::kEmitBlock), 0, st, *a);
        if (split) (void)hipEventRecord(split[3], st);
        const uint32_t wb = (a->count + 255) / 256;   // overlay rows <= placements
        hipLaunchKernelGGL(pe::k_emit_writeback, dim3(wb ? wb : 1), dim3(256), 0, st, *a);
    } else if (split) {
        (void)hipEventRecord(split[3], st);
    }
    if (split) (void)hipEventRecord(split[4], st);
    return hipGetLastError();
}

hipError_t pe_launch_rank_of(const uint32_t* list, uint32_t n_list, uint32_t* rank_of, uint32_t n_rows, hipStream_t st) {
    hipError_t e = hipMemsetAsync(rank_of, 0xFF, sizeof(uint32_t) * (size_t)n_rows, st);
    if (e != hipSuccess || !n_list) return e;
    hipLaunchKernelGGL(pe::k_rank_of, dim3((n_list + 255) / 256), dim3(256), 0, st, list, n_list, rank_of);
    return hipGetLastError();
}

hipError_t pe_launch_system(const pe::SystemArgs* a, hipStream_t st) {
    if (a->rank_of && a->res) {   // row order: coalesced evaluation, then the list-order gather
        uint32_t b1 = (a->n_rows + 255) / 256;
        if (b1 > 8192) b1 = 8192;
        if (b1 == 0) b1 = 1;
        static const bool scatter = [] {
            const char* e = std::getenv("PE_SYS_SCATTER");
            return e && e[0] == '1';
        }();
        if (scatter || !a->n_list) {   // outcomes stored at list positions directly (or kept by row)
            hipLaunchKernelGGL(pe::k_system_rows, dim3(b1), dim3(256), 0, st, *a);
            return hipGetLastError();
        }
        pe::SystemArgs r = *a;
        r.n_list = 0;   // outcomes by row into res
        hipLaunchKernelGGL(pe::k_system_rows, dim3(b1), dim3(256), 0, st, r);
        hipLaunchKernelGGL(pe::k_system_gather, dim3((a->n_list + 255) / 256), dim3(256), 0, st, a->list, a->n_list,
                           a->res, a->out_score, a->out_status);
        return hipGetLastError();
    }
    uint32_t blocks = (a->n_list + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_system, dim3(blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}

hipError_t pe_launch_commit(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, uint32_t row,
                            uint32_t offers, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_commit, dim3(1), dim3(64), 0, st, *s, *t, *a, row, offers);
    return hipGetLastError();
}

hipError_t pe_launch_apply_commits(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                                   const uint32_t* offers, uint32_t n, int sign, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pe::k_apply_commits, dim3((n + 255) / 256), dim3(256), 0, st, *s, *t, *a, rows, offers, n, sign);
    return hipGetLastError();
}

// Select with Preempt: per-position evict evaluation, then the window resolve.
hipError_t pe_launch_resolve(const pe::EvictResolveArgs* r, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_evict_resolve, dim3(1), dim3(pe::kResolveBlock), 0, st, *r);
    return hipGetLastError();
}

// Eviction widths (evict.inc): W = 1 (<= 32 allocs per node), 8 (<= 256) or
// 32 (<= 1024 allocs, ProposedAllocs <= 2048). A wide launch keeps its
// per-lane lists in scratch (lane-interleaved, so the lanes' accesses to one
// list element coalesce; W = 32 is ~19 KB per lane): the grid is capped lower
// so that the scratch reservation stays small (32 x 256 lanes: ~150 MB).
static inline bool evict_width_ok(uint32_t w) { return w == 1u || w == 8u || w == 32u; }
static inline uint32_t evict_blocks(uint32_t n, uint32_t w) {
    uint32_t blocks = (n + 255) / 256;
    const uint32_t cap = w == 1u ? 2048u : w == 8u ? 256u : 32u;
    if (blocks > cap) blocks = cap;
    return blocks ? blocks : 1u;
}

hipError_t pe_launch_evict(const pe::PreemptArgs* a, const pe::EvictResolveArgs* r, hipStream_t st) {
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    const uint32_t blocks = evict_blocks(a->n_visit, a->mask_words);
    if (a->mask_words == 1u) hipLaunchKernelGGL((pe::k_evict<false, 1>), dim3(blocks), dim3(256), 0, st, *a);
    else if (a->mask_words == 8u) hipLaunchKernelGGL((pe::k_evict<false, 8>), dim3(blocks), dim3(256), 0, st, *a);
    else hipLaunchKernelGGL((pe::k_evict<false, 32>), dim3(blocks), dim3(256), 0, st, *a);
    hipLaunchKernelGGL(pe::k_evict_resolve, dim3(1), dim3(pe::kResolveBlock), 0, st, *r);
    return hipGetLastError();
}

hipError_t pe_launch_census(const pe::BatchArgs* a, uint32_t* counts, uint8_t* status, double* score,
                            hipStream_t st, double* parts, uint8_t* nparts) {
    uint32_t blocks = (a->n_visit + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    if (parts) {
        if (!nparts || !status) return hipErrorInvalidValue;
        hipLaunchKernelGGL(pe::k_census<true>, dim3(blocks), dim3(256), 0, st, *a, counts, status, score, parts, nparts);
    } else {
        hipLaunchKernelGGL(pe::k_census<false>, dim3(blocks), dim3(256), 0, st, *a, counts, status, score, parts,
                           nparts);
    }
    return hipGetLastError();
}

hipError_t pe_launch_evict_only(const pe::PreemptArgs* a, hipStream_t st) {
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    const uint32_t blocks = evict_blocks(a->n_visit, a->mask_words);
    const uint32_t w = a->mask_words;
    if (a->parts_out) {
        if (!a->nparts_out || !a->mask_out || !a->offers_out) return hipErrorInvalidValue;
        if (w == 1u) hipLaunchKernelGGL((pe::k_evict<true, 1>), dim3(blocks), dim3(256), 0, st, *a);
        else if (w == 8u) hipLaunchKernelGGL((pe::k_evict<true, 8>), dim3(blocks), dim3(256), 0, st, *a);
        else hipLaunchKernelGGL((pe::k_evict<true, 32>), dim3(blocks), dim3(256), 0, st, *a);
    } else {
        if (w == 1u) hipLaunchKernelGGL((pe::k_evict<false, 1>), dim3(blocks), dim3(256), 0, st, *a);
        else if (w == 8u) hipLaunchKernelGGL((pe::k_evict<false, 8>), dim3(blocks), dim3(256), 0, st, *a);
        else hipLaunchKernelGGL((pe::k_evict<false, 32>), dim3(blocks), dim3(256), 0, st, *a);
    }
    return hipGetLastError();
}

// mask: mask_words + 1 words (the preempted set, then the kEvict* flags)
hipError_t pe_launch_evict_record(const pe::PreemptArgs* a, uint32_t row, pe_ranked_node* out, uint32_t* mask,
                                  hipStream_t st) {
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    if (a->mask_words == 1u) hipLaunchKernelGGL(pe::k_evict_record<1>, dim3(1), dim3(64), 0, st, *a, row, out, mask);
    else if (a->mask_words == 8u) hipLaunchKernelGGL(pe::k_evict_record<8>, dim3(1), dim3(64), 0, st, *a, row, out, mask);
    else hipLaunchKernelGGL(pe::k_evict_record<32>, dim3(1), dim3(64), 0, st, *a, row, out, mask);
    return hipGetLastError();
}

hipError_t pe_launch_commit_evicted(const pe::PreemptArgs* a, uint8_t* preempted, uint32_t* pcount,
                                    uint32_t* dev_free, uint32_t* placed, hipStream_t st) {
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    uint32_t blocks = (a->n_visit + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks == 0) blocks = 1;
    if (a->mask_words == 1u)
        hipLaunchKernelGGL(pe::k_commit_evicted<1>, dim3(blocks), dim3(256), 0, st, *a, preempted, pcount, dev_free,
                           placed);
    else if (a->mask_words == 8u)
        hipLaunchKernelGGL(pe::k_commit_evicted<8>, dim3(blocks), dim3(256), 0, st, *a, preempted, pcount, dev_free,
                           placed);
    else
        hipLaunchKernelGGL(pe::k_commit_evicted<32>, dim3(blocks), dim3(256), 0, st, *a, preempted, pcount, dev_free,
                           placed);
    return hipGetLastError();
}

// mask: mask_words words in device memory
hipError_t pe_launch_commit_preempt(const pe::PreemptArgs* a, uint32_t row, const uint32_t* mask, uint8_t* preempted,
                                    uint32_t* pcount, uint32_t* dev_free, hipStream_t st) {
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    if (a->mask_words == 1u)
        hipLaunchKernelGGL(pe::k_commit_preempt<1>, dim3(1), dim3(64), 0, st, *a, row, mask, preempted, pcount,
                           dev_free);
    else if (a->mask_words == 8u)
        hipLaunchKernelGGL(pe::k_commit_preempt<8>, dim3(1), dim3(64), 0, st, *a, row, mask, preempted, pcount,
                           dev_free);
    else
        hipLaunchKernelGGL(pe::k_commit_preempt<32>, dim3(1), dim3(64), 0, st, *a, row, mask, preempted, pcount,
                           dev_free);
    return hipGetLastError();
}

hipError_t pe_launch_upload(void* dst, const void* src_mapped, size_t bytes, hipStream_t st) {
    if (!bytes) return hipSuccess;
    if (((uintptr_t)dst | (uintptr_t)src_mapped) & 15) return hipErrorInvalidValue;
    size_t blocks = (bytes / 16 + 255) / 256;
    if (blocks > 256) blocks = 256;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_upload, dim3((uint32_t)blocks), dim3(256), 0, st, static_cast<unsigned char*>(dst),
                       static_cast<const unsigned char*>(src_mapped), bytes);
    return hipGetLastError();
}

hipError_t pe_launch_scatter_rows(void* dst, uint32_t words, const void* payload_mapped, uint32_t n, hipStream_t st) {
    if (!n || !words) return hipSuccess;
    if (((uintptr_t)dst | (uintptr_t)payload_mapped) & 3) return hipErrorInvalidValue;
    uint64_t blocks = ((uint64_t)n * words + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    hipLaunchKernelGGL(pe::k_scatter_rows, dim3((uint32_t)blocks), dim3(256), 0, st, static_cast<uint32_t*>(dst), words,
                       static_cast<const uint32_t*>(payload_mapped), n);
    return hipGetLastError();
}

hipError_t pe_launch_counts(const pe::CountDsts* d, uint32_t nd, uint32_t n, const uint2* ents, uint32_t m,
                            const pe::ResetArgs* r, hipStream_t st) {
    if (nd > (uint32_t)pe::kMaxCountDst || (m && !ents) || n >= (1u << 27)) return hipErrorInvalidValue;
    pe::ResetArgs R;
    std::memset(&R, 0, sizeof(R));
    if (r && r->rec) {
        if (!r->base_rec || !r->dev_free || !r->dev_free_base || (r->m && !r->preempted) || (r->keys && !r->pcount))
            return hipErrorInvalidValue;
        R = *r;
    }
    const uint32_t span = std::max(n, std::max(R.n, std::max(R.m, R.keys)));
    if (!span) return hipSuccess;
    uint32_t blocks = (span + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(pe::k_counts, dim3(blocks), dim3(256), 0, st, *d, nd, n, ents, m, R);
    return hipGetLastError();
}

hipError_t pe_launch_plan_stop(pe::NodeRec* rec, uint32_t* dev_free, const pe::PreemptAlloc* allocs,
                               uint8_t* preempted, const uint32_t* slots, const uint32_t* rows, uint32_t n, int sign,
                               uint64_t* core_used, const uint64_t* palloc_cores, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(pe::k_plan_stop, dim3((n + 63) / 64), dim3(64), 0, st, rec, dev_free, allocs, preempted, slots,
                       rows, n, sign, core_used, palloc_cores);
    return hipGetLastError();
}

hipError_t pe_launch_evict_trace(const pe::PreemptArgs* a, const uint32_t* rows, uint32_t n, uint32_t* code,
                                 double* named, hipStream_t st) {
    if (!n) return hipSuccess;
    if (!evict_width_ok(a->mask_words)) return hipErrorInvalidValue;
    if (a->mask_words == 1u)
        hipLaunchKernelGGL(pe::k_evict_trace<1>, dim3((n + 63) / 64), dim3(64), 0, st, *a, rows, n, code, named);
    else if (a->mask_words == 8u)
        hipLaunchKernelGGL(pe::k_evict_trace<8>, dim3((n + 63) / 64), dim3(64), 0, st, *a, rows, n, code, named);
    else
        hipLaunchKernelGGL(pe::k_evict_trace<32>, dim3((n + 63) / 64), dim3(64), 0, st, *a, rows, n, code, named);
    return hipGetLastError();
}

hipError_t pe_launch_commit_rows(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                                 uint32_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(pe::k_commit_rows, dim3((n + 255) / 256), dim3(256), 0, st, *s, *t, *a, rows, n);
    return hipGetLastError();
}

hipError_t pe_launch_reset_plan(pe::NodeRec* rec, const pe::NodeRec* base_rec, uint32_t* dev_free,
                                const uint32_t* dev_free_base, uint32_t n, uint8_t* preempted, uint32_t m,
                                uint32_t* pcount, uint32_t keys, hipStream_t st) {
    uint32_t w = n > m ? n : m;
    w = w > keys ? w : keys;
    uint32_t blocks = (w + 255) / 256;
    if (blocks > 1024) blocks = 1024;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_reset_plan, dim3(blocks), dim3(256), 0, st, rec, base_rec, dev_free, dev_free_base, n,
                       preempted, m, pcount, keys);
    return hipGetLastError();
}

hipError_t pe_launch_fold_feas(const pe::NodeSoA* s, const uint8_t* class_ok, const uint8_t* node_ok, uint8_t* feas,
                               hipStream_t st) {
    uint32_t blocks = (s->n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_fold_feas, dim3(blocks), dim3(256), 0, st, *s, class_ok, node_ok, feas);
    return hipGetLastError();
}

size_t pe_fold_feas_max_classes() { return pe::kFoldMaxClasses; }

hipError_t pe_launch_fold_feas_staged(const pe::NodeSoA* s, const unsigned char* class_src, uint8_t* class_dst,
                                      uint32_t ncls, const uint8_t* node_ok, uint8_t* feas, hipStream_t st) {
    if (ncls > pe::kFoldMaxClasses || !class_src || !class_dst) return hipErrorInvalidValue;
    uint32_t blocks = (s->n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_fold_feas_staged, dim3(blocks), dim3(256), 0, st, *s, class_src, class_dst, ncls,
                       node_ok, feas);
    return hipGetLastError();
}

hipError_t pe_launch_fold_aux(const pe::NodeSoA* s, const pe::TgTables* t, const uint8_t* aff_idx_class,
                              const uint8_t* aff_idx_node, uint32_t* aux, hipStream_t st) {
    uint32_t blocks = (s->n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks == 0) blocks = 1;
    hipLaunchKernelGGL(pe::k_fold_aux, dim3(blocks), dim3(256), 0, st, *s, *t, aff_idx_class, aff_idx_node, aux);
    return hipGetLastError();
}

static int sweep_variant() {
    const char* e = std::getenv("PE_SWEEP_VARIANT");
    return e ? std::atoi(e) : 0;
}

hipError_t pe_launch_sweep(const pe::SweepArgs* a, uint32_t blocks, pe::SweepRec* merged, hipStream_t st) {
    // PE_SWEEP_VARIANT selects measurement variants (tools/sweep_variants.py):
    // 1 = next-tile prefetch, 5 = streaming-only bound probe, 6 = arithmetic-only probe.
    if (a->node_aux) {
        hipLaunchKernelGGL((pe::k_sweep<256, false, 0, true>), dim3(blocks), dim3(256), 0, st, *a);
        hipLaunchKernelGGL(pe::k_sweep_merge, dim3(1), dim3(512), 0, st, (const pe::SweepRec*)a->recs, blocks, merged);
        return hipGetLastError();
    }
    switch (sweep_variant()) {
        case 1: hipLaunchKernelGGL((pe::k_sweep<256, true>), dim3(blocks), dim3(256), 0, st, *a); break;
        case 7: hipLaunchKernelGGL((pe::k_sweep<256, false, 1>), dim3(blocks), dim3(256), 0, st, *a); break;
        case 8: hipLaunchKernelGGL((pe::k_sweep<256, false, 2>), dim3(blocks), dim3(256), 0, st, *a); break;
        case 5: hipLaunchKernelGGL((pe::k_sweep_probe<256, 5>), dim3(blocks), dim3(256), 0, st, *a); break;
        case 6: hipLaunchKernelGGL((pe::k_sweep_probe<256, 6>), dim3(blocks), dim3(256), 0, st, *a); break;
        default: hipLaunchKernelGGL((pe::k_sweep<256, false>), dim3(blocks), dim3(256), 0, st, *a); break;
    }
    hipLaunchKernelGGL(pe::k_sweep_merge, dim3(1), dim3(512), 0, st, (const pe::SweepRec*)a->recs, blocks, merged);
    return hipGetLastError();
}

hipError_t pe_launch_trace_top(const uint32_t* codes, const double* sc, const pe::TraceSrc* src, uint32_t flags,
                               pe_metric_score* out, uint8_t* n_out, hipStream_t st, uint32_t n_entries,
                               uint32_t* n_other, uint2* other_list) {
    if (!src->n_rec) return hipSuccess;
    // waves per record: about 2048 entries each, 1 to kTopWaves
    const uint32_t avg = n_entries / src->n_rec;
    const uint32_t waves = std::max<uint32_t>(1u, std::min<uint32_t>(pe::kTopWaves, (avg + 2047u) / 2048u));
    hipLaunchKernelGGL(pe::k_trace_top, dim3(src->n_rec), dim3(64 * waves), 0, st, codes, sc, *src, flags, out,
                       n_out, n_other, other_list);
    return hipGetLastError();
}

// A shard's sweep merged to one record in the same launch (a->merged,
// a->done: the sharded count loop's exchange payload).
// Default: k_sweep, then k_sweep_merge into *merged (a second launch queued
// behind it); PE_SHARD_MERGE=fused: the sweep's last workgroup merges (one
// launch, but every workgroup's release at agent scope writes back its L2).
hipError_t pe_launch_sweep_local(const pe::SweepArgs* a, uint32_t blocks, hipStream_t st) {
    static const bool fused = [] {
        const char* e = std::getenv("PE_SHARD_MERGE");
        return e && std::strcmp(e, "fused") == 0;
    }();
    if (!a->merged || (fused && !a->done)) return hipErrorInvalidValue;
    if (fused) {
        if (a->node_aux) hipLaunchKernelGGL((pe::k_sweep<256, false, 0, true, true>), dim3(blocks), dim3(256), 0, st, *a);
        else hipLaunchKernelGGL((pe::k_sweep<256, false, 0, false, true>), dim3(blocks), dim3(256), 0, st, *a);
        return hipGetLastError();
    }
    if (a->node_aux) hipLaunchKernelGGL((pe::k_sweep<256, false, 0, true>), dim3(blocks), dim3(256), 0, st, *a);
    else hipLaunchKernelGGL((pe::k_sweep<256, false>), dim3(blocks), dim3(256), 0, st, *a);
    hipLaunchKernelGGL(pe::k_sweep_merge, dim3(1), dim3(512), 0, st, (const pe::SweepRec*)a->recs, blocks, a->merged);
    return hipGetLastError();
}

// Resident k_sweep<256> workgroups per CU (grid = one full wave of residency).
int pe_sweep_blocks_per_cu(bool aux) {
    int nb = 0;
    const hipError_t e = aux ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pe::k_sweep<256, false, 0, true>, 256, 0)
                             : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, pe::k_sweep<256, false>, 256, 0);
    if (e != hipSuccess || nb <= 0) nb = 4;
    return nb;
}

hipError_t pe_launch_node_record(const pe::SweepArgs* a, uint32_t row, pe_ranked_node* out, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_node_record, dim3(1), dim3(64), 0, st, *a, row, out);
    return hipGetLastError();
}

uint32_t pe_rec_winner(const pe::SweepRec* r) { return pe::rec_winner(*r); }
void pe_rec_init(pe::SweepRec* r) { pe::rec_init(*r); }
void pe_rec_merge(pe::SweepRec* a, const pe::SweepRec* b) { pe::rec_merge(*a, *b); }

hipError_t pe_launch_spread_table(const pe::TgTables* t, double* tab, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_spread_table, dim3(1), dim3(256), 0, st, *t, tab);
    return hipGetLastError();
}

void pe_rec_merge_host(pe::SweepRec* a, const pe::SweepRec* b) { pe::rec_merge(*a, *b); }
void pe_rec_init_host(pe::SweepRec* a) { pe::rec_init(*a); }

hipError_t pe_launch_trace(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                           uint32_t n, uint32_t* out, const uint32_t* penalty_bits, double log10,
                           const double* spread_tab, double* scores, hipStream_t st, const uint16_t* dks) {
    if (n == 0) return hipSuccess;
    pe::TraceSrc src{};
    src.rows = rows;
    src.dks = dks;
    hipLaunchKernelGGL(pe::k_trace, dim3((n + 255) / 256), dim3(256), 0, st, *s, *t, *a, src, n, out,
                       penalty_bits, log10, spread_tab, scores);
    return hipGetLastError();
}

// Every record of a speculative run in one launch (TraceSrc batched form).
hipError_t pe_launch_trace_batch(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a,
                                 const pe::TraceSrc* src, uint32_t n, uint32_t* out, double log10,
                                 const double* spread_tab, double* scores, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(pe::k_trace, dim3((n + 255) / 256), dim3(256), 0, st, *s, *t, *a, *src, n, out,
                       nullptr, log10, spread_tab, scores);
    return hipGetLastError();
}

// Spread boost tables of every record of a speculative run (k_spread_tables).
hipError_t pe_launch_spread_tables(const pe::TgTables* t, uint32_t n_rec, uint32_t* delta, double* tab,
                                   hipStream_t st) {
    if (n_rec == 0) return hipSuccess;
    hipLaunchKernelGGL(pe::k_spread_tables, dim3(n_rec), dim3(256), 0, st, *t, delta, tab);
    return hipGetLastError();
}

// One placement of the device-resident count loop: k_sweep (no merge) over
// `blocks` workgroups, then k_sweep_step.
hipError_t pe_launch_sweep_step(const pe::SweepArgs* a, uint32_t blocks, const uint32_t* visit, uint32_t n,
                                uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st) {
    if (a->node_aux) hipLaunchKernelGGL((pe::k_sweep<256, false, 0, true>), dim3(blocks), dim3(256), 0, st, *a);
    else hipLaunchKernelGGL((pe::k_sweep<256, false>), dim3(blocks), dim3(256), 0, st, *a);
    hipLaunchKernelGGL(pe::k_sweep_step, dim3(1), dim3(256), 0, st, *a, blocks, visit, n, offset, out, state);
    return hipGetLastError();
}

// The LDS-resident full-pass loop (one workgroup); dynamic LDS = 12 B per node.
size_t pe_fullpass_lds_bytes(uint32_t) { return (size_t)pe::kFullCap * (sizeof(double) + 2 * sizeof(uint32_t)); }

hipError_t pe_launch_fullpass_lds(const pe::SweepArgs* a_dev, int np, const uint32_t* visit, uint32_t n,
                                  uint32_t count, pe_ranked_node* out, uint32_t* state, unsigned long long* prof,
                                  hipStream_t st) {
    const size_t lds = pe_fullpass_lds_bytes(n);
    static bool attr = false;
    if (!attr) {
        for (const void* f : {reinterpret_cast<const void*>(&pe::k_fullpass_lds<0>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_lds<1>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_lds<2>)}) {
            const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     (int)pe_fullpass_lds_bytes(0));
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
    switch (np) {
        case 0:
            hipLaunchKernelGGL(pe::k_fullpass_lds<0>, dim3(1), dim3(pe::kFullThreads), lds, st, a_dev, visit, n, count,
                               out, state, prof);
            break;
        case 1:
            hipLaunchKernelGGL(pe::k_fullpass_lds<1>, dim3(1), dim3(pe::kFullThreads), lds, st, a_dev, visit, n, count,
                               out, state, prof);
            break;
        default:
            hipLaunchKernelGGL(pe::k_fullpass_lds<2>, dim3(1), dim3(pe::kFullThreads), lds, st, a_dev, visit, n, count,
                               out, state, prof);
            break;
    }
    return hipGetLastError();
}

size_t pe_fullpass_svc_bytes() { return (size_t)pe::kSvcCap * (2 * sizeof(double) + 4 * sizeof(uint32_t)); }
uint32_t pe_fullpass_svc_cap() { return pe::kSvcCap; }

hipError_t pe_launch_fullpass_svc(const pe::SweepArgs* a_dev, int np, bool lean, const uint32_t* visit, uint32_t n,
                                  uint32_t count, pe_ranked_node* out, uint32_t* state, hipStream_t st) {
    const size_t lds = pe_fullpass_svc_bytes();
    static bool attr = false;
    if (!attr) {
        for (const void* f : {reinterpret_cast<const void*>(&pe::k_fullpass_svc<0, false>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_svc<1, false>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_svc<2, false>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_svc<0, true>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_svc<1, true>),
                              reinterpret_cast<const void*>(&pe::k_fullpass_svc<2, true>)}) {
            const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        attr = true;
    }
#define PE_SVC_LAUNCH(NPV, L)                                                                                         \
    hipLaunchKernelGGL((pe::k_fullpass_svc<NPV, L>), dim3(1), dim3(pe::kFullThreads), lds, st, a_dev, visit, n, count, \
                       out, state)
    if (lean) {
        if (np == 0) PE_SVC_LAUNCH(0, true);
        else if (np == 1) PE_SVC_LAUNCH(1, true);
        else PE_SVC_LAUNCH(2, true);
    } else {
        if (np == 0) PE_SVC_LAUNCH(0, false);
        else if (np == 1) PE_SVC_LAUNCH(1, false);
        else PE_SVC_LAUNCH(2, false);
    }
#undef PE_SVC_LAUNCH
    return hipGetLastError();
}

// The sweep alone (per-workgroup records into a->recs, no merge).
hipError_t pe_launch_sweep_only(const pe::SweepArgs* a, uint32_t blocks, hipStream_t st) {
    if (a->node_aux) hipLaunchKernelGGL((pe::k_sweep<256, false, 0, true>), dim3(blocks), dim3(256), 0, st, *a);
    else hipLaunchKernelGGL((pe::k_sweep<256, false>), dim3(blocks), dim3(256), 0, st, *a);
    return hipGetLastError();
}

// The step alone (sharded loop: its records are the ranks' gathered ones).
hipError_t pe_launch_step_only(const pe::SweepArgs* a, uint32_t nrecs, const uint32_t* visit, uint32_t n,
                               uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st) {
    hipLaunchKernelGGL(pe::k_sweep_step, dim3(1), dim3(256), 0, st, *a, nrecs, visit, n, offset, out, state);
    return hipGetLastError();
}

// The persistent loop; `blocks` must all be resident (the host keeps it at
// most one workgroup per CU). state[0..4] zeroed by the caller.
hipError_t pe_launch_sweep_loop(const pe::SweepArgs* a, uint32_t blocks, uint32_t count, const uint32_t* visit,
                                uint32_t n, uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st) {
    if (a->node_aux)
        hipLaunchKernelGGL(pe::k_sweep_loop<true>, dim3(blocks), dim3(256), 0, st, *a, count, visit, n, offset, out, state);
    else
        hipLaunchKernelGGL(pe::k_sweep_loop<false>, dim3(blocks), dim3(256), 0, st, *a, count, visit, n, offset, out,
                           state);
    return hipGetLastError();
}

// Device-resident count loop over sparse options (one workgroup); dynamic LDS
// = 2 bits per position for each of the two outcome passes + 1 dependency bit,
// in what the workgroup's 160 KB leave beside the kernel's static LDS (which
// grows with the eviction width).
constexpr uint32_t kPLoopMaxN = 229376;
static size_t pe_ploop_lds_bytes(uint32_t n) { return (2u * ((n + 15u) / 16u) + (n + 31u) / 32u) * sizeof(uint32_t); }

static const void* ploop_fn(int wi) {
    return wi == 0 ? reinterpret_cast<const void*>(&pe::k_ploop<1>) : reinterpret_cast<const void*>(&pe::k_ploop<8>);
}

// The current device's LDS per workgroup (the opt-in limit where it reports
// one, else the default limit): 160 KB on gfx950.
static int lds_per_workgroup(int dev) {
    int optin = 0, dflt = 0;
    if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess) optin = 0;
    if (hipDeviceGetAttribute(&dflt, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess) dflt = 0;
    (void)hipGetLastError();
    return std::max(optin, dflt);
}

// dynamic LDS bytes the launch may use on the current device (0: none / no
// device), cached per device
static int ploop_max_dyn(int wi) {
    constexpr int kDevs = 64;
    static int v[kDevs][2];
    static bool init[kDevs][2];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kDevs) {
        (void)hipGetLastError();
        return 0;
    }
    if (!init[dev][wi]) {
        hipFuncAttributes fa;
        if (hipFuncGetAttributes(&fa, ploop_fn(wi)) != hipSuccess) {
            (void)hipGetLastError();
            return 0;
        }
        const int d = lds_per_workgroup(dev) - (int)fa.sharedSizeBytes;
        v[dev][wi] = d > 0 ? d : 0;
        init[dev][wi] = true;
    }
    return v[dev][wi];
}

uint32_t pe_ploop_max_n(uint32_t words) {
    if (words != 1u && words != 8u) return 0;   // k_ploop<1> / <8> only (pe::kPLoopMaxWords)
    const size_t d = (size_t)ploop_max_dyn(words == 1u ? 0 : 1);
    uint32_t n = (uint32_t)std::min<size_t>(kPLoopMaxN, d * 8u / 5u) & ~31u;   // 5/8 byte per position
    while (n && pe_ploop_lds_bytes(n) > d) n -= 32u;
    return n;
}

hipError_t pe_launch_ploop(const pe::PLoopArgs* a, hipStream_t st) {
    const uint32_t n = a->P.n_visit;
    if (n == 0 || n > pe_ploop_max_n(a->P.mask_words)) return hipErrorInvalidValue;
    const int wi = a->P.mask_words == 1u ? 0 : 1;
    {   // per device: the attribute is set on the current device's function
        static bool attr[64][2];
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return hipErrorInvalidDevice;
        if (!attr[dev][wi]) {
            const hipError_t e = hipFuncSetAttribute(ploop_fn(wi), hipFuncAttributeMaxDynamicSharedMemorySize,
                                                     ploop_max_dyn(wi));
            if (e != hipSuccess) return e;
            attr[dev][wi] = true;
        }
    }
    const size_t lds = pe_ploop_lds_bytes(n);
    if (wi == 0) hipLaunchKernelGGL(pe::k_ploop<1>, dim3(1), dim3(pe::kPLoopBlock), lds, st, *a);
    else hipLaunchKernelGGL(pe::k_ploop<8>, dim3(1), dim3(pe::kPLoopBlock), lds, st, *a);
    return hipGetLastError();
}

hipError_t pe_launch_static_gate(const uint8_t* blocked, const uint32_t* coll_tg, uint32_t* gate, uint32_t n,
                                 hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(pe::k_static_gate, dim3((n + 255) / 256), dim3(256), 0, st, blocked, coll_tg, gate, n);
    return hipGetLastError();
}

hipError_t pe_launch_md_gate(pe::MdNet* md, const uint32_t* coll_tg, uint32_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(pe::k_md_gate, dim3((n + 255) / 256), dim3(256), 0, st, md, coll_tg, n);
    return hipGetLastError();
}
