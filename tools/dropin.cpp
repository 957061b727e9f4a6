// Caller-side harness (bench / tests only, not the product): the loop the
// unchanged Go caller runs against a Stack, written in C so the measured time
// is the C ABI's and not an interpreter's. GenericScheduler.computePlacements
// (generic_sched.go:472-652) per evaluation: SetNodes once, then per placement
// Select with empty options, on nil a retry with Preempt=true when preemption
// is enabled (selectNextOption, :773-792), and on an option the plan append
// the cgo shim mirrors with Commit (AppendAlloc :627 + handlePreemptions
// :794-816). A nil after the retry ends the task group (failedTGAllocs,
// :519-523). Evaluations start from a fresh EvalContext (ResetPlan) and SetJob.
//
// The same loop drives the engine (pe_*) and the CPU oracle (oracle_*): the
// caller passes the entry points. With the engine's served-Select view
// (pe_spec_view_get, nomad_pe.h) the loop answers Select / Commit pairs (the
// Preempt retry included) from the view and calls C only when it deviates,
// as the Go shim does; a
// record with more than PE_MAX_PREEMPT preempted allocs is read in full with
// preempted_of before its Commit.
#include <chrono>
#include <cstdint>
#include <cstring>

#include "../include/nomad_pe.h"

extern "C" {

// Wall time per phase over every dropin_evals call since the last reset:
// reset_plan, set_job, set_nodes, the first Select of an evaluation, the rest
// of the Select/Commit loop.
static double g_phase[5];

void dropin_phase_seconds(double* out5, int reset) {
    for (int i = 0; i < 5; i++) {
        out5[i] = g_phase[i];
        if (reset) g_phase[i] = 0.0;
    }
}

struct dropin_api {
    int (*reset_plan)(void*);
    int (*set_job)(void*, const pe_strtab*, const pe_job*);
    int (*set_nodes)(void*, const uint32_t*, uint32_t, uint32_t*);
    int (*select)(void*, uint32_t, const pe_select_options*, pe_ranked_node*);
    int (*commit)(void*, uint32_t, int32_t);
    int (*commit_preempt)(void*, uint32_t, int32_t, const uint32_t*, uint32_t);
    int (*preempted_of)(const void*, uint32_t, uint32_t*, uint32_t);
    pe_spec_view* (*spec_view_get)(void*);   // null: every Select and Commit crosses
    pe_system_view* (*system_view_get)(void*);   // null: every per-node triple crosses
    int64_t (*last_metrics)(const void*, char*, size_t);   // AllocMetric text of the last Select (oracle)
    int (*last_metrics_bin)(const void*, const pe_metric_count**, uint32_t*, const pe_metric_score**,
                            uint32_t*);   // the engine's binary maps (null: the text)
};

// With metrics on, every Select's AllocMetric maps are copied out as the shim
// fills Allocation.Metrics (generic_sched.go:558, 587): the served record's
// binary maps from the view, else through last_metrics_bin (engine) or the
// text of last_metrics (oracle).
static int g_metrics = 0;
void dropin_use_metrics(int on) { g_metrics = on; }
static uint64_t g_metric_bytes = 0;
uint64_t dropin_metric_bytes(int reset) {
    const uint64_t x = g_metric_bytes;
    if (reset) g_metric_bytes = 0;
    return x;
}
static char g_mbuf[1 << 16];
static void copy_bin(const pe_metric_count* c, uint32_t nc, const pe_metric_score* sc, uint32_t ns) {
    size_t a = (size_t)nc * sizeof(*c), b = (size_t)ns * sizeof(*sc);
    if (a > sizeof(g_mbuf)) a = sizeof(g_mbuf);
    if (b > sizeof(g_mbuf) - a) b = sizeof(g_mbuf) - a;
    std::memcpy(g_mbuf, c, a);
    std::memcpy(g_mbuf + a, sc, b);
    g_metric_bytes += (uint64_t)nc * sizeof(*c) + (uint64_t)ns * sizeof(*sc);
}
static void metrics_from_view(const pe_spec_view* v, uint32_t k) {
    if (!g_metrics || !v->mcounts) return;
    const uint32_t a = v->mcounts_off[k], b = v->mscores_off[k];
    copy_bin(v->mcounts + a, v->mcounts_off[k + 1] - a, v->mscores + b, v->mscores_off[k + 1] - b);
}
static int metrics_from_c(const dropin_api* api, void* h) {
    if (!g_metrics) return 0;
    if (api->last_metrics_bin) {
        const pe_metric_count* c;
        const pe_metric_score* sc;
        uint32_t nc, ns;
        const int rc = api->last_metrics_bin(h, &c, &nc, &sc, &ns);
        if (rc) return rc;
        copy_bin(c, nc, sc, ns);
        return 0;
    }
    if (!api->last_metrics) return 0;
    const int64_t n = api->last_metrics(h, g_mbuf, sizeof(g_mbuf));
    if (n < 0) return (int)n;
    g_metric_bytes += (uint64_t)n;
    return 0;
}

static int g_use_view = 1;
void dropin_use_view(int on) { g_use_view = on; }
static uint64_t g_view_served = 0;   // Selects answered from the view since the last read
uint64_t dropin_view_served(int reset) {
    const uint64_t x = g_view_served;
    if (reset) g_view_served = 0;
    return x;
}

// Commit of a Select's option, with its whole PreemptedAllocs list.
static int commit_opt(const dropin_api* api, void* h, uint32_t tg, const pe_ranked_node& opt, uint32_t rec) {
    if (!opt.n_preempted) return api->commit(h, tg, opt.row);
    if (opt.n_preempted <= PE_MAX_PREEMPT) return api->commit_preempt(h, tg, opt.row, opt.preempted, opt.n_preempted);
    uint32_t buf[1024];
    if (opt.n_preempted > 1024 || !api->preempted_of) return PE_EUNSUPPORTED;
    const int n = api->preempted_of(h, rec, buf, opt.n_preempted);
    if (n != (int)opt.n_preempted) return n < 0 ? n : PE_ESTATE;
    return api->commit_preempt(h, tg, opt.row, buf, opt.n_preempted);
}

// Whether the next Select (plain, or the Preempt retry with `flag` =
// PE_SPEC_PREEMPT) is answered by the view (nomad_pe.h's rules).
static bool view_can(const pe_spec_view* v, uint32_t tg, uint32_t flag) {
    return v && v->n_rec && v->tg_index == tg && v->served == v->confirmed && v->served < v->n_rec &&
           (v->recs[v->served].flags & PE_SPEC_PREEMPT) == flag;
}

// One evaluation's placements of task group `tg`; rows[count] (may be null)
// receives the chosen rows, -1 after the loop stopped. Returns 0 or the first
// failing call's status.
int dropin_place(const dropin_api* api, void* h, uint32_t tg, uint32_t count, int preempt, int32_t* rows,
                 uint32_t* placed, uint64_t* selects) {
    pe_select_options none;
    std::memset(&none, 0, sizeof(none));
    pe_select_options pre = none;
    pre.preempt = 1;
    pe_ranked_node opt;
    uint32_t p = 0;
    uint64_t sel = 0;
    int rc = 0;
    using clk = std::chrono::steady_clock;
    auto t_first = clk::now();
    auto first_done = [&](uint32_t i) {
        if (i != 0) return;
        const auto t = clk::now();
        g_phase[3] += std::chrono::duration<double>(t - t_first).count();
        t_first = t;
    };
    pe_spec_view* v = (g_use_view && api->spec_view_get) ? api->spec_view_get(h) : nullptr;
    for (uint32_t i = 0; i < count; i++) {
        if (view_can(v, tg, 0)) {
            // a plain Select answered from the view; an option's Commit is
            // confirmed there, a nil is settled at once
            metrics_from_view(v, v->served);
            const pe_spec_rec& r = v->recs[v->served++];
            v->confirmed++;
            sel++;
            g_view_served++;
            first_done(i);
            if (r.row >= 0) {
                if (rows) rows[p] = r.row;
                p++;
                continue;
            }
            opt.row = -1;
        } else {
            rc = api->select(h, tg, &none, &opt);
            sel++;
            first_done(i);
            if (!rc) rc = metrics_from_c(api, h);
            if (rc) break;
        }
        if (opt.row < 0 && preempt) {
            if (view_can(v, tg, PE_SPEC_PREEMPT)) {
                // the Preempt retry from the view; its CommitPreempt names the
                // record's row and PreemptedAllocs, confirmed there
                metrics_from_view(v, v->served);
                const pe_spec_rec& r = v->recs[v->served++];
                v->confirmed++;
                sel++;
                g_view_served++;
                if (r.row < 0) break;
                if (rows) rows[p] = r.row;
                p++;
                continue;
            }
            rc = api->select(h, tg, &pre, &opt);
            sel++;
            if (!rc) rc = metrics_from_c(api, h);
            if (rc) break;
        }
        if (opt.row < 0) break;
        rc = commit_opt(api, h, tg, opt, 0);
        if (rc) break;
        if (rows) rows[p] = opt.row;
        p++;
    }
    g_phase[4] += std::chrono::duration<double>(clk::now() - t_first).count();
    for (uint32_t i = p; rows && i < count; i++) rows[i] = -1;
    *placed = p;
    if (selects) *selects += sel;
    return rc;
}

// Sequential evaluations, one visit order each (orders[e * n ...]), cycling
// through n_orders orders, until n_evals are done or max_seconds have passed
// (0: no time limit). out[0] placements, out[1] evaluations, out[2] Selects;
// *seconds the wall time of the loop. rows_last[count] gets the last
// evaluation's rows (may be null).
int dropin_evals(const dropin_api* api, void* h, const pe_strtab* strs, const pe_job* job, const uint32_t* orders,
                 uint32_t n_orders, uint32_t n, uint32_t tg, uint32_t count, int preempt, uint32_t n_evals,
                 double max_seconds, int32_t* rows_last, uint64_t* out, double* seconds) {
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    uint64_t placed_total = 0, evals = 0, selects = 0;
    int rc = 0;
    for (uint32_t e = 0; e < n_evals; e++) {
        auto ta = clk::now();
        rc = api->reset_plan(h);
        if (rc) break;
        auto tb = clk::now();
        g_phase[0] += std::chrono::duration<double>(tb - ta).count();
        rc = api->set_job(h, strs, job);
        if (rc) break;
        ta = clk::now();
        g_phase[1] += std::chrono::duration<double>(ta - tb).count();
        uint32_t limit = 0;
        rc = api->set_nodes(h, orders + (size_t)(e % n_orders) * n, n, &limit);
        if (rc) break;
        g_phase[2] += std::chrono::duration<double>(clk::now() - ta).count();
        uint32_t p = 0;
        rc = dropin_place(api, h, tg, count, preempt, rows_last, &p, &selects);
        if (rc) break;
        placed_total += p;
        evals++;
        if (max_seconds > 0 && std::chrono::duration<double>(clk::now() - t0).count() >= max_seconds) break;
    }
    *seconds = std::chrono::duration<double>(clk::now() - t0).count();
    out[0] = placed_total;
    out[1] = evals;
    out[2] = selects;
    return rc;
}

// SystemScheduler.computePlacements (scheduler_system.go:283-425) for one task
// group: for every node of `rows`, SetNodes([node]) then Select with empty
// options (BinPack evicts inside the Select when preemption is enabled); an
// option is appended to the plan (Commit, with its preempted allocs). Per node
// out: status 0 placed / 1 filtered / 2 exhausted, score (FinalScore or NaN).
// With the engine's served system-Select view (pe_system_view_get) the triple
// of a node the view covers is answered from host memory and logged, as the Go
// shim does; the others cross.
// `flush` (may be null) is called once at the end, inside the timed region:
// the entry point that forces queued device work (e.g. the next call that
// reads the device state). Returns 0 or the first failing status.
// Wall time of dropin_system's parts since the last reset: [0] the triples that
// crossed into C, [1] the whole loop (crossings included), [2] the final flush.
static double g_sys_phase[3];
void dropin_system_phases(double* out3, int reset) {
    for (int i = 0; i < 3; i++) {
        out3[i] = g_sys_phase[i];
        if (reset) g_sys_phase[i] = 0.0;
    }
}

int dropin_system(const dropin_api* api, void* h, uint32_t tg, const uint32_t* rows, uint32_t n, uint8_t* status,
                  double* score, uint32_t* placed, int (*flush)(void*), double* seconds) {
    pe_select_options none;
    std::memset(&none, 0, sizeof(none));
    pe_ranked_node opt;
    uint32_t p = 0;
    int rc = 0;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    pe_system_view* v = (g_use_view && api->system_view_get) ? api->system_view_get(h) : nullptr;
    // The shim's fast path keeps the view's fields in locals while it answers
    // from host memory, and writes its log count back before any C call (the
    // engine reads it there) and at the end.
    uint32_t n_rows = 0, log_cap = 0, n_log = 0, pre = 0;
    uint64_t* outcome = nullptr;
    uint32_t* log = nullptr;
    const uint32_t *mkey = nullptr, *mclass = nullptr, *mnc = nullptr;
    uint8_t* mfailed = nullptr;
    const double* mscore = nullptr;
    uint32_t m_inel = 0;
    auto load_view = [&]() {
        if (!v) return;
        n_rows = (v->tg_index == tg) ? v->n_rows : 0u;
        log_cap = v->log_cap;
        n_log = v->n_log;
        pre = v->preempt;
        outcome = v->outcome;
        log = v->log;
        mkey = v->mkey;
        mclass = v->mclass;
        mfailed = v->mfailed;
        mscore = v->mscore;
        mnc = v->mnode_class;
        m_inel = v->mkey_ineligible;
    };
    // With metrics on, a served Select's maps as the shim assembles them from
    // the view's per-row entries (nomad_pe.h pe_system_view)
    auto view_maps = [&](uint32_t row, uint32_t code, double sc) {
        if (!g_metrics || !mkey) return;
        pe_metric_count c[2];
        pe_metric_score m;
        uint32_t nc = 0, ns = 0;
        const uint32_t cls = mnc[row];
        if (code == 0) {
            std::memset(&m, 0, sizeof(m));
            m.row = (int32_t)row;
            m.n_scores = 1;
            m.norm = sc;
            m.scorer[0] = PE_SCORER_BINPACK;
            m.score[0] = mscore[row];
            ns = 1;
        } else if (code == 1) {
            uint32_t key = mkey[row];
            const uint32_t mc = mclass[row];
            if (mc != PE_NONE) {
                if (mfailed[mc]) key = m_inel;
                mfailed[mc] = 1;
            }
            if (cls != PE_NONE) c[nc++] = pe_metric_count{PE_METRIC_CLASS_FILTERED, cls, 1};
            c[nc++] = pe_metric_count{PE_METRIC_CONSTRAINT_FILTERED, key, 1};
        } else {
            if (cls != PE_NONE) c[nc++] = pe_metric_count{PE_METRIC_CLASS_EXHAUSTED, cls, 1};
            c[nc++] = pe_metric_count{PE_METRIC_DIMENSION_EXHAUSTED, mkey[row], 1};
        }
        copy_bin(c, nc, &m, ns);
    };
    load_view();
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t row = rows[i];
        if (row < n_rows && n_log < log_cap) {
            const uint64_t bits = outcome[row];
            const bool nan = (bits & 0x7FF8000000000000ull) == 0x7FF8000000000000ull;
            const uint32_t code = nan ? (uint32_t)(bits & 3u) : 0u;
            if (code != 3u && !(code == 2u && pre) && (!g_metrics || mkey)) {
                if (code) {   // nil: filtered or exhausted
                    view_maps(row, code, 0.0);
                    log[n_log++] = row | PE_SYS_NIL;
                    status[i] = (uint8_t)code;
                    score[i] = __builtin_nan("");
                } else {      // an option, appended to the plan
                    double sc;
                    std::memcpy(&sc, &bits, sizeof(sc));
                    view_maps(row, 0u, sc);
                    log[n_log++] = row | PE_SYS_COMMITTED;
                    outcome[row] = PE_SYS_STALE;
                    status[i] = 0;
                    score[i] = sc;
                    p++;
                }
                g_view_served++;
                continue;
            }
        }
        if (v) v->n_log = n_log;   // the engine takes the log over first
        const auto tc = clk::now();
        uint32_t limit;
        rc = api->set_nodes(h, rows + i, 1, &limit);
        if (!rc) rc = api->select(h, tg, &none, &opt);
        if (!rc) rc = metrics_from_c(api, h);   // Allocation.Metrics (scheduler_system.go:334-337)
        if (!rc && opt.row >= 0) rc = commit_opt(api, h, tg, opt, 0);
        load_view();   // the crossing may have replaced or withdrawn the view
        g_sys_phase[0] += std::chrono::duration<double>(clk::now() - tc).count();
        if (rc) break;
        if (opt.row < 0) {
            status[i] = opt.nodes_filtered > 0 ? 1 : 2;
            score[i] = __builtin_nan("");
            continue;
        }
        status[i] = 0;
        score[i] = opt.final_score;
        p++;
    }
    if (v) v->n_log = n_log;
    const auto tf = clk::now();
    if (!rc && flush) rc = flush(h);
    const auto te = clk::now();
    g_sys_phase[2] += std::chrono::duration<double>(te - tf).count();
    *seconds = std::chrono::duration<double>(te - t0).count();
    g_sys_phase[1] += *seconds - std::chrono::duration<double>(te - tf).count();
    *placed = p;
    return rc;
}

}  // extern "C"
