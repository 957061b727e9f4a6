// Shared host/device layout of the placement engine's HBM state and the
// per-launch parameter block.
#pragma once
#include <stddef.h>
#include <stdint.h>
#include "../../include/nomad_pe.h"

namespace pe {

constexpr int kMaxPsets = 16;         // spread + distinct_property sets of a task group on the device
// Per-value tables (spread boosts, use counts) are laid out set after set
// (TgTables::pset_tab_off / pset_cnt_off), so a set may hold any number of
// values. Kernels stage them in LDS while they fit kLdsPsetValues entries in
// all and read them from HBM otherwise.
constexpr int kLdsPsetValues = 2048;
constexpr uint32_t kMissing = 0xFFFFFFFFu;   // node has no value for the property
constexpr int32_t kDynPortCapacity = 32000 - 20000 + 1;   // IndexesInRange is inclusive
constexpr int kMaxSkip = 3;           // stack.go:17 maxSkip
constexpr int kPlaceBlock = 256;      // threads of the persistent count-loop workgroup
constexpr int kMaxDevReq = 4;         // device requests per task group on device
constexpr int kMaxDevGroups = 4;      // device groups per node on device (u8 free counts packed in a u32)

// Static device-match table of one ComputedClass for the task group's device
// requests (class-exact: Node.ComputeClass hashes device identity and
// attributes, node_class.go:86-101). For request q and device group g of the
// class: match bit (nodeDeviceMatches), the AssignDevice choice score
// (Σ matched affinity weights / Σ |weights|, 0 without affinities) and the
// matched weight sum.
// k_trace outcome codes (AllocMetric reasons after the FeasibilityWrapper)
enum : uint32_t {
    kTrOption = 0, kTrDistinctHosts = 1, kTrDistinctProp = 2,
    kTrNoAddr = 10, kTrDynPorts = 11, kTrNoNetworks = 12, kTrBandwidth = 13, kTrTaskDyn = 14,
    kTrStaticPort = 15,         // the reason string is rebuilt on the host (static_port_reason)
    kTrTaskStatic = 16,         // the task network's static ports (task_port_reason)
    kTrDevNone = 20, kTrDevZero = 21, kTrDevNoMatch = 22,
    kTrCpu = 30, kTrMemory = 31, kTrDisk = 32, kTrCores = 33,
    kTrMismatch = 254,          // device verdict disagrees with the host walk (bug guard)
    kTrPenalty = 1u << 16,      // option: node in the rescheduling penalty set
};

// The entries of a k_trace launch. Plain: entry i is rows[i], with dks[i]
// (or 0) placements the state lacks. Batched (rec_end set: every record of a
// speculative run, spec_metrics): entry i belongs to record k, the first with
// rec_end[k] > i, as its j-th row: rows[rsrc[k] + j] (a window walked on the
// host), or with kTraceRot set list[(rsrc[k] - kTraceRot + j) mod n_list] (a
// whole-list walk the memo no longer changes, rotated to the record's start);
// its dk counts the run's placements (row << 32 | record, sorted) on the row
// by records before k.
constexpr uint32_t kTraceRot = 0x80000000u;
struct TraceSrc {
    const uint32_t* rows;
    const uint16_t* dks;
    const uint32_t* rec_end;
    const uint32_t* rsrc;
    const uint32_t* list;
    const uint64_t* pl;
    uint32_t n_rec, n_list, n_pl;
};

struct DevClass {
    uint8_t match[kMaxDevReq];            // bit g: group g matches request q
    uint32_t n_groups;
    double choice[kMaxDevReq][kMaxDevGroups];
    double matched[kMaxDevReq][kMaxDevGroups];
};

// One node of the snapshot in HBM: a 64-byte record (one cache line, four
// 16-byte loads per lane) holding everything BinPack needs. Capacities are
// static (pe_set_state); the used_* fields and coll_job are the proposed state
// (existing allocs + plan placements) and change with every commit.
struct alignas(16) NodeRec {
    int64_t cap_cpu, cap_mem, cap_disk;      // NodeResources - ReservedResources (AllocsFit "available")
    int64_t used_cpu, used_mem, used_disk;   // Σ proposed non-terminal allocs
    uint32_t cls;                            // dense ComputedClass index
    int32_t avail_mbits;                     // bandwidth of the first host device network (-1: none)
    int32_t used_mbits;                      // bandwidth held on the host device
    int32_t used_dyn;                        // ports held in the dynamic range (incl. node-reserved)
};
static_assert(sizeof(NodeRec) == 64, "NodeRec must be one 64-byte line");

struct NodeSoA {
    uint32_t n;
    NodeRec* rec;                // [n], row order of the snapshot (job independent)
    uint32_t* coll_job;          // [n] proposed allocs of the job (distinct_hosts only)
    // reserved cores (rank.go:437-466), null when no node has core sets: per
    // node 4 x u64 masks over core ids < 256
    const uint64_t* core_rsvable;   // ReservableCpuCores
    const uint64_t* core_avail;     // ReservableCpuCores - ReservedCpuCores (AllocsFit Superset)
    uint64_t* core_used;            // Σ proposed allocs' ReservedCores
    const int64_t* core_spc;        // [n] SharesPerCore = CpuShares / TotalCpuCores
};

// A node with several host network devices, or with allocs on a device other
// than its first ("multi-device node"): NetworkIndex keeps bandwidth per device
// (UsedBandwidth / AvailBandwidth, network.go:36-43, 108-114, 196-217) and
// AssignNetwork walks the AvailNetworks in order (yieldIP, network.go:294-315,
// 407-482), which the one device of the NodeRec does not hold. The host
// (engine.cpp build_md) gives such a node's task-network outcome per task
// group: placements of the group are admitted while coll_tg + dk < lim (first
// fit over the devices, as consecutive AssignNetwork calls place them; lim is
// ~0u on other nodes), `code` is the kTr* outcome of the first refused one
// (kTrTaskStatic with the port's index in bits 8-15, kMdInvalidPort for a port
// out of range, kMdCoded), and `ev` the Preempt Select's outcome at coll_tg ==
// coll: the offer fits as is, PreemptForNetwork (preemption.go:270-455)
// preempts the listed allocs (CSR-relative indices, one byte each) and the
// retried offer fits, the node is skipped, or outside the modelled surface
// (candidates on two devices: the reference ranges over a Go map).
enum : uint8_t { kMdFit = 0, kMdPre = 1, kMdSkip = 2, kMdUnsup = 3 };
constexpr uint32_t kMdCoded = 1u << 17;         // a kTrTaskStatic code whose port index is in bits 8-15
constexpr uint32_t kMdInvalidPort = 1u << 16;   // ... and that port is out of range
struct alignas(8) MdNet {
    uint32_t lim, coll, code;
    uint8_t ev, n_pre, _pad[2];
    uint64_t pre;
};
static_assert(sizeof(MdNet) == 24, "MdNet is 24 bytes");
constexpr uint32_t kMdUnbounded = 0xFFFFFFFEu;   // MdNet::lim as built: no placement limit

// Per (job, task group) feasibility / affinity / spread tables for a Select.
// kPort* flags of TgTables.port_info
constexpr uint8_t kPortCount = 0x0F;     // holders listed
constexpr uint8_t kPortFail = 0x10;      // a needed port is held by an alloc too close in priority: nil
constexpr uint8_t kPortBlocked = 0x20;   // a needed port is blocked by what no preemption removes
constexpr uint8_t kPortUnsup = 0x40;     // one alloc holds two ports of the ask, or too many holders

struct TgTables {
    const uint8_t* class_ok;     // [ncls] memoised job+tg feasibility per class
    const uint8_t* node_ok;      // [n] or null: per-node verdict (escaped constraints)
    const uint8_t* node_feas;    // [n] or null: class_ok[cls] & node_ok folded per node
    const double* class_aff;     // [ncls] or null: normalised node-affinity score (0 = not appended)
    const double* node_aff;      // [n] or null
    const uint8_t* alias_ok;     // [n] or null: node has an address for the tg's port network
    uint32_t* coll_tg;           // [n] proposed allocs of (job, tg) per node
    const uint32_t* static_gate; // [n] or null: static port asks; 0 = a port is taken (or no address), else
                                 // coll_tg + 1 when the gate was built (a later placement of the group holds them)
    const uint32_t* task_gate;   // [n] or null: the same for the task network's static ports (AssignNetwork)
    // [n] or null: PreemptForNetwork's reserved-port step of the static ask
    // (group or task network): holders to preempt first (CSR-relative alloc
    // indices, one byte each, ask order) and kPort* flags
    const uint64_t* port_list;
    const uint8_t* port_info;
    const uint64_t* port_block;  // [n] or null: allocs holding a needed port on the ask's address (up to 8
                                 // CSR-relative indices, one byte each, 0xFF ends the list)
    const MdNet* md;             // [n] or null: the task network on multi-device nodes (host-built)
    int n_psets;                                 // spread property sets first, then distinct_property sets
    int n_spread;                                // psets [0, n_spread) score, [n_spread, n_psets) filter
    uint32_t pset_allowed[kMaxPsets];            // distinct_property: allowed use count per value
    const uint32_t* pset_val_class[kMaxPsets];   // [ncls] value index or kMissing
    const uint32_t* pset_val_node[kMaxPsets];    // [n] or null (escaped property)
    uint32_t* pset_counts[kMaxPsets];            // [nvals] combined use (existing + proposed)
    const double* pset_desired[kMaxPsets];       // [nvals] desired count, NaN = no target -> -1
    int pset_nvals[kMaxPsets];
    int pset_even[kMaxPsets];                    // no targets: evenSpreadScoreBoost
    double pset_weight_frac[kMaxPsets];          // float64(weight) / float64(sumSpreadWeights)
    // table layout: set p's boosts at spread table entries [tab_off[p], tab_off[p] + nvals + 1)
    // (one spare entry per set), its counts at [cnt_off[p], cnt_off[p] + nvals)
    uint32_t pset_tab_off[kMaxPsets], pset_cnt_off[kMaxPsets];
    uint32_t pset_tab_total, pset_cnt_total;
    // devices (only when the task group requests devices, else null)
    uint32_t* dev_free;                          // [n] free healthy instances per group, 4 x u8
    const DevClass* dev_cls;                     // [ncls]
};

struct Ask {
    int64_t cpu, mem, disk;       // AllocatedResources.Comparable() of the task group
    int32_t tg_dyn;               // tg network dynamic ports (AssignPorts)
    int32_t has_task_net;         // task-level network asks (the number of tasks with a network)
    int32_t task_mbits, task_dyn; // Σ over task networks
    int32_t commit_mbits, commit_dyn;   // NetworkIndex contribution of the placed alloc
    int32_t desired_count;        // tg.Count for job anti-affinity
    int32_t distinct_job, distinct_tg;
    int32_t algo_spread;
    int32_t anti_aff;             // JobAntiAffinityIterator present (GenericStack only)
    int32_t cores;                // Σ Resources.Cores of the tasks (cpu: the other tasks' CpuShares)
    int32_t static_dyn;           // static ports of the ask inside the dynamic range (skipped by the dynamic picks)
    int32_t n_dev;                // device requests of the task group (tasks in order)
    uint32_t dev_aff;             // bit q: request q has affinities
    int32_t dev_cnt[kMaxDevReq];  // RequestedDevice.Count
    double dev_tw;                // Σ |affinity weight| over requests with affinities (0: no score)
};

// One Select of a deferred-record k_chain launch (BatchArgs::emit).
struct ChainEmit {
    int32_t row;                  // winner, -1 = nil
    uint32_t dk;                  // placements of the launch on the row before this one
    uint32_t consumed, filtered, exhausted, new_offset;
    uint32_t pos;                 // the winner's visit position, or PE_NONE (an exhausted stream's)
    double score;                 // FinalScore
};

// Per-node count arrays rewritten by one k_counts launch (own allocs, job and
// task-group collisions); null entries are skipped.
constexpr int kMaxCountDst = 32;
struct CountDsts {
    uint32_t* d[kMaxCountDst];
};

// ResetPlan's state copy (proposed state back to the snapshot) when it rides in
// the next k_counts launch (rec null: none)
struct ResetArgs {
    NodeRec* rec;
    const NodeRec* base_rec;
    uint32_t* dev_free;
    const uint32_t* dev_free_base;
    uint32_t n;
    uint8_t* preempted;
    uint32_t m;
    uint32_t* pcount;
    uint32_t keys;
};

// SetJob's collision counts (and a deferred ResetPlan copy) as a launch
// carries them: the k_counts launch, or the fused k_chain of a short list
// (BatchArgs::counts, nd 0: none)
struct CountArgs {
    CountDsts D;
    uint32_t nd, n;
    const uint2* ents;            // sorted (row << 5 | array, count), possibly in the mapped staging ring
    uint32_t m;
    ResetArgs R;
};

// Select result as k_emit hands it to the host: the leading fields of
// pe_ranked_node (row .. new_offset, byte-identical) and the device offers;
// the host widens it (no preemptions or reserved cores on the chain path).
// It is the public pe_spec_rec (the served-Select view, nomad_pe.h).
using EmitRec = pe_spec_rec;
static_assert(sizeof(EmitRec) % 8 == 0, "record copy granule");
static_assert(offsetof(EmitRec, n_device_offers) == offsetof(pe_ranked_node, n_preempted),
              "EmitRec shares pe_ranked_node's leading fields");

// The FeasibilityWrapper verdicts folded into one byte per node (k_fold_feas_staged's
// work) carried by the next windowed-chain launch instead of a launch of its
// own: k_base (or a fused k_chain) pulls the class table from the staging ring
// into LDS, stores node_feas for every row and evaluates with the table.
struct FoldArgs {
    const uint8_t* class_src;    // class verdict table in the mapped staging ring
    uint8_t* class_dst;          // its device copy (written by one workgroup)
    uint32_t ncls;
    const uint8_t* node_ok;      // [n] or null
    uint8_t* feas;               // [n] node_feas; null: no fold carried
};

// One launch = n_evals independent evaluations (one workgroup each) of the same
// task group over the same snapshot; eval e visits perms + e*perm_stride.
struct BatchArgs {
    // FULL k_place: the per-value tables in HBM, one set per evaluation
    // (pset_tab_total doubles / pset_cnt_total counts each), when they exceed
    // the LDS budget; null: in dynamic LDS (pset_lds bytes)
    double* pset_g_tab;
    uint32_t* pset_g_cnt;
    uint32_t pset_lds;
    NodeSoA soa;
    TgTables tg;
    Ask ask;
    const uint32_t* perms;        // visit orders (SetNodes lists after shuffle)
    // single-evaluation chain: k_base reads the visit order from the staging
    // ring (perm_src, mapped) and stores it to perm_dst (= perms), or null
    const uint32_t* perm_src;
    uint32_t* perm_dst;
    uint32_t perm_stride;         // 0: all evals share one order
    uint32_t class_ok_stride;     // 0: shared class table, else per-eval tables
    const uint32_t* offsets;      // per-eval StaticIterator cursor, or null -> offset0
    uint32_t offset0;
    uint32_t n_visit;             // length of each visit list
    uint32_t limit;               // LimitIterator limit
    uint32_t count;               // placements to attempt per eval
    const uint32_t* penalty_bits; // bitmask over rows or null
    double log10;                 // go_log(10), computed on host
    int hash_bits;                // LDS overlay capacity = 1 << hash_bits (>= 2 * count)
    int net_overlay;              // overlay tracks network deltas
    int packed_overlay;           // one u32 per overlay entry: row << 8 | k (rows < 2^24, count <= 255)
    int commit;                 // apply Plan.AppendAlloc after each placement
    int writeback;                // merge the overlay into the HBM SoA at the end
    // Phase-static windowed loop (k_chain): base[row] = the row's pipeline
    // result with no placement of this launch on it (finite FinalScore, -inf
    // filtered, +inf exhausted), computed once per launch by k_base for all
    // evaluations. Null: the lazy per-position loop (k_window).
    double* base;
    // base_by_pos: one evaluation; base[j] is the value of visit position j
    // (k_base walks the visit list, k_chain then reads the window coalesced)
    int base_by_pos;
    // base1 (or null): the same with one placement of this launch on the row
    // (a row's value in the phase after its first placement)
    double* base1;
    // Single-evaluation k_chain with deferred records (or null): k_chain writes
    // one ChainEmit per Select and dumps its overlay (row, placements) into
    // emit_ov; k_emit builds the full records and writes the placements back.
    // emit_n: [0] entries, [1] overlay rows to write back.
    ChainEmit* emit;
    uint2* emit_ov;
    uint32_t* emit_n;
    uint32_t* done_flag;          // or null: k_emit's workgroup b stores done_seq to done_flag[b] (system scope)
    uint32_t done_seq;
    unsigned long long* prof;     // k_chain step clocks (PE_CHAIN_PROF), or null
    // FUSED k_chain (or null): the score parts of every position's first-phase
    // evaluation (PE_MAX_SCORES doubles and a count per visit position); a
    // record whose row held no placement of the launch copies them instead of
    // evaluating the row again
    double* fused_parts;
    uint8_t* fused_nparts;
    // k_chain scratch, kChainMaxN doubles per workgroup: the window's values
    // by relative position (one thread per Select walks its own positions)
    double* chain_vs;
    FoldArgs fold;                // a fold carried by this launch (fold.feas null: none)
    CountArgs counts;             // SetJob's counts carried by a fused k_chain (counts.nd 0: none)
    // Short lists, one evaluation: k_chain alone (no k_base / k_emit /
    // k_emit_writeback launches) evaluates the first phase's positions itself,
    // builds the records, writes the placements back and raises done_flag[0]
    int fused;
    pe_ranked_node* full_out;     // [n_evals][count] full records, or null
    EmitRec* emit_out;            // k_emit's records (single-evaluation chain), or null
    pe_placement* out;            // [n_evals][count] compact records, or null
    uint32_t* eval_status;        // [n_evals][2]: placed, final cursor
};

// Full-scan Select reduction record (one per workgroup, and per GPU shard).
// With limit >= options the LimitIterator returns every option, the first
// kMaxSkip non-positive ones (in visit order) moved to the end; MaxScore then
// takes the first strict maximum. The record keeps
// exactly what that rule needs and merges associatively.
struct SweepRec {
    double max_score;            // -inf: no option
    uint32_t max_rank[4];        // earliest visit ranks scoring max_score (sorted, ~0u = empty)
    uint32_t np_rank[kMaxSkip];  // earliest non-positive options (sorted by rank)
    uint32_t options, filtered, exhausted, _pad;
    double np_score[kMaxSkip];
};

static_assert(sizeof(SweepRec) == sizeof(pe_shard_rec), "pe_shard_rec carries one SweepRec");

struct SweepArgs {
    NodeSoA soa;
    TgTables tg;
    Ask ask;
    const uint32_t* rank_of;      // [n rows] visit position of the row, ~0u = not in the list
    uint32_t n_visit;
    uint32_t offset;              // StaticIterator cursor: rank = (pos - offset) mod n_visit
    uint32_t row_begin, row_end;  // rows this launch (shard) sweeps
    const uint32_t* penalty_bits;
    double log10;
    const double* spread_tab;     // [kMaxPsets][kMaxValues+1] or null
    // Folded per-node score inputs (k_fold_aux), or null: bit 31 the
    // FeasibilityWrapper verdict, bits 0-7 an index into aff_vals (the node's
    // NodeAffinityIterator score), bits 8+8p the node's value of spread
    // property p (kAuxMissing = no value), for at most kAuxPsets properties.
    const uint32_t* node_aux;     // [n rows]
    const double* aff_vals;       // [kAuxValues]
    SweepRec* recs;               // [gridDim.x]
    // k_sweep<..., MERGE>: the last workgroup to finish merges the grid's
    // records into *merged (one record per shard); done counts finished
    // workgroups and is left at 0
    SweepRec* merged;
    uint32_t* done;
};
constexpr int kAuxPsets = 2;
constexpr int kAuxValues = 256;
constexpr uint32_t kAuxMissing = 255;

// ---- preemption (BinPack with eviction, scheduler/preemption.go) -------------
constexpr int kMaxNodeAllocs = 32;    // allocs of one node staged in LDS by k_ploop (the narrow width)
constexpr int kMaxProposed = 64;      // ProposedAllocs list length (state allocs + plan placements)

// A non-terminal state alloc as the Preemptor sees it (Allocation.ComparableResources,
// structs.go:9656-9688; Job.Priority; TaskGroup.Migrate.MaxParallel).
struct PreemptAlloc {
    int64_t cpu, mem, disk;
    int32_t priority, max_parallel;
    uint32_t job_key;        // dense (job id, namespace)
    uint32_t jtg_key;        // dense (job id, namespace, task group): plan preemption counter
    int32_t mbits, dyn;      // NetworkIndex contribution (released on eviction)
    uint32_t dev_g, dev_c;   // device entries: group / instances, one byte each
    uint32_t n_dev;          // device entries (<= 4)
    uint32_t state_index;    // row of the pe_alloc_table snapshot; bit 31 kAllocHasNet
};
constexpr uint32_t kAllocHasNet = 1u << 31;   // Flattened.Networks non-empty (PreemptForNetwork)
constexpr uint32_t kPlacedSlots = 64;          // SystemArgs.placed: counters the host sums
static_assert(sizeof(PreemptAlloc) == 64, "PreemptAlloc is one 64-byte line");

struct PreemptArgs {
    NodeSoA soa;
    TgTables tg;
    Ask ask;
    const uint32_t* node_alloc_off;   // [n + 1] CSR over rows: non-terminal state allocs in table order
    const PreemptAlloc* allocs;       // [m]
    const uint8_t* preempted;         // [m] Plan.NodePreemptions membership
    const uint32_t* pcount;           // [keys] plan preemptions per (job, namespace, task group)
    const uint32_t* own_existing;     // [n] non-terminal state allocs of the job being placed
    uint32_t job_key;                 // (job, namespace) of the job being placed
    int32_t job_priority;
    const uint32_t* visit;            // visit list (rows)
    uint32_t n_visit;
    const uint32_t* penalty_bits;
    double log10;
    const double* spread_tab;
    int32_t score_preemption;         // PreemptionScoringIterator in the chain (GenericStack only)
    // per visit position
    uint8_t* status;                  // kOption / kFiltered / kExhausted / kSkipped
    double* score;
    uint32_t* mask_out;               // or null: preempted allocs (mask_words words of bits over the node's allocs)
    uint32_t* offers_out;             // or null: device offers, one byte per request
    uint32_t* flags;                  // [1] bit 0: a node outside the modelled surface; bit 1: a node wider
                                      // than mask_words (rerun wider)
    uint8_t* dep_out;                 // or null: per position, the outcome read the plan's preemption counts
    const uint64_t* palloc_cores;     // [m x 4] or null: reserved cores held by each alloc (by CSR slot)
    // or null: per position the option's score parts (PE_MAX_SCORES each) and
    // their count, kept with mask_out / offers_out so the loop's winner record
    // is read instead of re-evaluated (k_ploop)
    double* parts_out;
    uint8_t* nparts_out;
    // eviction width (evict.inc): preempted sets are mask_words x 32 bits over a
    // node's allocs; the launch evaluates nodes of up to 32 x mask_words allocs
    // and ProposedAllocs lists of up to 64 x mask_words (kEvictWidths)
    uint32_t mask_words;
};
constexpr uint32_t kEvictWidths[3] = {1u, 8u, 32u};   // instantiated widths, narrowest first
constexpr uint32_t kEvictMaxWords = 32u;
constexpr uint32_t kPLoopMaxWords = 8u;               // k_ploop's widest (its lists live in LDS)
constexpr uint32_t kEvictUnsup = 1u;   // PreemptArgs::flags: a node outside what the device path models
constexpr uint32_t kEvictWider = 2u;   // a node's alloc list exceeds the launch's eviction width
constexpr uint32_t kEvictMaxAllocs = 32u * kEvictMaxWords;   // node allocs the widest launch evaluates

// LimitIterator + MaxScoreIterator over per-position results.
struct EvictResolveArgs {
    const uint8_t* status;
    const double* score;
    uint32_t n, offset, limit;
    int32_t* out;                     // [0] winner position (relative) or -1, [1] consumed, [2] filtered, [3] exhausted
};

// Device-resident count loop over sparse options (k_ploop): the plain Select
// and its Preempt retry of every placement resolved in one workgroup from
// per-position outcomes kept in LDS; only committed rows are re-evaluated.
struct PLoopArgs {
    PreemptArgs P;                    // P.status / P.score: evict outcomes by position (k_evict, refreshed lazily)
    const uint8_t* st_plain;          // [n] plain outcomes by position (k_census)
    const uint8_t* dep_init;          // [n] or null: Preempt outcomes that read the preemption counts (k_evict)
    double* sc_plain;                 // [n] plain scores by position (rewritten for committed rows)
    double* parts_plain;              // [n * PE_MAX_SCORES] their score parts, [n] their count (options only):
    uint8_t* nparts_plain;            // a plain winner's record is read, not re-evaluated
    uint8_t* preempted;               // Plan.NodePreemptions flags (apply_preempt)
    uint32_t* pcount;
    uint32_t* dev_free;
    uint32_t offset, limit, count;
    int32_t retry;                    // selectNextOption: a nil plain Select retries with Preempt
    int32_t check_dead;               // PE_PLOOP_CHECK_DEAD: run the plain resolves the loop skips as provably
                                      // failing anyway and stop with error 3 if one finds a winner
    pe_ranked_node* out;              // [count] records (a nil record ends the loop)
    uint32_t* out_mask;               // [count] preempted allocs of each placement (bits over the node's allocs)
    // [4 * count] or null: per placement whose plain Select came back nil
    // (the Preempt retry then answered it), that nil Select's nodes
    // evaluated / filtered / exhausted and cursor; untouched otherwise
    uint32_t* nil_out;
    uint32_t* state;                  // [0] placements, [1] cursor, [2] error (1: node outside the device limits,
                                      // 2: winner not an option, 3: a skipped plain resolve had a winner), [3] records
    unsigned long long* prof;         // [24] or null (PE_PLACE_PROF): wall-clock ticks of the plain resolve, refresh,
                                      // Preempt resolve, winner; refreshed dirty rows, refreshed pcount readers
                                      // ([6..15] winner record, commit, probes, resolve steps, plain re-evaluation;
                                      // [17..21] the winner section's parts)
};

struct SystemArgs {
    NodeSoA soa;
    TgTables tg;
    Ask ask;
    const uint32_t* list;         // SetNodes list (diff.place order)
    uint32_t n_list;
    double log10;
    double* out_score;            // [n_list]
    uint8_t* out_status;          // [n_list] 0 placed 1 filtered 2 exhausted
    uint32_t* placed;             // [1] atomic counter
    int commit;                   // Plan.AppendAlloc of the options in the kernel (0: the caller commits)
    // Row-order form (a list that covers a large part of the snapshot): the
    // kernel walks rows 0..n_rows-1 (coalesced NodeRec / count / verdict
    // accesses; the list's rows found through rank_of) and stores each
    // outcome at the row's list position, or with n_list == 0 into res[row]
    // (the FinalScore, or a NaN whose payload is the outcome).
    const uint32_t* rank_of;      // [n_rows] list position of each row, or PE_NONE; null: list-order kernel
    uint64_t* res;                // [n_rows]
    uint32_t n_rows;
};

}  // namespace pe
