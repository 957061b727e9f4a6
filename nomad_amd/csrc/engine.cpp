// Host side of the MI355X placement engine: the C ABI of include/nomad_pe.h.
//
// Responsibilities (everything that is string work or per-eval setup):
//  - pe_set_state: intern the snapshot, build the node SoA (row order) and
//    upload it to HBM; base proposed usage from the non-terminal allocs.
//  - pe_set_job:   parse the job, compute the task groups' resource asks
//    (AllocatedResources.Comparable, structs.go:3445-3487), collision counts
//    and spread use counts from the snapshot's allocs.
//  - per Select:   pre-resolve constraints / drivers / volumes / networks per
//    ComputedClass with the EvalEligibility memo emulated exactly (first node
//    of a class in visit order decides, context.go:293-345, feasible.go:1061),
//    node affinity per class, spread property values per class; upload the
//    tables and launch the fused kernel (kernels.hip).
// Nothing here evaluates a node's ranking on the CPU: feasibility of resources,
// scoring and selection all run on the device.
#include <hip/hip_runtime.h>

#include <array>
#include <charconv>
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include <dlfcn.h>
#include <mutex>
#include <rccl/rccl.h>

#include "../../include/nomad_pe.h"
#include "constraint_eval.h"
#include "engine_types.h"
#include "gomath_dev.h"
#include "gosort.h"

// ---- RCCL, bound at run time ------------------------------------------------
// The engine's collectives (pe_comm_init / pe_place_sharded, the one-handle
// multi-GPU split) call the RCCL the process already has mapped when there is
// one: a Python caller that imported torch has torch's librccl (soname
// librccl.so.1) loaded, and a second copy from /opt/rocm would give the process
// two RCCL instances with separate proxies and shared-memory state. Otherwise
// /opt/rocm's library is loaded. pe_comm_library() names the one in use.
namespace {
struct RcclApi {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGetVersion) GetVersion = nullptr;
    std::string path;     // the library in use, with its version
    std::string error;    // why it was refused
    bool ok = false;
};

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);   // matches a loaded library by soname
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
#define PE_RCCL_SYM(x) api.x = reinterpret_cast<decltype(api.x)>(dlsym(h, "nccl" #x))
        PE_RCCL_SYM(GetUniqueId);
        PE_RCCL_SYM(CommInitRank);
        PE_RCCL_SYM(CommInitAll);
        PE_RCCL_SYM(AllGather);
        PE_RCCL_SYM(CommDestroy);
        PE_RCCL_SYM(GroupStart);
        PE_RCCL_SYM(GroupEnd);
        PE_RCCL_SYM(GetErrorString);
        PE_RCCL_SYM(GetVersion);
#undef PE_RCCL_SYM
        api.ok = api.GetUniqueId && api.CommInitRank && api.CommInitAll && api.AllGather && api.CommDestroy &&
                 api.GroupStart && api.GroupEnd && api.GetErrorString && api.GetVersion;
        Dl_info info;
        if (api.GetUniqueId && dladdr(reinterpret_cast<void*>(api.GetUniqueId), &info) && info.dli_fname)
            api.path = info.dli_fname;
        // The engine is compiled against /opt/rocm's rccl.h: the enums, the
        // 128-byte ncclUniqueId and the calls it uses are fixed within a major
        // version (the torch-bundled copy is usually a minor version apart).
        // Another major version is refused, and the version is reported.
        int ver = 0;
        if (api.ok && api.GetVersion(&ver) != ncclSuccess) ver = 0;
        const int major = ver >= 10000 ? ver / 10000 : ver / 1000;
        const int minor = ver >= 10000 ? (ver / 100) % 100 : (ver / 100) % 10;
        if (api.ok && major != NCCL_MAJOR) {
            api.ok = false;
            api.error = "RCCL " + std::to_string(major) + "." + std::to_string(minor) + " at " + api.path +
                        ": the engine is built against RCCL " + std::to_string(NCCL_MAJOR) + "." +
                        std::to_string(NCCL_MINOR);
        } else if (!api.ok) {
            api.error = "RCCL library unavailable (dlopen librccl.so.1 failed or a symbol is missing)";
        }
        if (ver) api.path += " (RCCL " + std::to_string(major) + "." + std::to_string(minor) + "." + std::to_string(ver % 100) + ")";
    });
    return api;
}

ncclResult_t rc_GetUniqueId(ncclUniqueId* id) {
    return rccl().ok ? rccl().GetUniqueId(id) : ncclSystemError;
}
ncclResult_t rc_CommInitRank(ncclComm_t* c, int n, ncclUniqueId id, int rank) {
    return rccl().ok ? rccl().CommInitRank(c, n, id, rank) : ncclSystemError;
}
ncclResult_t rc_CommInitAll(ncclComm_t* c, int n, const int* devs) {
    return rccl().ok ? rccl().CommInitAll(c, n, devs) : ncclSystemError;
}
ncclResult_t rc_AllGather(const void* src, void* dst, size_t count, ncclDataType_t t, ncclComm_t c,
                          hipStream_t st) {
    return rccl().ok ? rccl().AllGather(src, dst, count, t, c, st) : ncclSystemError;
}
ncclResult_t rc_CommDestroy(ncclComm_t c) { return rccl().ok ? rccl().CommDestroy(c) : ncclSystemError; }
ncclResult_t rc_GroupStart() { return rccl().ok ? rccl().GroupStart() : ncclSystemError; }
ncclResult_t rc_GroupEnd() { return rccl().ok ? rccl().GroupEnd() : ncclSystemError; }
const char* rc_GetErrorString(ncclResult_t r) {
    return rccl().ok ? rccl().GetErrorString(r) : rccl().error.c_str();
}
}  // namespace

size_t pe_place_lds_bytes(bool full, int hash_bits, bool packed, size_t pset_bytes);
hipError_t pe_launch_place(const pe::BatchArgs* a, uint32_t n_evals, bool full, hipStream_t st);
hipError_t pe_launch_system(const pe::SystemArgs* a, hipStream_t st);
hipError_t pe_launch_rank_of(const uint32_t* list, uint32_t n_list, uint32_t* rank_of, uint32_t n_rows, hipStream_t st);
hipError_t pe_launch_upload(void* dst, const void* src_mapped, size_t bytes, hipStream_t st);
hipError_t pe_launch_scatter_rows(void* dst, uint32_t words, const void* payload_mapped, uint32_t n, hipStream_t st);
hipError_t pe_launch_counts(const pe::CountDsts* d, uint32_t nd, uint32_t n, const uint2* ents, uint32_t m,
                            const pe::ResetArgs* r, hipStream_t st);
size_t pe_fullpass_lds_bytes(uint32_t n);
hipError_t pe_launch_fullpass_svc(const pe::SweepArgs* a_dev, int np, bool lean, const uint32_t* visit, uint32_t n,
                                  uint32_t count, pe_ranked_node* out, uint32_t* state, hipStream_t st);
hipError_t pe_launch_fullpass_lds(const pe::SweepArgs* a_dev, int np, const uint32_t* visit, uint32_t n,
                                  uint32_t count, pe_ranked_node* out, uint32_t* state, unsigned long long* prof,
                                  hipStream_t st);
hipError_t pe_launch_sweep_only(const pe::SweepArgs* a, uint32_t blocks, hipStream_t st);
hipError_t pe_launch_sweep_local(const pe::SweepArgs* a, uint32_t blocks, hipStream_t st);
hipError_t pe_launch_trace_top(const uint32_t* codes, const double* sc, const pe::TraceSrc* src, uint32_t flags,
                               pe_metric_score* out, uint8_t* n_out, hipStream_t st, uint32_t n_entries,
                               uint32_t* n_other = nullptr, uint2* other_list = nullptr);
hipError_t pe_launch_step_only(const pe::SweepArgs* a, uint32_t nrecs, const uint32_t* visit, uint32_t n,
                               uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st);
hipError_t pe_launch_commit_rows(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                                 uint32_t n, hipStream_t st);
hipError_t pe_launch_evict_trace(const pe::PreemptArgs* a, const uint32_t* rows, uint32_t n, uint32_t* code,
                                 double* named, hipStream_t st);
hipError_t pe_launch_plan_stop(pe::NodeRec* rec, uint32_t* dev_free, const pe::PreemptAlloc* allocs,
                               uint8_t* preempted, const uint32_t* slots, const uint32_t* rows, uint32_t n, int sign,
                               uint64_t* core_used, const uint64_t* palloc_cores, hipStream_t st);
hipError_t pe_launch_reset_plan(pe::NodeRec* rec, const pe::NodeRec* base_rec, uint32_t* dev_free,
                                const uint32_t* dev_free_base, uint32_t n, uint8_t* preempted, uint32_t m,
                                uint32_t* pcount, uint32_t keys, hipStream_t st);
hipError_t pe_launch_commit(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, uint32_t row,
                            uint32_t offers, hipStream_t st);
hipError_t pe_launch_evict(const pe::PreemptArgs* a, const pe::EvictResolveArgs* r, hipStream_t st);
hipError_t pe_launch_apply_commits(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                                   const uint32_t* offers, uint32_t n, int sign, hipStream_t st);
hipError_t pe_launch_evict_record(const pe::PreemptArgs* a, uint32_t row, pe_ranked_node* out, uint32_t* mask,
                                  hipStream_t st);
hipError_t pe_launch_commit_preempt(const pe::PreemptArgs* a, uint32_t row, const uint32_t* mask, uint8_t* preempted,
                                    uint32_t* pcount, uint32_t* dev_free, hipStream_t st);
hipError_t pe_launch_evict_only(const pe::PreemptArgs* a, hipStream_t st);
hipError_t pe_launch_census(const pe::BatchArgs* a, uint32_t* counts, uint8_t* status, double* score,
                            hipStream_t st, double* parts = nullptr, uint8_t* nparts = nullptr);
hipError_t pe_launch_resolve(const pe::EvictResolveArgs* r, hipStream_t st);
hipError_t pe_launch_ploop(const pe::PLoopArgs* a, hipStream_t st);
hipError_t pe_launch_md_gate(pe::MdNet* md, const uint32_t* coll_tg, uint32_t n, hipStream_t st);
hipError_t pe_launch_static_gate(const uint8_t* blocked, const uint32_t* coll_tg, uint32_t* gate, uint32_t n,
                                 hipStream_t st);
uint32_t pe_ploop_max_n(uint32_t words);
hipError_t pe_launch_commit_evicted(const pe::PreemptArgs* a, uint8_t* preempted, uint32_t* pcount,
                                    uint32_t* dev_free, uint32_t* placed, hipStream_t st);
size_t pe_fold_feas_max_classes();
hipError_t pe_launch_fold_feas_staged(const pe::NodeSoA* s, const unsigned char* class_src, uint8_t* class_dst,
                                      uint32_t ncls, const uint8_t* node_ok, uint8_t* feas, hipStream_t st);
hipError_t pe_launch_fold_feas(const pe::NodeSoA* s, const uint8_t* class_ok, const uint8_t* node_ok, uint8_t* feas,
                               hipStream_t st);
hipError_t pe_launch_sweep(const pe::SweepArgs* a, uint32_t blocks, pe::SweepRec* merged, hipStream_t st);
hipError_t pe_launch_node_record(const pe::SweepArgs* a, uint32_t row, pe_ranked_node* out, hipStream_t st);
hipError_t pe_launch_spread_table(const pe::TgTables* t, double* tab, hipStream_t st);
uint32_t pe_rec_winner(const pe::SweepRec* r);
void pe_rec_init(pe::SweepRec* r);
void pe_rec_merge(pe::SweepRec* a, const pe::SweepRec* b);
int pe_sweep_blocks_per_cu(bool aux);
hipError_t pe_launch_fold_aux(const pe::NodeSoA* s, const pe::TgTables* t, const uint8_t* aff_idx_class,
                              const uint8_t* aff_idx_node, uint32_t* aux, hipStream_t st);
uint32_t pe_chain_max_n();
uint32_t pe_chain_fused_max_n();
int pe_chain_shape(uint32_t n_visit);
uint32_t pe_chain_fused_max_count();
uint32_t pe_chain_fused_max_classes();
uint32_t pe_emit_grid(uint32_t count);
uint32_t pe_chain_max_limit();
size_t pe_chain_lds_bytes(int hash_bits, bool packed, uint32_t n);
int pe_chain_blocks_per_cu(size_t lds);
hipError_t pe_launch_chain(const pe::BatchArgs* a, uint32_t n_evals, uint32_t max_blocks, hipStream_t st,
                           hipEvent_t* split = nullptr);
hipError_t pe_launch_sweep_step(const pe::SweepArgs* a, uint32_t blocks, const uint32_t* visit, uint32_t n,
                                uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st);
hipError_t pe_launch_sweep_loop(const pe::SweepArgs* a, uint32_t blocks, uint32_t count, const uint32_t* visit,
                                uint32_t n, uint32_t offset, pe_ranked_node* out, uint32_t* state, hipStream_t st);
hipError_t pe_launch_trace(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a, const uint32_t* rows,
                           uint32_t n, uint32_t* out, const uint32_t* penalty_bits, double log10,
                           const double* spread_tab, double* scores, hipStream_t st, const uint16_t* dks = nullptr);
hipError_t pe_launch_trace_batch(const pe::NodeSoA* s, const pe::TgTables* t, const pe::Ask* a,
                                 const pe::TraceSrc* src, uint32_t n, uint32_t* out, double log10,
                                 const double* spread_tab, double* scores, hipStream_t st);
hipError_t pe_launch_spread_tables(const pe::TgTables* t, uint32_t n_rec, uint32_t* delta, double* tab,
                                   hipStream_t st);

namespace {

using pe::Target;

static std::string g_error;   // errors without a handle (create failures)

struct DevMem {
    void* p = nullptr;
    size_t bytes = 0;
    DevMem() = default;
    DevMem(const DevMem&) = delete;
    DevMem& operator=(const DevMem&) = delete;
    ~DevMem() { release(); }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    // at least b bytes (contents not kept); 1/8 headroom, so sizes that creep
    // up call after call (a run's traced rows) do not reallocate each time
    hipError_t ensure(size_t b) {
        if (b <= bytes && p) return hipSuccess;
        release();
        const size_t want = std::max<size_t>(b + b / 8, 16);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    // at least b bytes, the first `keep` bytes kept (device copy on `st`);
    // 25 % headroom so rows appended one update at a time do not copy each time
    hipError_t grow(size_t b, size_t keep, hipStream_t st) {
        if (b <= bytes && p) return hipSuccess;
        void* q = nullptr;
        const size_t want = b + b / 4;
        hipError_t e = hipMalloc(&q, want ? want : 16);
        if (e != hipSuccess) return e;
        if (p && keep) {
            e = hipMemcpyAsync(q, p, std::min(keep, bytes), hipMemcpyDeviceToDevice, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);   // before the old block is freed
        }
        if (e != hipSuccess) { (void)hipFree(q); return e; }
        release();
        p = q;
        bytes = want ? want : 16;
        return hipSuccess;
    }
};

// Page-locked host buffer: device-to-host result copies run at DMA rate and the
// caller can view the results in place (pe_batch_results).
struct PinnedMem {
    void* p = nullptr;
    size_t bytes = 0;
    PinnedMem() = default;
    PinnedMem(const PinnedMem&) = delete;
    PinnedMem& operator=(const PinnedMem&) = delete;
    ~PinnedMem() { release(); }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
        dp_of = nullptr;
    }
    hipError_t ensure(size_t b) {   // 1/8 headroom, as DevMem::ensure
        if (b <= bytes && p) return hipSuccess;
        release();
        const size_t want = std::max<size_t>(b + b / 8, 16);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocMapped);
        if (e == hipSuccess) bytes = want;
        return e;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    // the same bytes as seen from the device (kernels store results directly);
    // looked up once per allocation
    template <class T> T* dev() const {
        if (!p) return nullptr;
        if (dp_of != p) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) return nullptr;
            dp = d;
            dp_of = p;
        }
        return static_cast<T*>(dp);
    }
    mutable void* dp = nullptr;
    mutable void* dp_of = nullptr;
};

// Fixed per-node fields; the variable-length maps live in stack-owned CSR
// arrays (sorted per node) and are reached through NodeView.
struct HostNode {
    uint32_t id, name, dc, node_class, cclass;
    uint32_t cls;
    uint32_t sig;          // (class, drivers, networks, aliases, volumes, devices) signature
    int32_t first_mbits;
    uint32_t first_dev;    // string id of the first host network device (PE_NONE: none)
    uint16_t n_device_nets, n_devices;
    // that network's IP field and the one address AssignNetwork yields from its
    // CIDR (PE_NONE: none, or not known / not one address)
    uint32_t first_ipfield = PE_NONE, first_yield = PE_NONE;
    bool yield_known = false;
};

template <class T>
struct Span {
    const T* p = nullptr;
    uint32_t n = 0;
    const T* begin() const { return p; }
    const T* end() const { return p + n; }
    size_t size() const { return n; }
    bool empty() const { return n == 0; }
};

using KV = std::pair<uint32_t, uint32_t>;
using KF = std::pair<uint32_t, uint8_t>;

struct NodeView {
    const HostNode* h;
    uint32_t row;
    Span<KV> attrs, meta;          // sorted by key id
    Span<KF> drivers, volumes;     // sorted by name id
    Span<uint32_t> net_modes, aliases;
    uint32_t id() const { return h->id; }
};

struct HostAlloc {
    uint32_t row, ns, job, tg;
    bool terminal;
    int32_t priority = 0, max_parallel = 0;
    int64_t cpu = 0, mem = 0, disk = 0;
    int32_t mbits = 0, dyn = 0;            // network use: bandwidth on device net_dev, dynamic-range ports
    bool has_net = false;                  // Flattened.Networks non-empty (PreemptForNetwork candidates)
    uint32_t net_dev = PE_NONE;            // Device of its networks (str id; PE_NONE: the node's first)
    uint32_t dev_begin = 0, dev_end = 0;   // into pe_stack::alloc_dev
    uint64_t cores[4] = {0, 0, 0, 0};      // Flattened.Cpu.ReservedCores (ids < 256)
    bool cores_beyond = false;             // a reserved core id >= 256
    uint32_t port_begin = 0, port_end = 0; // into pe_stack::alloc_ports: (HostIP str id, port) held
};

// One AvailNetworks entry of a node (NodeResources.Networks with a Device,
// network.go:108-114): device, MBits, its IP field and the one address
// yieldIP gives from its CIDR (PE_NONE: unknown).
struct HostNet {
    uint32_t dev, ipfield, yield;
    int32_t mbits;
};

// One NodeNetworks address (NetworkIndex.SetNode, network.go:92-141).
struct HostAddr {
    uint32_t alias, ip;
    std::vector<int> reserved;             // its ReservedPorts, parsed
};

// One device group of a node (NodeResources.Devices[i], structs.go:2980-3010).
struct HostDevGroup {
    uint32_t vendor, type, name, healthy;
    uint32_t attr_begin, attr_end;          // into pe_stack::dev_attr
};

// Where each node's variable-length list sits in its item vector: items
// [off[r], off[r] + cnt[r]). A row rewritten with at most as many items keeps
// its place; a longer one moves to the end of the vector (its old range turns
// dead); the vector is compacted into row order once dead items outnumber the
// live ones. pe_update_nodes then costs O(changed rows), not O(table).
struct RowIndex {
    std::vector<uint32_t> off, cnt;
    size_t dead = 0;
    uint32_t b(uint32_t r) const { return off[r]; }
    uint32_t e(uint32_t r) const { return off[r] + cnt[r]; }
    uint32_t n(uint32_t r) const { return cnt[r]; }
    void clear() { off.clear(); cnt.clear(); dead = 0; }
    void rows(uint32_t n_rows) { off.resize(n_rows, 0); cnt.resize(n_rows, 0); }
};

// Row r of `ix` becomes k items written by fill(T* dst) (rows() covers r).
template <typename T, typename Fill>
void row_set(RowIndex& ix, std::vector<T>& items, uint32_t r, uint32_t k, Fill fill) {
    if (k <= ix.cnt[r]) {
        ix.dead += ix.cnt[r] - k;
        fill(items.data() + ix.off[r]);
        ix.cnt[r] = k;
        return;
    }
    ix.dead += ix.cnt[r];
    ix.off[r] = (uint32_t)items.size();
    items.resize(items.size() + k);
    fill(items.data() + ix.off[r]);
    ix.cnt[r] = k;
}

template <typename T>
void row_compact(RowIndex& ix, std::vector<T>& items) {
    if (ix.dead == 0 || ix.dead * 2 <= items.size()) return;
    std::vector<T> out;
    out.reserve(items.size() - ix.dead);
    for (size_t r = 0; r < ix.off.size(); r++) {
        const uint32_t b = (uint32_t)out.size();
        out.insert(out.end(), items.begin() + ix.off[r], items.begin() + ix.off[r] + ix.cnt[r]);
        ix.off[r] = b;
    }
    items.swap(out);
    ix.dead = 0;
}

// A device-request target parsed once (resolveDeviceTarget, feasible.go:1304-1330).
struct DevTarget {
    int kind;            // 0 literal, 1 model, 2 vendor, 3 type, 4 attr, 5 unknown interpolation
    pe::DevAttr literal;
    uint32_t key;        // attr key str id (PE_NONE: never interned -> absent)
};
struct DevCond { DevTarget l, r; std::string op; int32_t weight; };
struct DevReqSpec {
    std::string vendor, type, name;   // RequestedDevice.ID() (structs.go:2738-2761)
    bool nil_id;
    uint32_t count;
    std::vector<DevCond> constraints, affinities;
};

enum TargetKind { T_LITERAL, T_ID, T_DC, T_NAME, T_CLASS, T_ATTR, T_META, T_NIL };
struct ParsedTarget {
    TargetKind kind;
    uint32_t key;          // attr/meta key str id (PE_NONE: key never interned -> absent)
    std::string literal;
    bool escapes;
};

struct ParsedConstraint {
    ParsedTarget l, r;
    std::string op;
    bool escapes;
    std::string ltext, text;   // LTarget, Constraint.String() "l op r" (structs.go:8292)
    // checkConstraint outcome per (left value, right value) pair of interned
    // node values (see meets): nodes and classes share a handful of values
    mutable std::unordered_map<uint64_t, uint8_t> memo;
};

struct ParsedAffinity {
    ParsedConstraint c;
    int32_t weight;
};

struct SpreadSpec {
    uint32_t attribute;            // str id of the attribute target
    int32_t weight;
    std::vector<std::pair<uint32_t, int32_t>> targets;
};

struct PsetDev {
    ParsedTarget target;
    std::unordered_map<uint32_t, uint32_t> value_index;   // str id -> dense
    std::vector<uint32_t> value_str;
    DevMem val_class, val_node, counts, desired;
    std::vector<uint32_t> h_counts;
    std::vector<double> h_desired;
    bool even = false;
    double weight_frac = 0;
    bool per_node = false;
    bool distinct = false;         // distinct_property set (filter) instead of a spread (score)
    uint32_t allowed = 1;
    std::string target_text;       // LTarget of the distinct_property constraint (metrics reasons)
    std::vector<uint32_t> h_val_class, h_val_node;   // value index per class / per node (host copies)
};

struct TgPlan {
    uint32_t name;
    int32_t count;
    pe::Ask ask;
    std::vector<ParsedConstraint> constraints;   // tg + task constraints
    std::set<uint32_t> drivers;
    std::vector<std::pair<uint32_t, bool>> volumes;
    bool has_network = false;
    uint32_t net_mode = 0, net_host = 0;
    int32_t net_ports = 0;
    std::vector<ParsedAffinity> affinities;      // job + tg + task
    std::vector<SpreadSpec> spreads;             // tg spreads (job spreads kept on the job)
    bool escaped = false;
    std::string unsupported;
    // device tables
    DevMem class_ok, node_ok, class_aff, node_aff, alias_ok, coll_tg;
    bool tables_valid = false;
    bool has_aff_table = false, node_aff_used = false, node_ok_used = false, alias_used = false;
    // what alias_ok holds: the host network it was built for and the node
    // table generation (it travels with the buffer when the plan is recycled)
    uint32_t alias_for = 0xFFFFFFFFu;
    uint64_t alias_gen = 0;
    // static port asks (tg network ReservedPorts): (value, label) and the per-node gate
    std::vector<std::pair<int32_t, uint32_t>> rports;
    DevMem static_gate, static_blocked;
    // the task network's ReservedPorts (AssignNetwork, network.go:407-442) and their gate
    std::vector<std::pair<int32_t, uint32_t>> trports;
    DevMem task_gate, task_blocked;
    // PreemptForNetwork's reserved-port step per node (host-built, preemption.go:
    // 309-342): the holders to preempt first (CSR-relative alloc indices, one
    // byte each, in ask order) and flags (kPort*)
    DevMem port_list, port_info, port_block;
    // multi-device nodes (TgTables::md, build_md): the per-node records, the
    // device network each plan placement of the group took on a node (index
    // into the node's AvailNetworks, plan order), the last Preempt verdicts'
    // choices, and the other groups' plan entries when the records were built
    DevMem md_dev;
    bool md_on = false;
    std::unordered_map<uint32_t, std::vector<uint8_t>> md_hist;
    std::unordered_map<uint32_t, uint8_t> md_vdev;
    size_t md_other = 0;
    std::vector<std::unique_ptr<PsetDev>> psets;
    bool psets_built = false;
    bool elig_complete = false;   // every class's EvalEligibility entries are known (pe_get_eligibility)
    bool psets_dynamic = false;        // plan stops clear values: counts rebuilt on the host after every commit
    int n_spread = 0;                  // psets[0, n_spread) are spreads, the rest distinct_property
    std::vector<ParsedConstraint> distinct_props;   // tg + task distinct_property constraints
    // device requests (tasks in order) and the per-class match table
    std::vector<DevReqSpec> dev_reqs;
    DevMem dev_cls;
    bool dev_cls_valid = false;
    uint32_t* dev_free = nullptr;      // stack's dynamic free-instance column when dev_reqs is non-empty
    // memo emulation inputs
    std::vector<uint8_t> sig_tg, class_uniform, class_verdict, job_ok_node;
    std::vector<uint32_t> nonuniform;
    DevMem class_ok_batch, node_feas;
    // folded sweep inputs (SweepArgs::node_aux), rebuilt with the tables
    std::vector<double> h_aff_class, h_aff_node;
    DevMem node_aux, aff_vals, aff_idx;
    bool aux_valid = false, aux_ok = false;
};

static inline bool has_static(const TgPlan& g) { return !g.rports.empty() || !g.trports.empty(); }

}  // namespace

// A reference-memo entry the AllocMetric walk set: (task-group memo?, class, value).
struct MemoDelta {
    bool tg;
    uint32_t cls;
    int8_t v;
};

struct pe_stack {
    pe_config cfg{};
    std::string err;
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr;
    // per-kernel events of the windowed chain (PE_KERNEL_SPLIT / pe_set_kernel_split):
    // before k_base, after k_base, k_chain, k_emit, k_emit_writeback of the last launch
    bool kernel_split = false;
    bool split_valid = false;
    hipEvent_t ev_split[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    double last_ms = 0;
    bool last_ms_pending = false;      // last_ms still to be read from ev0 / ev1
    bool spin_wait = true;             // PE_SPIN_WAIT=0: chain launches wait with a stream sync
    bool counts_defer_ok = true;       // PE_COUNTS_DEFER=0: SetJob launches its counts at once
    uint64_t nodes_gen = 1;            // bumped whenever the node table changes (apply_nodes)
    uint32_t place_seq = 0;            // completion word sequence (run_place)
    int n_cu = 256;
    int sweep_per_cu = 4, sweep_per_cu_aux = 4;
    uint32_t last_sweep_bytes = 0;   // algorithmic bytes per node of the last sweep

    // strings
    std::vector<std::string> strs;
    std::unordered_map<std::string, uint32_t> sid;

    // state
    std::vector<HostNode> nodes;
    RowIndex attr_ix, meta_ix, drv_ix, net_ix, alias_ix, hv_ix;
    std::vector<KV> attr_kv, meta_kv;
    std::vector<KF> drv_kf, hv_kf;
    std::vector<uint32_t> net_mode_ids, alias_ids;
    std::vector<HostAlloc> allocs;
    std::vector<std::pair<uint32_t, uint32_t>> alloc_dev;   // (device group on the node, instances held)
    std::vector<std::pair<uint32_t, int32_t>> alloc_ports;  // (HostIP, port) held by allocs
    std::vector<std::vector<HostAddr>> node_addrs;          // per node, node order
    std::vector<std::vector<HostNet>> node_dnets;           // nodes with several device networks: all of them
    uint32_t n_multi_net = 0;                               // nodes with several device networks
    std::vector<std::vector<int>> node_rhp;                 // per node ReservedHostPorts, parsed
    // device groups per node and their attributes
    RowIndex dev_ix;
    std::vector<HostDevGroup> dev_groups;
    std::vector<std::pair<uint32_t, pe::DevAttr>> dev_attr;   // sorted by key per group
    size_t dev_attr_dead = 0;          // attributes of groups rewritten since the last compaction
    uint32_t n_dev_big = 0;            // live groups with more than 255 healthy instances
    uint32_t max_dev_groups = 0;
    bool dev_packable = true;          // every node fits the packed 4 x u8 free-count column
    std::vector<uint32_t> h_dev_free;  // snapshot free healthy instances per group (no plan)
    DevMem d_dev_free, d_dev_free_base;
    // ResetPlan's state copy not launched yet: it rides in SetJob's k_counts
    // launch, any other call launches it first (flush_reset)
    bool reset_pending = false;
    // The FeasibilityWrapper fold of the last build_tables, not launched yet:
    // place_impl lets it ride in the windowed chain's first launch (k_base, or
    // the fused k_chain) and launches it on its own on every other path
    // (flush_fold); nothing leaves place_impl with it pending.
    bool fold_defer_ok = false;
    bool fold_pending = false;
    pe::FoldArgs pending_fold{};
    // SetJob's collision counts (with a deferred ResetPlan copy) not launched
    // yet: a short list's fused k_chain carries them (one launch per
    // evaluation); the first other launch that reads the plan's state
    // launches them first (HIP_TRY_STATE, flush_counts)
    bool counts_pending = false;
    pe::CountArgs pending_counts{};
    // preemption: non-terminal state allocs per node (CSR, table order) as PreemptAlloc
    std::vector<uint32_t> h_node_alloc_off, h_palloc_index;   // CSR; slot -> alloc-table row
    std::vector<uint32_t> alloc_slot;          // alloc-table row -> slot (PE_NONE: terminal)
    std::vector<uint8_t> h_preempted;          // host mirror of Plan.NodePreemptions membership
    std::map<std::pair<uint32_t, uint32_t>, uint32_t> job_keys;   // (job, ns) -> key
    uint32_t n_jtg_keys = 0;
    std::string preempt_unsupported;           // snapshot outside the on-device limits
    // what build_alloc_state found, kept so that a node upsert recomputes only
    // its rows: per-row reasons (kRow*) with their counts, the allocation-only
    // reasons, the Preemptor records
    std::vector<uint8_t> row_flags;
    uint32_t n_row_overheld = 0, n_row_devent = 0, n_row_core_out = 0;
    bool evict_too_many = false, any_alloc_cores = false, alloc_state_ok = false;
    std::string cores_unsup_allocs;
    std::vector<pe::PreemptAlloc> h_palloc;
    // eviction width of the snapshot (PreemptArgs::mask_words, evict.inc): 1
    // while every node holds <= 32 non-terminal allocs, else 8 (<= 256)
    uint32_t evict_words = 1;
    // PreemptedAllocs past the PE_MAX_PREEMPT a record carries inline, of the
    // last record-producing call: (record index, the full list)
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> pre_overflow;
    // reserved cores (rank.go:437-466): 4 x u64 masks per node over core ids < 256
    bool has_cores = false;                    // some node has ReservableCpuCores / ReservedCpuCores
    std::string cores_tg_unsupported;          // why task groups asking cores stay on the host path
    uint64_t net_other_dev = 0;                // allocs on a network device other than their node's first
    std::string cores_unsupported;             // alloc core sets that fail every AllocsFit (overlap, outside)
    std::vector<uint64_t> h_core_rsvable, h_core_avail, h_core_base, h_core_used;   // used: host mirror of the plan
    std::vector<int64_t> h_core_spc;
    std::vector<uint8_t> h_core_bad;           // per node: ids >= 256, or reservable cores with TotalCpuCores 0
    uint32_t n_core_bad = 0, n_core_rows = 0;  // rows with h_core_bad / with reservable cores
    DevMem d_core_rsvable, d_core_avail, d_core_base, d_core_used, d_core_spc, d_palloc_cores;
    DevMem d_node_alloc_off, d_palloc, d_preempted, d_pcount, d_own_existing;
    DevMem d_ev_status, d_ev_score, d_ev_flags, d_ev_out, d_ev_mask, d_ev_rows, d_ev_masks, d_ev_offers, d_ev_named, d_ev_tcodes;
    uint32_t job_key = PE_NONE;
    // device offers of the last Select's pick (committed as chosen)
    int32_t offer_row = -1;
    uint32_t offers = 0xFFFFFFFFu;
    uint32_t ncls = 0;
    std::vector<uint32_t> class_rep;   // a member row of each class (the first, unless it changed)
    std::unordered_map<uint32_t, uint32_t> cls_of;                   // ComputedClass str id -> dense class
    std::unordered_map<uint64_t, std::vector<uint32_t>> sig_of;      // checker-input hash -> live signatures
    std::vector<uint64_t> sig_hash;                                   // per signature
    // Nodes with equal ComputedClass AND equal non-hashed checker inputs
    // (drivers, networks, host-network aliases, host volumes, device count)
    // share a signature: every FeasibilityChecker verdict is a function of it.
    std::vector<uint32_t> sig_rep, sig_cls;
    std::vector<std::vector<uint32_t>> class_sigs;
    // staged visit orders for pe_place_batch
    DevMem d_orders, d_batch_out, d_batch_status, d_sys_out;
    // full-scan sweep path
    DevMem d_count_ents;   // sparse per-node counts (build_collisions)
    DevMem d_rank_of, d_sweep_recs, d_sweep_merged, d_spread_tab, d_record;
    uint32_t sweep_min = 1u << 15;     // visit lists at least this long use the multi-CU sweep
    uint32_t loop_sweep_min = 8192;    // full-pass count loops this long run device-resident sweeps
    bool visit_unique = true;
    bool rank_of_valid = false;        // d_rank_of holds the current SetNodes list's positions
    std::vector<uint32_t> seen_stamp;  // SetNodes duplicate check
    uint32_t seen_gen = 0;
    double last_sweep_ms = 0;
    std::vector<uint32_t> h_orders;
    uint32_t staged_evals = 0, staged_n = 0;
    // Every mutating entry point bumps `gen`; a batch launch prepared at the
    // current gen (fresh-memo tables, limit, overlay size) is reused as is.
    uint64_t gen = 1, batch_gen = 0;
    uint32_t batch_tgi = 0, batch_count = 0;
    bool batch_full = false, batch_direct = false;
    bool results_via_copy = false;     // PE_RESULTS_VIA_COPY=1: device buffer + one D2H copy
    pe::BatchArgs batch_A{};
    PinnedMem h_batch_out, h_batch_status;
    PinnedMem h_sys_out;   // SystemStack results, staged for the caller's arrays
    PinnedMem h_place_out, h_place_status;   // single-evaluation count loop results (mapped)
    PinnedMem h_emit_done;                   // k_emit's per-workgroup completion words (mapped)
    PinnedMem h_emit_out;                    // k_emit's compact records (mapped)
    PinnedMem h_stage;                 // upload staging ring (upload_s)
    unsigned char* stage_dev = nullptr;   // the ring as seen from the device (k_upload reads it)
    DevMem d_emit, d_emit_ov, d_emit_n;   // k_chain deferred records (k_emit)
    size_t stage_off = 0;
    double phase_ms[4] = {0, 0, 0, 0};   // host prep, kernels, result copy, total (last batch)
    std::vector<pe::NodeRec> h_base_rec;     // snapshot proposed state (no plan)
    std::vector<pe::NodeRec> h_node_rec;     // node-only part (capacities, class, reserved ports)
    DevMem d_rec, d_base_rec, d_coll_job;
    DevMem d_base;                     // windowed loops: per-row base value table
    DevMem d_base1;                    // the same with one placement on the row
    DevMem d_chain_vs;                 // k_chain per-workgroup scratch (window values by position)
    DevMem d_prof;                     // k_chain step profile (PE_CHAIN_PROF)
    bool orders_unique = true;         // every staged order lists each row at most once
    bool use_base = true;              // PE_WINDOW_LAZY=1: lazy per-position evaluation (k_window)
    bool batch_chain = false;          // the prepared batch runs k_base + k_chain
    uint32_t chain_grid = 256;
    bool have_state = false;

    // job
    bool have_job = false, have_job_version = false;
    uint64_t job_version = 0;
    uint32_t job_id = 0, job_ns = 0;
    int32_t job_priority = 0;
    std::vector<ParsedConstraint> job_constraints;
    bool job_escaped = false;
    // per row for the metrics walk: the job checkers' FilterNode reason,
    // kJfPass, or null (not yet run); and the row's dense class
    std::vector<const char*> jf;
    // the job constraints jf was filled for (job_checker_key) and their texts,
    // which the jf entries point into: SetJob keeps jf while they are the same
    std::string jf_key;
    std::vector<std::string> jf_texts;
    std::vector<uint32_t> jf_cls;
    std::vector<uint32_t> jf_mclass;   // the row's metric class key (node_class, PE_NONE when empty)
    std::vector<ParsedAffinity> job_affinities;
    std::vector<SpreadSpec> job_spreads;
    std::vector<std::unique_ptr<TgPlan>> tgs;
    // retired task groups whose device tables the next SetJob reuses: freeing
    // them (hipFree) would synchronise the device on every evaluation
    std::vector<std::unique_ptr<TgPlan>> tg_pool;
    std::vector<std::pair<uint32_t, uint32_t>> plan;   // committed (tg name id, row); read through plan_of
    // a system placement's plan entries not yet written out: the rows of
    // `visit` whose staged outcome is 0 (written by plan_settle when the plan
    // is next read, dropped by ResetPlan)
    struct PlanDefer {
        bool active = false;
        uint32_t name = 0, n = 0;
        const uint8_t* status = nullptr;
    } plan_defer;

    // SpreadIterator bookkeeping (spread.go:99-102, 254)
    std::set<uint32_t> spread_info_done;
    int32_t sum_spread_weights = 0;

    // EvalEligibility memo, per task-group name: class -> -1 undecided / 0 / 1
    std::map<uint32_t, std::vector<int8_t>> tg_memo;
    std::vector<int8_t> job_memo;
    // Per-class checker results of earlier SetJobs on this node table: the
    // job's constraints, a task group's checkers (per signature) and its node
    // affinities are pure functions of the node attributes, so a job set
    // again (every evaluation of the same job) reuses them (cls_cache_*).
    uint64_t cc_gen = 0;
    std::unordered_map<std::string, std::vector<int8_t>> cc_job;
    std::unordered_map<std::string, std::vector<uint8_t>> cc_sig;
    std::unordered_map<std::string, std::vector<double>> cc_aff;
    // a spread target's values: interned value ids in first-seen class order, and per class
    std::unordered_map<std::string, std::pair<std::vector<uint32_t>, std::vector<uint32_t>>> cc_val;

    // AllocMetric maps (pe_set_metrics): the memo as the reference chain has
    // seen it so far (classes become known only when one of their nodes is
    // visited), and the last Select's maps as text
    bool metrics_on = false, metrics_valid = false;
    std::map<uint32_t, std::vector<int8_t>> ref_tg_memo;
    std::vector<int8_t> ref_job_memo;
    std::string metrics_text;          // pe_last_metrics: built from the binary maps on demand
    bool metrics_text_ok = false;
    // the last Select's maps in binary form (pe_last_metrics_bin)
    std::vector<pe_metric_count> m_counts;
    std::vector<pe_metric_score> m_scores;
    // engine strings of metric keys (PE_METRIC_ENGINE_KEY | index)
    std::vector<std::string> mstrs;
    std::unordered_map<std::string, uint32_t> mstr_ix;
    const char* mk_last_p = nullptr;   // the last interned C string (a reason pointer repeats)
    uint32_t mk_last_id = 0;
    uint32_t mkey(std::string_view t) {
        auto it = mstr_ix.find(std::string(t));
        if (it != mstr_ix.end()) return it->second;
        const uint32_t id = PE_METRIC_ENGINE_KEY | (uint32_t)mstrs.size();
        mstrs.emplace_back(t);
        mstr_ix.emplace(mstrs.back(), id);
        return id;
    }
    uint32_t mkey_p(const char* p) {   // reasons that are C strings (checker texts, literals)
        // the last pointer's key, when the text there is still the same
        if (p != mk_last_p || std::strcmp(p, mstrs[mk_last_id & ~PE_METRIC_ENGINE_KEY].c_str()) != 0) {
            mk_last_id = mkey(p);
            mk_last_p = p;
        }
        return mk_last_id;
    }

    // EvalEligibility as the reference chain holds it (pe_get_eligibility,
    // context.go:190-356): every Select logs the visit-list span its chain
    // pulled; spans resolve in visit order into the job-level and per task
    // group class maps (the memo entries FeasibilityWrapper.Next writes,
    // feasible.go:1061-1153). Resolution is lazy (SetNodes, SetJob, a get) and
    // stops as soon as every class has been seen.
    struct EligSpan { uint32_t tgi, begin, len; };
    struct ExTg { std::vector<int8_t> st; std::vector<uint8_t> seen; uint32_t unseen = 0; };
    std::vector<EligSpan> elig_log;
    std::vector<int8_t> ex_job;                          // per dense class: -1 unknown / 0 / 1
    std::vector<uint8_t> ex_job_seen;
    uint32_t ex_job_unseen = 0;
    std::map<uint32_t, ExTg> ex_tg;                      // task group name -> class map
    std::map<uint32_t, bool> ex_tg_escaped;              // tgEscapedConstraints (kept across SetJob)
    std::vector<std::pair<uint32_t, uint32_t>> ex_dirty; // (tg name or PE_NONE, class) since the last get
    std::vector<uint32_t> cls_str;                       // dense class -> ComputedClass str id
    bool elig_mute = false;                              // place_impl inside pe_place / spec_start

    // The unchanged SystemScheduler caller (scheduler_system.go:289-302):
    // SetNodes([node]) then Select for every node. From the third single-node
    // Select of a task group on, one k_system pass over every snapshot row
    // (no commit) answers the rest from a per-row cache; the caller's commits
    // queue on the host and reach HBM in one k_commit_rows launch when any
    // other call needs the device state (sys_flush). Rows a commit, stop or
    // preemption touched since the pass are answered by the single Select.
    struct SysSpec {
        bool active = false;
        uint32_t tgi = 0, singles = 0, singles_tgi = PE_NONE;
        int32_t served_row = -1;          // the last served Select's pick, awaiting its commit
        std::vector<uint32_t> pending;    // committed rows not yet in HBM
        uint64_t passes = 0, served = 0;
        // with AllocMetric on: every row's k_trace outcome and score values
        // at the cache pass (the maps of a served Select on that row)
        std::vector<uint32_t> tcode;
        std::vector<double> tscore;
        // ... and the served system-Select view's per-row entries
        // (pe_system_view.mkey / mclass / mscore / mnode_class); mfailed is
        // the caller's memo of failed classes, mfailed_eng the engine's copy
        // as of the log entries taken over
        std::vector<uint32_t> mkey, mclass, mnode_class;
        std::vector<double> mscore;
        std::vector<uint8_t> mfailed, mfailed_eng;
        bool mready = false;
    } sys;
    PinnedMem h_sys_cache;                // per row: FinalScore, or a NaN carrying the outcome (kSysDirty: stale)
    uint32_t sys_res_n = 0;               // pe_system_results: entries of the last pe_system_place
    DevMem d_identity;
    uint32_t identity_n = 0;
    DevMem d_sys_res;                     // k_system_rows outcomes by row
    uint64_t test_fallback_every = 0, test_select_calls = 0;   // PE_TEST_FALLBACK_EVERY
    DevMem d_trace_rows, d_trace_out, d_trace_scores;
    PinnedMem h_trace_top;   // spec_metrics: the batched trace's ScoreMetaData and outcome codes
    DevMem d_cm_ends;        // compute_metrics: the one record's end and source (k_trace_top)
    DevMem d_trace_top;
    DevMem d_trace_delta, d_trace_tabs;   // spec_metrics: per record spread use counts and boost tables
    DevMem d_wc_list;                     // compute_metrics: a settled whole-list walk's passing rows
    DevMem d_loop_out, d_loop_state;   // device-resident full-pass count loop
    DevMem d_ploop_mask, d_ev_score_p, d_ev_status_p, d_ev_dep;
    DevMem d_pre_mask;                       // a commit's preempted set (evict_words words)
    DevMem d_pset_g, d_pset_gb;              // FULL k_place per-value tables beyond the LDS budget (batch: gb)  // device-resident parallel count loop (k_ploop)
    DevMem d_ploop_parts, d_ploop_nparts;   // k_ploop: Preempt records per position (parts, count)
    DevMem d_fused_parts, d_fused_nparts;   // fused k_chain: first-phase score parts per position
    DevMem d_ploop_pparts, d_ploop_pnparts;   // k_ploop: plain records per position (parts, count)

    // Speculative count loop behind pe_select / pe_commit: the
    // first plain Select of a task group runs the device count loop for the
    // group's remaining placements, committing into HBM after a checkpoint of
    // the dynamic columns; later Selects are served from the records while each
    // pe_commit matches the predicted row. Any other call first flushes: the
    // device state is rolled back to the checkpoint plus the confirmed commits.
    struct Spec {
        bool active = false;
        bool pending = false;          // a served option awaits its pe_commit
        uint32_t tgi = 0;
        std::vector<pe_ranked_node> recs;
        std::vector<pe::EmitRec> crecs;   // the chain's compact records (compact = true), widened when served
        std::vector<pe::EmitRec> vrecs;   // recs narrowed for the served-Select view (compact = false)
        bool compact = false;
        uint32_t n_rec = 0, placed = 0, served = 0, confirmed = 0;
        uint32_t grow = 1;             // run length on costly paths, doubles while runs get used up
        bool checkpoint = false;       // dynamic columns saved at the start (device asks, evictions)
        // A run with the Preempt retry (preemption enabled, §25): records are
        // Select answers, a placement that evicts is two of them (the plain
        // nil, then the Preempt option), so served / confirmed count records
        // and these map records to placements.
        bool evict = false;
        std::vector<uint32_t> rec_place;   // record -> placement index, PE_NONE for a nil record
        std::vector<uint32_t> place_rec;   // placement -> its record
        std::vector<uint32_t> rflags;      // record -> PE_SPEC_* flags
        std::vector<uint32_t> pre_off, pre_list;   // record -> PreemptedAllocs (CSR, alloc-table rows)
        // AllocMetric maps of every record (pe_set_metrics on, §10/§25): the
        // texts pe_last_metrics returns (CSR), the reference-memo changes each
        // record's walk made (CSR) and the memo the run started from
        bool metrics = false;
        std::vector<pe_metric_count> mcounts;
        std::vector<uint32_t> mcounts_off;
        std::vector<pe_metric_score> mscores;
        std::vector<uint32_t> mscores_off;
        std::vector<MemoDelta> memo_log;
        std::vector<uint32_t> memo_off;
        std::vector<int8_t> memo_job0, memo_tg0;
        // an evicting run frees the evicted allocs' reserved cores (host mirror
        // and d_core_used): the run's starting used sets, for the rollback
        std::vector<uint64_t> core_used0;
    } spec;
    // place_impl with the Preempt retry: per placement, the plain nil Select
    // the retry followed (nodes evaluated / filtered / exhausted, cursor;
    // evaluated PE_NONE when the placement took no retry)
    std::vector<std::array<uint32_t, 4>>* nil_sink = nullptr;
    DevMem d_ploop_nil;
    DevMem ck_preempted, ck_pcount, ck_core_used;
    std::vector<pe::EmitRec>* emit_sink = nullptr;   // run_place: keep chain records compact here
    bool emit_sunk = false;                          // ... and it did
    pe_spec_view sview{};              // the run's records for caller-served Selects (pe_spec_view_get)
    pe_system_view sysview{};          // the per-row cache for caller-served system Selects (pe_system_view_get)
    std::vector<uint32_t> sys_log;     // its log
    uint32_t sys_taken = 0;            // log entries taken over
    bool spec_on = true;               // PE_SPECULATE=0: every Select runs on its own
    uint64_t spec_stats[4] = {0, 0, 0, 0};   // runs, Selects served, rollbacks, records computed
    DevMem ck_rec, ck_coll_job, ck_coll_tg, ck_dev_free, ck_pset[pe::kMaxPsets];
    DevMem d_commit_rows, d_commit_offers;

    // visit order
    std::vector<uint32_t> visit;
    DevMem d_visit, d_pref, d_penalty, d_out, d_status;
    bool d_visit_is_visit = false;     // d_visit holds the SetNodes list (skips re-uploads)
    uint32_t offset = 0;
    uint32_t limit = 2;
    double log10 = 0;

    std::unordered_map<uint32_t, std::vector<uint32_t>> job_allocs;   // job -> non-terminal alloc indices
    // Plan.NodeUpdate (pe_plan_stop): per node the stopped snapshot allocs in
    // append order, and per alloc its number of entries
    std::map<uint32_t, std::vector<uint32_t>> node_update;
    std::vector<uint32_t> stop_count;
    DevMem d_stop_slots, d_stop_rows;
    bool stopped(uint32_t ai) const { return ai < stop_count.size() && stop_count[ai] > 0; }

    // multi-GPU handle (pe_comm_init): an RCCL communicator over the ranks'
    // engines, one GPU each; the sharded count loop gathers per-rank records
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    // pe_comm_init_host: the caller's all-gather over host buffers instead of RCCL
    pe_exchange_fn xfn = nullptr;
    void* xctx = nullptr;
    void* h_xbuf = nullptr;   // pinned: this rank's record, then nranks records
    DevMem d_sweep_done;      // k_sweep<..., MERGE> arrival counter

    // One handle over several devices (pe_config.device_count > 1): `kids`
    // hold replicas of the snapshot, job and plan on the other devices. The
    // per-evaluation calls (state, job) are forwarded as they come; the plan
    // mutations (commits, preemptions, stops) are logged and replayed into the
    // kids before a sharded call, which also copies the cursor, limit, spread
    // bookkeeping and class memo. Sharded full-pass count loops exchange their
    // records with ncclAllGather over `group_comms` (ncclCommInitAll), or with
    // device copies when every id names one GPU (loopback). A root-only call
    // the log cannot replay (a batch system placement with evictions) marks
    // the kids stale until the next evaluation context.
    struct ReplayOp { uint8_t kind; uint32_t tgi; int32_t row; std::vector<uint32_t> a; };
    std::vector<pe_stack*> kids;
    std::vector<ncclComm_t> group_comms;
    bool loopback = false, kids_valid = true;
    std::vector<ReplayOp> replay;
    DevMem d_gather;
    pe::SweepArgs h_full_args;   // k_fullpass_lds arguments (read through d_full_args)
    DevMem d_full_args;
    hipEvent_t ev_x0 = nullptr, ev_x1 = nullptr;   // around one sampled all-gather per chunk
    double last_exchange_us = 0;
    double last_exchange_stats[4] = {0, 0, 0, 0};   // mean, min, max us, placements timed
    std::vector<hipEvent_t> ev_xs;                   // pe_place_sharded: a pair per placement of a chunk

    // PE_API_PROF=1: wall time per named host step, printed at pe_stack_destroy
    bool api_prof = false;
    std::map<std::string, std::pair<double, uint64_t>> api_acc;

    // ---- helpers --------------------------------------------------------
    int fail(int code, const std::string& m) { err = m; return code; }
    const std::vector<uint32_t>& own_allocs() const {
        static const std::vector<uint32_t> none;
        auto it = job_allocs.find(job_id);
        return it == job_allocs.end() ? none : it->second;
    }
    const std::string& S(uint32_t id) const {
        static const std::string empty;
        return id < strs.size() ? strs[id] : empty;
    }
    NodeView view(uint32_t row) const {
        NodeView v;
        v.h = &nodes[row];
        v.row = row;
        v.attrs = {attr_kv.data() + attr_ix.b(row), attr_ix.n(row)};
        v.meta = {meta_kv.data() + meta_ix.b(row), meta_ix.n(row)};
        v.drivers = {drv_kf.data() + drv_ix.b(row), drv_ix.n(row)};
        v.volumes = {hv_kf.data() + hv_ix.b(row), hv_ix.n(row)};
        v.net_modes = {net_mode_ids.data() + net_ix.b(row), net_ix.n(row)};
        v.aliases = {alias_ids.data() + alias_ix.b(row), alias_ix.n(row)};
        return v;
    }
    uint32_t lookup(const std::string& s) const {
        auto it = sid.find(s);
        return it == sid.end() ? PE_NONE : it->second;
    }
    void add_strings(const pe_strtab* t) {
        for (uint32_t i = (uint32_t)strs.size(); t && i < t->count; i++) {
            strs.emplace_back(t->bytes + t->offsets[i], t->offsets[i + 1] - t->offsets[i]);
            sid.emplace(strs.back(), i);
        }
    }
};

// The deferred system placement's Plan.AppendAlloc entries (list order).
static void plan_settle(pe_stack* s) {
    pe_stack::PlanDefer& d = s->plan_defer;
    if (!d.active) return;
    d.active = false;
    const uint32_t n = std::min<uint32_t>(d.n, (uint32_t)s->visit.size());
    size_t p = 0;
    for (uint32_t i = 0; i < n; i++) p += d.status[i] == 0;
    const size_t base = s->plan.size();
    s->plan.resize(base + p + 1);   // one slot of slack: the writes below are branch-free
    std::pair<uint32_t, uint32_t>* w = s->plan.data() + base;
    for (uint32_t i = 0; i < n; i++) {
        w->first = d.name;
        w->second = s->visit[i];
        w += d.status[i] == 0;
    }
    s->plan.resize(base + p);
}

static inline std::vector<std::pair<uint32_t, uint32_t>>& plan_of(pe_stack* s) {
    plan_settle(s);
    return s->plan;
}

extern "C" {
static void elig_log_span(pe_stack* s, uint32_t tgi, uint32_t begin, uint32_t len);
static void metrics_set_last_sys(pe_stack* s, uint32_t row, uint32_t code, bool failed_before);
static void kid_log(pe_stack* s, uint8_t kind, uint32_t tgi, int32_t row, const uint32_t* a, uint32_t n);
}

static void elig_resolve(pe_stack* s);   // the served system-Select view replays it
namespace {

constexpr uint32_t kFullLdsMaxN = 32768;          // k_fullpass_lds tried up to this list length
constexpr uint32_t kStalledFlag = 0x80000000u;   // k_chain cursor flag (kChainStalled)
constexpr uint32_t kChainErrFlag = 0x40000000u;   // k_chain bounds guard tripped (kChainError)

double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Accumulates the enclosing scope's wall time under `name` (PE_API_PROF).
struct ApiScope {
    pe_stack* s;
    const char* name;
    double t0;
    ApiScope(pe_stack* st, const char* n) : s(st), name(n), t0(st && st->api_prof ? now_us() : 0.0) {}
    ~ApiScope() {
        if (s && s->api_prof) {
            auto& a = s->api_acc[name];
            a.first += now_us() - t0;
            a.second++;
        }
    }
};

#define HIP_TRY(s, expr)                                                                \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess) return (s)->fail(PE_EHIP, std::string(#expr ": ") +       \
                                               hipGetErrorString(_e));                  \
    } while (0)

// A launch that reads the plan's device state (node records, device free
// counts, preemptions): the deferred ResetPlan copy must have been launched
// before it (every entry point starts with PE_FLUSH_RESET); a launch that
// would read the previous evaluation's state fails instead.
static int flush_counts(pe_stack* s);
#define HIP_TRY_STATE(s, expr)                                                          \
    do {                                                                                \
        if ((s)->counts_pending) {                                                      \
            const int crc_ = flush_counts(s);                                           \
            if (crc_) return crc_;                                                      \
        }                                                                               \
        if ((s)->fold_pending) {                                                        \
            const int frc_ = flush_fold(s);                                             \
            if (frc_) return frc_;                                                      \
        }                                                                               \
        if ((s)->reset_pending)                                                         \
            return (s)->fail(PE_EINTERNAL, std::string(#expr ": the deferred ResetPlan " \
                                                       "copy was not launched first")); \
        HIP_TRY(s, expr);                                                               \
    } while (0)

// Host -> device upload ordered on the engine stream: the bytes are staged in
// a page-locked ring and copied asynchronously, so an entry point does not
// wait for the device; the ring restarts after a stream synchronisation when
// it is full. Large uploads synchronise and copy directly.
constexpr size_t kStageBytes = 8u << 20;
static int flush_fold(pe_stack* s);

template <class T>
hipError_t upload_s(pe_stack* s, DevMem& m, const std::vector<T>& h) {
    const size_t b = h.size() * sizeof(T);
    hipError_t e = m.ensure(b);
    if (e != hipSuccess || b == 0) return e;
    if (b > kStageBytes / 4) {
        if (s->fold_pending && flush_fold(s) != PE_OK) return hipErrorLaunchFailure;   // it reads its staged table
        if (s->counts_pending && flush_counts(s) != PE_OK) return hipErrorLaunchFailure;   // its staged entries
        e = hipStreamSynchronize(s->stream);
        if (e != hipSuccess) return e;
        s->stage_off = 0;
        return hipMemcpy(m.p, h.data(), b, hipMemcpyHostToDevice);
    }
    if (!s->h_stage.p) {
        e = s->h_stage.ensure(kStageBytes);
        if (e != hipSuccess) return e;
    }
    size_t off = (s->stage_off + 255) & ~size_t(255);
    if (off + b > kStageBytes) {
        // the ring restarts: a pending fold / count launch still reads its staged table
        if (s->fold_pending && flush_fold(s) != PE_OK) return hipErrorLaunchFailure;
        if (s->counts_pending && flush_counts(s) != PE_OK) return hipErrorLaunchFailure;
        e = hipStreamSynchronize(s->stream);
        if (e != hipSuccess) return e;
        off = 0;
    }
    unsigned char* dst = s->h_stage.as<unsigned char>() + off;
    std::memcpy(dst, h.data(), b);
    s->stage_off = off + b;
    if (!s->stage_dev) s->stage_dev = s->h_stage.dev<unsigned char>();
    if (s->stage_dev) return pe_launch_upload(m.p, s->stage_dev + off, b, s->stream);
    return hipMemcpyAsync(m.p, dst, b, hipMemcpyHostToDevice, s->stream);
}

// Copies `h` into the page-locked staging ring without a copy launch and
// returns the staged bytes as the device sees them (a kernel that consumes a
// small table reads it from there itself), or null when it does not fit.
template <class T>
const unsigned char* stage_only(pe_stack* s, const std::vector<T>& h) {
    const size_t b = h.size() * sizeof(T);
    if (b == 0 || b > kStageBytes / 4) return nullptr;
    if (!s->h_stage.p && s->h_stage.ensure(kStageBytes) != hipSuccess) return nullptr;
    size_t off = (s->stage_off + 255) & ~size_t(255);
    if (off + b > kStageBytes) {
        if (s->fold_pending && flush_fold(s) != PE_OK) return nullptr;   // it reads its staged table
        if (s->counts_pending && flush_counts(s) != PE_OK) return nullptr;
        if (hipStreamSynchronize(s->stream) != hipSuccess) return nullptr;
        off = 0;
    }
    if (!s->stage_dev) s->stage_dev = s->h_stage.dev<unsigned char>();
    if (!s->stage_dev) return nullptr;
    std::memcpy(s->h_stage.as<unsigned char>() + off, h.data(), b);
    s->stage_off = off + b;
    return s->stage_dev + off;
}

// Visit order into d_visit; the SetNodes list itself is uploaded once per SetNodes.
hipError_t upload_visit(pe_stack* s, const std::vector<uint32_t>& order) {
    const bool is_visit = &order == &s->visit;
    if (is_visit && s->d_visit_is_visit) return hipSuccess;
    hipError_t e = upload_s(s, s->d_visit, order);
    s->d_visit_is_visit = is_visit && e == hipSuccess;
    return e;
}

ParsedTarget parse_target(const pe_stack* s, const std::string& t) {
    ParsedTarget p;
    p.key = PE_NONE;
    p.escapes = pe::target_escapes(t);
    if (t.rfind("${", 0) != 0) { p.kind = T_LITERAL; p.literal = t; return p; }
    if (t == "${node.unique.id}") { p.kind = T_ID; return p; }
    if (t == "${node.datacenter}") { p.kind = T_DC; return p; }
    if (t == "${node.unique.name}") { p.kind = T_NAME; return p; }
    if (t == "${node.class}") { p.kind = T_CLASS; return p; }
    auto strip = [&](size_t pre) {
        std::string k = t.substr(pre);
        if (!k.empty() && k.back() == '}') k.pop_back();
        return k;
    };
    if (t.rfind("${attr.", 0) == 0) { p.kind = T_ATTR; p.key = s->lookup(strip(7)); return p; }
    if (t.rfind("${meta.", 0) == 0) { p.kind = T_META; p.key = s->lookup(strip(7)); return p; }
    p.kind = T_NIL;
    return p;
}

bool find_kv(const Span<KV>& v, uint32_t key, uint32_t* val) {
    auto it = std::lower_bound(v.begin(), v.end(), std::make_pair(key, 0u));
    if (it == v.end() || it->first != key) return false;
    *val = it->second;
    return true;
}

// resolveTarget (feasible.go:748-781) on a host node; returns the value str id
// in *vid when the value comes from the node (PE_NONE for literals / absent).
Target resolve(const pe_stack* s, const ParsedTarget& p, const NodeView& n, uint32_t* vid = nullptr) {
    Target t;
    t.nil = false;
    uint32_t v = PE_NONE;
    switch (p.kind) {
        case T_LITERAL: t.found = true; t.value = p.literal; break;
        case T_ID: v = n.h->id; break;
        case T_DC: v = n.h->dc; break;
        case T_NAME: v = n.h->name; break;
        case T_CLASS: v = n.h->node_class; break;
        case T_ATTR:
        case T_META: {
            uint32_t x;
            if (p.key != PE_NONE && find_kv(p.kind == T_ATTR ? n.attrs : n.meta, p.key, &x)) v = x;
            else { t.found = false; t.value.clear(); if (vid) *vid = PE_NONE; return t; }
            break;
        }
        case T_NIL: t.nil = true; t.found = false; if (vid) *vid = PE_NONE; return t;
    }
    if (v != PE_NONE) { t.found = true; t.value = s->S(v); }
    if (vid) *vid = v;
    return t;
}

ParsedConstraint parse_constraint(const pe_stack* s, const pe_constraint& c) {
    ParsedConstraint p;
    p.l = parse_target(s, s->S(c.ltarget));
    p.r = parse_target(s, s->S(c.rtarget));
    p.op = s->S(c.operand);
    p.escapes = p.l.escapes || p.r.escapes;
    p.ltext = s->S(c.ltarget);
    p.text = p.ltext + " " + p.op + " " + s->S(c.rtarget);
    return p;
}

// The resolved target as a code: the interned value id, or a marker for a
// literal (fixed per constraint), an absent value and a nil target.
uint32_t target_code(const ParsedTarget& p, const NodeView& n) {
    constexpr uint32_t kLiteral = 0xFFFFFFFCu, kAbsent = 0xFFFFFFFDu, kNil = 0xFFFFFFFEu;
    switch (p.kind) {
        case T_LITERAL: return kLiteral;
        case T_ID: return n.h->id == PE_NONE ? kAbsent : n.h->id;
        case T_DC: return n.h->dc == PE_NONE ? kAbsent : n.h->dc;
        case T_NAME: return n.h->name == PE_NONE ? kAbsent : n.h->name;
        case T_CLASS: return n.h->node_class == PE_NONE ? kAbsent : n.h->node_class;
        case T_ATTR:
        case T_META: {
            uint32_t x;
            if (p.key != PE_NONE && find_kv(p.kind == T_ATTR ? n.attrs : n.meta, p.key, &x)) return x;
            return kAbsent;
        }
        default: return kNil;
    }
}

// checkConstraint (feasible.go:783-846) on a node, memoised per pair of
// resolved values: the outcome is a function of the two targets alone.
bool meets(const pe_stack* s, pe::ConstraintEvaluator& ev, const ParsedConstraint& c, const NodeView& n) {
    const uint64_t key = ((uint64_t)target_code(c.l, n) << 32) | target_code(c.r, n);
    auto it = c.memo.find(key);
    if (it != c.memo.end()) return it->second != 0;
    Target l = resolve(s, c.l, n), r = resolve(s, c.r, n);
    const bool ok = ev.check(c.op, l, r);
    c.memo.emplace(key, ok ? 1 : 0);
    return ok;
}

// ---- devices (host side) ------------------------------------------------------
DevTarget parse_dev_target(const pe_stack* s, const std::string& t) {
    DevTarget d;
    d.key = PE_NONE;
    if (t.rfind("${", 0) != 0) { d.kind = 0; d.literal = pe::parse_dev_attr(t); return d; }
    if (t == "${device.model}") { d.kind = 1; return d; }
    if (t == "${device.vendor}") { d.kind = 2; return d; }
    if (t == "${device.type}") { d.kind = 3; return d; }
    if (t.rfind("${device.attr.", 0) == 0) {
        std::string k = t.substr(14);
        if (!k.empty() && k.back() == '}') k.pop_back();
        d.kind = 4;
        d.key = s->lookup(k);
        return d;
    }
    d.kind = 5;
    return d;
}

// resolveDeviceTarget (feasible.go:1304-1330); returns found
bool dev_resolve(const pe_stack* s, const DevTarget& t, const HostDevGroup& g, pe::DevAttr* out) {
    switch (t.kind) {
        case 0: *out = t.literal; return true;
        case 1: out->kind = pe::DevAttr::kString; out->s = s->S(g.name); return true;
        case 2: out->kind = pe::DevAttr::kString; out->s = s->S(g.vendor); return true;
        case 3: out->kind = pe::DevAttr::kString; out->s = s->S(g.type); return true;
        case 4: {
            if (t.key == PE_NONE) return false;
            auto b = s->dev_attr.begin() + g.attr_begin, e = s->dev_attr.begin() + g.attr_end;
            auto it = std::lower_bound(b, e, t.key, [](const auto& x, uint32_t k) { return x.first < k; });
            if (it == e || it->first != t.key) return false;
            *out = it->second;
            return true;
        }
        default: return false;
    }
}

bool dev_cond(const pe_stack* s, pe::ConstraintEvaluator& ev, const DevCond& c, const HostDevGroup& g) {
    pe::DevAttr l, r;
    const bool lf = dev_resolve(s, c.l, g, &l), rf = dev_resolve(s, c.r, g, &r);
    return ev.check_attr(c.op, l, lf, r, rf);
}

// nodeDeviceMatches (feasible.go:1278-1300) with DeviceIdTuple.Matches (structs.go:3130-3148)
bool dev_matches(const pe_stack* s, pe::ConstraintEvaluator& ev, const DevReqSpec& q, const HostDevGroup& g) {
    if (q.nil_id) return false;
    if (!q.name.empty() && q.name != s->S(g.name)) return false;
    if (!q.vendor.empty() && q.vendor != s->S(g.vendor)) return false;
    if (!q.type.empty() && q.type != s->S(g.type)) return false;
    for (auto& c : q.constraints)
        if (!dev_cond(s, ev, c, g)) return false;
    return true;
}

// DeviceChecker.hasDevices (feasible.go:1206-1274): healthy instances, groups in node order.
bool has_devices(const pe_stack* s, pe::ConstraintEvaluator& ev, const TgPlan& g, uint32_t row) {
    if (g.dev_reqs.empty()) return true;
    const uint32_t b = s->dev_ix.b(row), e = s->dev_ix.e(row);
    if (b == e) return false;
    std::vector<int64_t> avail(e - b);
    for (uint32_t k = b; k < e; k++) avail[k - b] = s->dev_groups[k].healthy;
    for (const DevReqSpec& q : g.dev_reqs) {
        bool ok = false;
        for (uint32_t k = b; k < e; k++) {
            if (s->dev_groups[k].healthy == 0) continue;
            const int64_t unused = avail[k - b];
            if (unused == 0 || unused < (int64_t)q.count) continue;
            if (dev_matches(s, ev, q, s->dev_groups[k])) {
                avail[k - b] -= q.count;
                ok = true;
                break;
            }
        }
        if (!ok) return false;
    }
    return true;
}

DevReqSpec parse_dev_request(const pe_stack* s, const pe_job* j, const pe_device_request& r) {
    DevReqSpec q;
    const std::string nm = s->S(r.name);
    q.nil_id = nm.empty();
    std::vector<std::string> parts;   // strings.SplitN(name, "/", 3)
    size_t start = 0;
    while (parts.size() < 2) {
        const size_t k = nm.find('/', start);
        if (k == std::string::npos) break;
        parts.push_back(nm.substr(start, k - start));
        start = k + 1;
    }
    parts.push_back(nm.substr(start));
    if (parts.size() == 1) q.type = parts[0];
    else if (parts.size() == 2) { q.vendor = parts[0]; q.type = parts[1]; }
    else { q.vendor = parts[0]; q.type = parts[1]; q.name = parts[2]; }
    q.count = (uint32_t)std::min<uint64_t>(r.count, 0xFFFFFFFFull);
    for (uint32_t k = 0; k < r.constraint_count; k++) {
        const pe_constraint& c = j->device_constraints[r.constraint_off + k];
        q.constraints.push_back(DevCond{parse_dev_target(s, s->S(c.ltarget)), parse_dev_target(s, s->S(c.rtarget)),
                                        s->S(c.operand), 0});
    }
    for (uint32_t k = 0; k < r.affinity_count; k++) {
        const pe_affinity& a = j->device_affinities[r.affinity_off + k];
        q.affinities.push_back(DevCond{parse_dev_target(s, s->S(a.ltarget)), parse_dev_target(s, s->S(a.rtarget)),
                                       s->S(a.operand), a.weight});
    }
    return q;
}

// Per-class device table: match bits and AssignDevice scores of each request
// against each device group of the class (class representative's groups).
int build_dev_classes(pe_stack* s, TgPlan& g) {
    pe::ConstraintEvaluator ev;
    std::vector<pe::DevClass> tab(std::max<uint32_t>(s->ncls, 1));
    std::memset(tab.data(), 0, sizeof(pe::DevClass) * tab.size());
    for (uint32_t c = 0; c < s->ncls; c++) {
        const uint32_t row = s->class_rep[c];
        const uint32_t b = s->dev_ix.b(row), e = s->dev_ix.e(row);
        pe::DevClass& d = tab[c];
        d.n_groups = e - b;
        for (size_t q = 0; q < g.dev_reqs.size(); q++) {
            const DevReqSpec& r = g.dev_reqs[q];
            for (uint32_t k = b; k < e; k++) {
                const HostDevGroup& grp = s->dev_groups[k];
                if (!dev_matches(s, ev, r, grp)) continue;
                d.match[q] |= (uint8_t)(1u << (k - b));
                double choice = 0, sum = 0;
                if (!r.affinities.empty()) {   // device.go:72-93
                    double total = 0;
                    for (auto& a : r.affinities) {
                        total += std::fabs((double)a.weight);
                        if (!dev_cond(s, ev, a, grp)) continue;
                        choice += (double)a.weight;
                        sum += (double)a.weight;
                    }
                    choice /= total;
                }
                d.choice[q][k - b] = choice;
                d.matched[q][k - b] = sum;
            }
        }
    }
    HIP_TRY(s, upload_s(s, g.dev_cls, tab));
    g.dev_cls_valid = true;
    g.dev_free = s->d_dev_free.as<uint32_t>();
    return PE_OK;
}

// job checkers (ConstraintChecker over job constraints)
// First failing job checker's FilterNode reason, or nullptr (feasible).
const char* job_fail(const pe_stack* s, pe::ConstraintEvaluator& ev, const NodeView& n) {
    for (auto& c : s->job_constraints) if (!meets(s, ev, c, n)) return c.text.c_str();
    return nullptr;
}

bool job_feasible(const pe_stack* s, pe::ConstraintEvaluator& ev, const NodeView& n) {
    return job_fail(s, ev, n) == nullptr;
}

// job_fail of a row, cached per row for the job and snapshot (the checkers
// are a pure function of the node's attributes and the job's constraints)
const char kJfPass[] = "";
static void jf_ready(pe_stack* s) {
    if (s->jf.size() == s->nodes.size()) return;
    s->jf.assign(s->nodes.size(), nullptr);
    s->jf_cls.resize(s->nodes.size());
    s->jf_mclass.resize(s->nodes.size());
    for (size_t r = 0; r < s->nodes.size(); r++) {
        s->jf_cls[r] = s->nodes[r].cls;
        const uint32_t nc = s->nodes[r].node_class;
        s->jf_mclass[r] = (nc != PE_NONE && !s->S(nc).empty()) ? nc : PE_NONE;
    }
}

const char* job_fail_cached(pe_stack* s, pe::ConstraintEvaluator& ev, uint32_t row) {
    const char* w = s->jf[row];
    if (!w) {
        w = kJfPass;
        const NodeView n = s->view(row);
        for (size_t k = 0; k < s->job_constraints.size(); k++)
            if (!meets(s, ev, s->job_constraints[k], n)) {
                w = s->jf_texts[k].c_str();   // the same text, kept across SetJob
                break;
            }
        s->jf[row] = w;
    }
    return w == kJfPass ? nullptr : w;
}

// tg checkers in GenericStack/SystemStack order: drivers, constraints, host
// volumes, devices, network (stack.go:241-247, 374-380)
// First failing task-group checker's FilterNode reason (feasible.go:353, 378,
// 467, 539-556, ConstraintChecker: Constraint.String()), or nullptr.
const char* tg_fail(const pe_stack* s, pe::ConstraintEvaluator& ev, const TgPlan& g, const NodeView& n) {
    static const char* kDrivers = "missing drivers";
    static const char* kVolumes = "missing compatible host volumes";
    static const char* kDevices = "missing devices";
    static const char* kNetwork = "missing network";
    static const char* kHostNet = "missing host network";
    static const char* kBadHostNet = "invalid host network";
    for (uint32_t d : g.drivers) {   // DriverChecker.hasDrivers (feasible.go:462-500)
        auto it = std::lower_bound(n.drivers.begin(), n.drivers.end(), std::make_pair(d, (uint8_t)0));
        if (it != n.drivers.end() && it->first == d) {
            const uint8_t f = it->second;
            if (f & 4) return kDrivers;
            if ((f & 1) && (f & 2)) continue;
            return kDrivers;
        }
        uint32_t key = s->lookup("driver." + s->S(d)), val;
        if (key == PE_NONE || !find_kv(n.attrs, key, &val)) return kDrivers;
        const std::string& v = s->S(val);
        if (v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True") continue;
        return kDrivers;   // "0"/false or ParseBool error
    }
    for (auto& c : g.constraints) if (!meets(s, ev, c, n)) return c.text.c_str();
    if (!g.volumes.empty()) {   // HostVolumeChecker.hasVolumes (feasible.go:171-207)
        std::map<uint32_t, std::vector<bool>> req;
        for (auto& v : g.volumes) req[v.first].push_back(v.second);
        if (req.size() > n.volumes.size()) return kVolumes;
        for (auto& kv : req) {
            auto it = std::lower_bound(n.volumes.begin(), n.volumes.end(), std::make_pair(kv.first, (uint8_t)0));
            if (it == n.volumes.end() || it->first != kv.first) return kVolumes;
            if (!it->second) continue;
            for (bool ro : kv.second) if (!ro) return kVolumes;
        }
    }
    if (!has_devices(s, ev, g, n.row)) return kDevices;
    {   // NetworkChecker (feasible.go:362-429): runs for every task group; without a
        // tg network it keeps the mode of the last one set (default "host").
        const std::string want = s->S(g.net_mode).empty() ? std::string("host") : s->S(g.net_mode);
        bool has = false;
        for (uint32_t m : n.net_modes) {
            const std::string& mode = s->S(m).empty() ? std::string("host") : s->S(m);
            if (mode == want) { has = true; break; }
        }
        if (!has) {
            bool legacy = false;
            if (want == "bridge") {
                uint32_t key = s->lookup("nomad.version"), val;
                pe::SemVer v, c;
                if (key != PE_NONE && find_kv(n.attrs, key, &val) && pe::parse_version(s->S(val), true, &v) &&
                    pe::parse_version("0.12", false, &c)) {
                    const bool pre_ok = v.pre.empty();
                    legacy = pre_ok && pe::compare_versions(v, c) == -1;
                }
            }
            if (!legacy) return kNetwork;
        } else if (g.net_ports > 0) {
            // hasHostNetworks: every port's host network must be an alias on the node
            ParsedTarget hn = parse_target(s, s->S(g.net_host));
            Target t = resolve(s, hn, n);
            if (!t.found) return kBadHostNet;
            uint32_t want_id = s->lookup(t.value);
            if (std::find(n.aliases.begin(), n.aliases.end(), want_id) == n.aliases.end()) return kHostNet;
        }
    }
    return nullptr;
}

bool tg_feasible(const pe_stack* s, pe::ConstraintEvaluator& ev, const TgPlan& g, const NodeView& n) {
    return tg_fail(s, ev, g, n) == nullptr;
}

// AllocatedResources.Comparable() with lifecycle rules (structs.go:3445-3487)
void tg_ask(const pe_job* j, const pe_task_group& t, pe::Ask* a) {
    int64_t sc_c = 0, sc_m = 0, eph_c = 0, eph_m = 0, main_c = 0, main_m = 0, ps_c = 0, ps_m = 0;
    a->task_mbits = 0; a->task_dyn = 0; a->has_task_net = 0;
    a->cores = 0;
    for (uint32_t k = 0; k < t.task_count; k++) {
        const pe_task& x = j->tasks[t.task_off + k];
        // a task with reserved cores holds SharesPerCore x cores CpuShares on the
        // chosen node (rank.go:461-463): its cpu is the per-node part of the ask
        const int64_t cpu = x.cores > 0 ? 0 : x.cpu;
        if (x.cores > 0) a->cores += x.cores;
        switch (x.lifecycle) {
            case PE_LC_MAIN: main_c += cpu; main_m += x.memory_mb; break;
            case PE_LC_PRESTART: eph_c += cpu; eph_m += x.memory_mb; break;
            case PE_LC_PRESTART_SIDECAR: sc_c += cpu; sc_m += x.memory_mb; break;
            case PE_LC_POSTSTOP: ps_c += cpu; ps_m += x.memory_mb; break;
            default: break;
        }
        if (x.has_network) {
            a->has_task_net += 1;   // the number of task networks (AssignNetwork per task)
            a->task_mbits += x.net_mbits;
            a->task_dyn += x.net_dyn_ports;
        }
    }
    eph_c = std::max(std::max(eph_c, main_c), ps_c);
    eph_m = std::max(std::max(eph_m, main_m), ps_m);
    a->cpu = sc_c + eph_c;
    a->mem = sc_m + eph_m;
    a->disk = t.ephemeral_disk_mb;
    a->tg_dyn = t.has_network ? t.net_dyn_ports : 0;
    a->static_dyn = 0;   // static ports in [MinDynamicPort, MaxDynamicPort]: the dynamic picks skip them
    for (uint32_t k = 0; t.has_network && j->rport_value && k < t.rport_count; k++) {
        const int32_t v = j->rport_value[t.rport_off + k];
        a->static_dyn += (v >= 20000 && v <= 32000) ? 1 : 0;
    }
    // NetworkIndex.AddAllocs contribution of the placed alloc (network.go:144-193)
    if (t.has_network && t.net_dyn_ports + t.net_reserved_ports > 0) {
        a->commit_mbits = 0;
        a->commit_dyn = t.net_dyn_ports + a->static_dyn;
    } else {
        a->commit_mbits = a->task_mbits;
        a->commit_dyn = a->task_dyn;
    }
    a->desired_count = t.count;
}

int append_allocs(pe_stack* s, const pe_alloc_table* at, const uint32_t* index);
int build_alloc_state(pe_stack* s);

// Node rows of a pe_node_table into the host mirror (build_state, and the
// node upserts of pe_update_nodes): source row i of `nt` becomes row
// target[i]; rows not targeted keep their data; the list grows to n_new rows.
// The variable-length maps and the device groups are rebuilt as one pass of
// copies; ComputedClass and checker signatures are interned into the persistent
// maps, and a class / signature whose representative row changed gets another
// member as its representative.
// structs.ParsePortRanges (funcs.go:495-548) as NetworkIndex uses it: a spec
// that does not parse reserves nothing; ports >= 65536 are dropped (the
// reference stops at the first one in map order; ascending is one legal order).
std::vector<int> parse_port_ranges(const std::string& spec) {
    std::vector<int> out;
    if (spec.empty()) return out;
    size_t b = 0;
    while (b <= spec.size()) {
        size_t e = spec.find(',', b);
        if (e == std::string::npos) e = spec.size();
        std::string part = spec.substr(b, e - b);
        while (!part.empty() && part.front() == ' ') part.erase(part.begin());
        while (!part.empty() && part.back() == ' ') part.pop_back();
        auto num = [](const std::string& x, uint64_t* v) {
            if (x.empty() || x.size() > 19) return false;
            uint64_t r = 0;
            for (char c : x) { if (c < '0' || c > '9') return false; r = r * 10 + (uint64_t)(c - '0'); }
            *v = r;
            return true;
        };
        const size_t dash = part.find('-');
        uint64_t lo, hi;
        if (dash == std::string::npos) {
            if (!num(part, &lo)) return {};
            hi = lo;
        } else {
            if (part.find('-', dash + 1) != std::string::npos) return {};
            if (!num(part.substr(0, dash), &lo) || !num(part.substr(dash + 1), &hi) || hi < lo) return {};
        }
        for (uint64_t v = lo; v <= hi && v < 65536; v++) out.push_back((int)v);
        b = e + 1;
    }
    std::sort(out.begin(), out.end());
    out.erase(std::unique(out.begin(), out.end()), out.end());
    return out;
}

int apply_nodes(pe_stack* s, const pe_node_table* nt, const std::vector<uint32_t>& target, uint32_t n_new) {
    s->nodes_gen++;   // node-table-derived device buffers (alias_ok) are stale
    const uint32_t n_old = (uint32_t)s->nodes.size();
    const uint32_t m = nt->n;
    // the source rows in target-row order (classes and signatures are interned
    // in row order, as a full build does); every target once, appended rows
    // exactly n_old .. n_new - 1
    std::vector<uint32_t> order(m);
    for (uint32_t i = 0; i < m; i++) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return target[x] < target[y]; });
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t t = target[order[j]];
        if (t >= n_new || (j && t == target[order[j - 1]])) return s->fail(PE_EINVAL, "bad node row");
    }
    {
        uint32_t n_app = 0;
        for (uint32_t j = 0; j < m; j++) n_app += target[order[j]] >= n_old;
        if (n_app != n_new - n_old) return s->fail(PE_EINVAL, "appended node rows must be contiguous");
    }
    // variable-length node maps, rewritten row by row (sorted per node)
    auto span = [](const uint32_t* off, uint32_t i) -> uint32_t {
        return off && off[i + 1] > off[i] ? off[i + 1] - off[i] : 0;
    };
    auto put = [&](RowIndex& ix, auto& items, const uint32_t* noff, auto item_of, bool sorted) {
        ix.rows(n_new);
        for (uint32_t j = 0; j < m; j++) {
            const uint32_t i = order[j];
            const uint32_t k = span(noff, i), k0 = k ? noff[i] : 0;
            row_set(ix, items, target[i], k, [&](auto* dst) {
                for (uint32_t q = 0; q < k; q++) dst[q] = item_of(k0 + q);
                if (sorted) std::sort(dst, dst + k);
            });
        }
        row_compact(ix, items);
    };
    put(s->attr_ix, s->attr_kv, nt->attr_off, [&](uint32_t k) { return KV(nt->attr_key[k], nt->attr_val[k]); }, true);
    put(s->meta_ix, s->meta_kv, nt->meta_off, [&](uint32_t k) { return KV(nt->meta_key[k], nt->meta_val[k]); }, true);
    put(s->drv_ix, s->drv_kf, nt->drv_off, [&](uint32_t k) { return KF(nt->drv_name[k], nt->drv_flags[k]); }, true);
    put(s->net_ix, s->net_mode_ids, nt->net_off, [&](uint32_t k) { return nt->net_mode[k]; }, false);
    put(s->alias_ix, s->alias_ids, nt->alias_off, [&](uint32_t k) { return nt->alias_name[k]; }, true);
    put(s->hv_ix, s->hv_kf, nt->hv_off, [&](uint32_t k) { return KF(nt->hv_name[k], nt->hv_read_only[k]); }, true);
    // device groups (NodeResources.Devices) with typed attributes
    {
        s->dev_ix.rows(n_new);
        bool max_dirty = false;
        for (uint32_t j = 0; j < m; j++) {
            const uint32_t i = order[j], r = target[i];
            for (uint32_t g = s->dev_ix.b(r); g < s->dev_ix.e(r); g++) {   // the row's old groups leave
                const HostDevGroup& d = s->dev_groups[g];
                s->n_dev_big -= d.healthy > 255;
                s->dev_attr_dead += d.attr_end - d.attr_begin;
            }
            if (s->dev_ix.n(r) && s->dev_ix.n(r) == s->max_dev_groups) max_dirty = true;
            const uint32_t k = span(nt->dev_off, i), g0 = k ? nt->dev_off[i] : 0;
            row_set(s->dev_ix, s->dev_groups, r, k, [&](HostDevGroup* dst) {
                for (uint32_t j = 0; j < k; j++) {
                    const uint32_t g = g0 + j;
                    HostDevGroup d{nt->dev_vendor[g], nt->dev_type[g], nt->dev_name[g], nt->dev_healthy[g], 0, 0};
                    d.attr_begin = (uint32_t)s->dev_attr.size();
                    for (uint32_t q = nt->dev_attr_off ? nt->dev_attr_off[g] : 0;
                         nt->dev_attr_off && q < nt->dev_attr_off[g + 1]; q++) {
                        const pe_attr& pa = nt->dev_attr_val[q];
                        pe::DevAttr at;
                        switch (pa.kind) {
                            case PE_ATTR_INT: at.kind = pe::DevAttr::kInt; at.i = pa.i; at.unit = s->S(pa.unit); break;
                            case PE_ATTR_FLOAT: at.kind = pe::DevAttr::kFloat; at.f = pa.f; at.unit = s->S(pa.unit); break;
                            case PE_ATTR_BOOL: at.kind = pe::DevAttr::kBool; at.b = pa.i != 0; break;
                            default: at.kind = pe::DevAttr::kString; at.s = s->S(pa.s); break;
                        }
                        s->dev_attr.emplace_back(nt->dev_attr_key[q], at);
                    }
                    d.attr_end = (uint32_t)s->dev_attr.size();
                    std::sort(s->dev_attr.begin() + d.attr_begin, s->dev_attr.begin() + d.attr_end,
                              [](const auto& x, const auto& y) { return x.first < y.first; });
                    s->n_dev_big += d.healthy > 255;
                    dst[j] = d;
                }
            });
            s->max_dev_groups = std::max(s->max_dev_groups, k);
        }
        row_compact(s->dev_ix, s->dev_groups);
        if (s->dev_attr_dead && s->dev_attr_dead * 2 > s->dev_attr.size()) {   // attributes back into group order
            std::vector<std::pair<uint32_t, pe::DevAttr>> attrs;
            attrs.reserve(s->dev_attr.size() - s->dev_attr_dead);
            for (uint32_t r = 0; r < n_new; r++)
                for (uint32_t g = s->dev_ix.b(r); g < s->dev_ix.e(r); g++) {
                    HostDevGroup& d = s->dev_groups[g];
                    const uint32_t b = (uint32_t)attrs.size();
                    attrs.insert(attrs.end(), s->dev_attr.begin() + d.attr_begin, s->dev_attr.begin() + d.attr_end);
                    d.attr_begin = b;
                    d.attr_end = (uint32_t)attrs.size();
                }
            s->dev_attr.swap(attrs);
            s->dev_attr_dead = 0;
        }
        if (max_dirty) {   // a row that held the maximum changed: the exact maximum again
            s->max_dev_groups = 0;
            for (uint32_t r = 0; r < n_new; r++) s->max_dev_groups = std::max(s->max_dev_groups, s->dev_ix.n(r));
        }
        s->dev_packable = s->n_dev_big == 0 && s->max_dev_groups <= (uint32_t)pe::kMaxDevGroups;
    }
    // fixed per-node fields, ComputedClass interning; the changed rows' old
    // class and signature (representatives of those move to another member)
    s->nodes.resize(n_new);
    s->h_node_rec.resize(n_new);
    std::unordered_map<uint32_t, std::pair<uint32_t, uint32_t>> old_of;
    old_of.reserve(m * 2);
    for (uint32_t i = 0; i < m; i++)
        if (target[i] < n_old) old_of.emplace(target[i], std::make_pair(s->nodes[target[i]].cls, s->nodes[target[i]].sig));
    auto changed = [&](uint32_t r) { return r >= n_old || old_of.count(r) != 0; };
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t i = order[j], r = target[i];
        HostNode& h = s->nodes[r];
        if (r < n_old && h.n_device_nets > 1) s->n_multi_net--;
        h = HostNode();
        h.id = nt->id[i]; h.name = nt->name[i]; h.dc = nt->datacenter[i];
        h.node_class = nt->node_class[i]; h.cclass = nt->computed_class[i];
        auto it = s->cls_of.find(h.cclass);
        if (it == s->cls_of.end()) {
            it = s->cls_of.emplace(h.cclass, (uint32_t)s->class_rep.size()).first;
            s->class_rep.push_back(r);
            s->class_sigs.emplace_back();
        }
        h.cls = it->second;
        h.n_device_nets = 0;
        h.first_mbits = -1;
        h.first_dev = PE_NONE;
        h.first_ipfield = h.first_yield = PE_NONE;
        h.yield_known = false;
        for (uint32_t k = nt->net_off[i]; k < nt->net_off[i + 1]; k++) {
            if (!s->S(nt->net_device[k]).empty()) {
                if (h.n_device_nets == 0) {
                    h.first_mbits = nt->net_mbits[k];
                    h.first_dev = nt->net_device[k];
                    if (nt->net_ip) h.first_ipfield = nt->net_ip[k];
                    if (nt->net_cidr_ip) { h.first_yield = nt->net_cidr_ip[k]; h.yield_known = h.first_yield != PE_NONE; }
                }
                h.n_device_nets++;
            }
        }
        s->node_dnets.resize(n_new);
        s->node_dnets[r].clear();
        if (h.n_device_nets > 1) {   // AvailNetworks in node order (yieldIP walks them, network.go:294-315)
            s->n_multi_net++;
            for (uint32_t k = nt->net_off[i]; k < nt->net_off[i + 1]; k++)
                if (!s->S(nt->net_device[k]).empty())
                    s->node_dnets[r].push_back(HostNet{nt->net_device[k], nt->net_ip ? nt->net_ip[k] : PE_NONE,
                                                       nt->net_cidr_ip ? nt->net_cidr_ip[k] : PE_NONE,
                                                       nt->net_mbits[k]});
        }
        h.n_devices = (uint16_t)s->dev_ix.n(r);
        pe::NodeRec& rec = s->h_node_rec[r];
        std::memset(&rec, 0, sizeof(rec));
        rec.cls = h.cls;
        rec.cap_cpu = nt->cpu_shares[i] - nt->reserved_cpu[i];
        rec.cap_mem = nt->memory_mb[i] - nt->reserved_memory_mb[i];
        rec.cap_disk = nt->disk_mb[i] - nt->reserved_disk_mb[i];
        rec.avail_mbits = h.first_mbits;
        rec.used_dyn = nt->reserved_dyn_ports ? nt->reserved_dyn_ports[i] : 0;
    }
    // reserved cores (rank.go:437-466, structs.go:3891-3906): reservable and
    // AllocsFit-available (reservable - node reserved) masks, SharesPerCore
    s->h_core_rsvable.resize(4 * (size_t)n_new, 0);
    s->h_core_avail.resize(4 * (size_t)n_new, 0);
    s->h_core_spc.resize(n_new, 0);
    s->h_core_bad.resize(n_new, 0);
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t i = order[j], r = target[i];
        uint64_t* rs = &s->h_core_rsvable[4 * (size_t)r];
        uint64_t* av = &s->h_core_avail[4 * (size_t)r];
        s->n_core_bad -= s->h_core_bad[r];
        s->n_core_rows -= (rs[0] | rs[1] | rs[2] | rs[3]) != 0;
        uint64_t rsv[4] = {0, 0, 0, 0};
        for (int w = 0; w < 4; w++) rs[w] = av[w] = 0;
        uint8_t bad = 0;
        for (uint32_t k = nt->core_off ? nt->core_off[i] : 0; nt->core_off && k < nt->core_off[i + 1]; k++) {
            const uint16_t c = nt->core_id[k];
            if (c >= 256) { bad = 1; continue; }
            rs[c >> 6] |= 1ull << (c & 63);
        }
        for (uint32_t k = nt->rsv_core_off ? nt->rsv_core_off[i] : 0; nt->rsv_core_off && k < nt->rsv_core_off[i + 1]; k++) {
            const uint16_t c = nt->rsv_core_id[k];
            if (c < 256) rsv[c >> 6] |= 1ull << (c & 63);
        }
        for (int w = 0; w < 4; w++) av[w] = rs[w] & ~rsv[w];
        const uint32_t total = nt->total_cores ? nt->total_cores[i] : 0;
        s->h_core_spc[r] = total ? nt->cpu_shares[i] / (int64_t)total : 0;
        if (total == 0 && (rs[0] | rs[1] | rs[2] | rs[3])) bad = 1;
        s->h_core_bad[r] = bad;
        s->n_core_bad += bad;
        s->n_core_rows += (rs[0] | rs[1] | rs[2] | rs[3]) != 0;
    }
    // NodeNetworks addresses and ReservedHostPorts (static port asks)
    s->node_addrs.resize(n_new);
    s->node_rhp.resize(n_new);
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t i = order[j], r = target[i];
        auto& av = s->node_addrs[r];
        av.clear();
        for (uint32_t k = nt->addr_off ? nt->addr_off[i] : 0; nt->addr_off && k < nt->addr_off[i + 1]; k++) {
            HostAddr a;
            a.alias = nt->addr_alias[k];
            a.ip = nt->addr_ip[k];
            if (nt->addr_rsv_ports && nt->addr_rsv_ports[k] != PE_NONE) a.reserved = parse_port_ranges(s->S(nt->addr_rsv_ports[k]));
            av.push_back(std::move(a));
        }
        s->node_rhp[r].clear();
        if (nt->rsv_host_ports && nt->rsv_host_ports[i] != PE_NONE) s->node_rhp[r] = parse_port_ranges(s->S(nt->rsv_host_ports[i]));
    }
    // the device copies of the core masks are made by build_alloc_state /
    // refresh_node_rows (whole, or the changed rows)
    s->has_cores = s->n_core_rows > 0;
    s->cores_tg_unsupported = s->n_core_bad ? "core ids >= 256, or reservable cores with TotalCpuCores 0" : "";
    s->ncls = (uint32_t)s->class_rep.size();
    // checker-input signatures: nodes with equal ComputedClass AND equal
    // non-hashed checker inputs (drivers, networks, aliases, volumes, device
    // health). A 64-bit hash of the inputs; equal hashes are verified exactly
    // against the signature's representative before being merged.
    auto same_inputs = [&](uint32_t a_row, uint32_t b_row) {
        const NodeView x = s->view(a_row), y = s->view(b_row);
        auto eq = [](auto u, auto v) { return u.size() == v.size() && std::equal(u.begin(), u.end(), v.begin()); };
        if (x.h->n_devices != y.h->n_devices) return false;
        for (uint32_t k = 0; k < x.h->n_devices; k++)   // DeviceChecker reads healthy counts
            if (s->dev_groups[s->dev_ix.b(a_row) + k].healthy != s->dev_groups[s->dev_ix.b(b_row) + k].healthy)
                return false;
        return x.h->cls == y.h->cls && eq(x.drivers, y.drivers) &&
               eq(x.net_modes, y.net_modes) && eq(x.aliases, y.aliases) && eq(x.volumes, y.volumes);
    };
    auto sig_hash = [&](uint32_t r) {
        const HostNode& h = s->nodes[r];
        const NodeView v = s->view(r);
        uint64_t x = 1469598103934665603ull;
        auto mix = [&](uint64_t y) { x = (x ^ y) * 1099511628211ull; x ^= x >> 29; };
        mix(h.cls);
        mix(h.n_devices);
        for (uint32_t k = s->dev_ix.b(r); k < s->dev_ix.e(r); k++) mix(s->dev_groups[k].healthy);
        mix(v.drivers.size());
        for (auto& d : v.drivers) { mix(d.first); mix(d.second); }
        mix(v.net_modes.size());
        for (uint32_t mm : v.net_modes) mix(mm);
        mix(v.aliases.size());
        for (uint32_t al : v.aliases) mix(al);
        mix(v.volumes.size());
        for (auto& vv : v.volumes) { mix(vv.first); mix(vv.second); }
        return x;
    };
    // representatives of changed rows move to another member first: the first
    // unchanged member in row order (a scan from row 0 that stops once every
    // such class and signature has one)
    {
        std::unordered_set<uint32_t> need_cls, need_sig;
        for (uint32_t c = 0; c < (uint32_t)s->class_rep.size(); c++) {
            const uint32_t rep = s->class_rep[c];
            auto it = old_of.find(rep);
            if (rep < n_old && it != old_of.end() && it->second.first == c) need_cls.insert(c);
        }
        for (uint32_t g = 0; g < (uint32_t)s->sig_rep.size(); g++)
            if (changed(s->sig_rep[g])) need_sig.insert(g);
        if (!need_cls.empty() || !need_sig.empty()) {
            std::unordered_set<uint32_t> got_cls, got_sig;
            for (uint32_t r = 0; r < n_new && (got_cls.size() < need_cls.size() || got_sig.size() < need_sig.size()); r++) {
                if (changed(r)) continue;
                const uint32_t c = s->nodes[r].cls, g = s->nodes[r].sig;
                if (need_cls.count(c) && got_cls.insert(c).second) s->class_rep[c] = r;
                if (need_sig.count(g) && got_sig.insert(g).second) s->sig_rep[g] = r;
            }
            // a class with no member left keeps its representative index
            for (uint32_t g : need_sig) {
                if (got_sig.count(g)) continue;
                // no member left: out of its class and of the hash buckets (the
                // representative row index stays valid for the tables)
                auto& cs = s->class_sigs[s->sig_cls[g]];
                cs.erase(std::remove(cs.begin(), cs.end(), g), cs.end());
                auto& bk = s->sig_of[s->sig_hash[g]];
                bk.erase(std::remove(bk.begin(), bk.end(), g), bk.end());
            }
        }
    }
    for (uint32_t j = 0; j < m; j++) {
        const uint32_t i = order[j], r = target[i];
        HostNode& h = s->nodes[r];
        const uint64_t hv = sig_hash(r);
        auto& bucket = s->sig_of[hv];
        uint32_t found = PE_NONE;
        for (uint32_t sg : bucket)
            if (same_inputs(s->sig_rep[sg], r)) { found = sg; break; }
        if (found == PE_NONE) {
            found = (uint32_t)s->sig_rep.size();
            bucket.push_back(found);
            s->sig_rep.push_back(r);
            s->sig_cls.push_back(h.cls);
            s->sig_hash.push_back(hv);
            s->class_sigs[h.cls].push_back(found);
        }
        h.sig = found;
    }
    // a class whose representative left it (and had no other member then) takes
    // a member that joined it later
    {
        std::vector<uint32_t> stale;
        for (uint32_t c = 0; c < s->ncls; c++)
            if (s->nodes[s->class_rep[c]].cls != c) stale.push_back(c);
        if (!stale.empty()) {
            std::vector<uint32_t> first(s->ncls, PE_NONE);
            for (uint32_t r = 0; r < n_new; r++)
                if (first[s->nodes[r].cls] == PE_NONE) first[s->nodes[r].cls] = r;
            for (uint32_t c : stale)
                if (first[c] != PE_NONE) s->class_rep[c] = first[c];
        }
    }
    return PE_OK;
}

int build_state(pe_stack* s, const pe_node_table* nt, const pe_alloc_table* at) {
    s->nodes.clear();
    s->h_node_rec.clear();
    s->cls_of.clear();
    s->class_rep.clear();
    s->class_sigs.clear();
    s->sig_of.clear();
    s->sig_hash.clear();
    s->sig_rep.clear();
    s->sig_cls.clear();
    for (RowIndex* ix : {&s->attr_ix, &s->meta_ix, &s->drv_ix, &s->net_ix, &s->alias_ix, &s->hv_ix, &s->dev_ix})
        ix->clear();
    s->attr_kv.clear(); s->meta_kv.clear(); s->drv_kf.clear(); s->hv_kf.clear();
    s->net_mode_ids.clear(); s->alias_ids.clear();
    s->dev_groups.clear(); s->dev_attr.clear();
    s->dev_attr_dead = 0;
    s->n_dev_big = 0;
    s->max_dev_groups = 0;
    s->h_core_rsvable.clear(); s->h_core_avail.clear(); s->h_core_spc.clear(); s->h_core_bad.clear();
    s->n_core_bad = s->n_core_rows = 0;
    s->node_dnets.clear();
    s->n_multi_net = 0;
    std::vector<uint32_t> target(nt->n);
    for (uint32_t i = 0; i < nt->n; i++) target[i] = i;
    int rc = apply_nodes(s, nt, target, nt->n);
    if (rc) return rc;
    s->allocs.clear();
    s->alloc_dev.clear();
    s->alloc_ports.clear();
    s->net_other_dev = 0;
    rc = append_allocs(s, at, nullptr);
    if (rc) return rc;
    return build_alloc_state(s);
}

// Whether an alloc's bandwidth is on its node's first device network (the one
// the NodeRec keeps, NetworkIndex.UsedBandwidth[device]).
static inline bool on_first_dev(const pe_stack* s, const HostAlloc& a) {
    const uint32_t f = s->nodes[a.row].first_dev;
    return a.net_dev == PE_NONE || (f != PE_NONE && s->S(a.net_dev) == s->S(f));
}

// Allocations of a pe_alloc_table into the host mirror: appended, or, with
// `index`, written over existing entries (index[i] < allocs.size()) or
// appended (index[i] == PE_NONE).
int append_allocs(pe_stack* s, const pe_alloc_table* at, const uint32_t* index) {
    const uint32_t n = (uint32_t)s->nodes.size();
    for (uint32_t i = 0; at && i < at->count; i++) {
        const uint32_t row = at->node_row[i];
        if (row >= n) return s->fail(PE_EINVAL, "alloc node_row out of range");
        HostAlloc a{row, at->ns[i], at->job_id[i], at->task_group[i], at->terminal[i] != 0};
        a.priority = at->priority ? at->priority[i] : 0;
        a.max_parallel = at->max_parallel ? at->max_parallel[i] : 0;
        a.cpu = at->cpu_shares[i]; a.mem = at->memory_mb[i]; a.disk = at->disk_mb[i];
        a.mbits = at->net_mbits[i];
        a.dyn = at->dyn_ports[i];
        a.dev_begin = (uint32_t)s->alloc_dev.size();
        for (uint32_t k = at->dev_off ? at->dev_off[i] : 0; at->dev_off && k < at->dev_off[i + 1]; k++)
            s->alloc_dev.emplace_back(at->dev_group[k], at->dev_count[k]);
        a.dev_end = (uint32_t)s->alloc_dev.size();
        a.port_begin = (uint32_t)s->alloc_ports.size();
        for (uint32_t k = at->port_off ? at->port_off[i] : 0; at->port_off && k < at->port_off[i + 1]; k++)
            s->alloc_ports.emplace_back(at->port_ip[k], at->port_value[k]);
        a.port_end = (uint32_t)s->alloc_ports.size();
        a.has_net = at->has_network ? at->has_network[i] != 0 : (a.mbits > 0 || a.dyn > 0 || a.port_end > a.port_begin);
        if (at->net_device && at->net_device[i] != PE_NONE) {
            a.net_dev = at->net_device[i];
            if (a.has_net && (s->nodes[row].first_dev == PE_NONE || s->S(a.net_dev) != s->S(s->nodes[row].first_dev)))
                s->net_other_dev++;   // its bandwidth is not on the device the NodeRec keeps: a multi-device node
        }
        for (uint32_t k = at->core_off ? at->core_off[i] : 0; at->core_off && k < at->core_off[i + 1]; k++) {
            const uint16_t c = at->core_id[k];
            if (c >= 256) a.cores_beyond = true;
            else a.cores[c >> 6] |= 1ull << (c & 63);
        }
        const uint32_t at_index = index ? index[i] : PE_NONE;
        if (at_index == PE_NONE) {
            s->allocs.push_back(a);
        } else {
            if (at_index >= s->allocs.size()) return s->fail(PE_EINVAL, "alloc update index out of range");
            s->allocs[at_index] = a;
        }
    }
    return PE_OK;
}

// Everything derived from the snapshot's allocations: base proposed usage,
// device free counts, the Preemptor's per-node candidate lists.
constexpr uint8_t kRowOverheld = 1;   // device instances held beyond a group's healthy count
constexpr uint8_t kRowDevEnt = 2;     // an alloc's device entries beyond the packed 4 x 255
constexpr uint8_t kRowCoreOut = 4;    // allocs hold cores outside the node's available set

// The unsupported-snapshot reasons from the per-row counts, in the order the
// full build assigns them (the last assignment wins there).
static void alloc_state_reasons(pe_stack* s) {
    s->preempt_unsupported = s->n_row_devent ? "alloc device entries beyond 4 x 255"
                             : s->evict_too_many ? "more than 1024 allocs on a node"
                             : s->n_row_overheld ? "device instances held beyond the healthy count"
                                                 : "";
    s->cores_unsupported = s->n_row_core_out ? "allocs holding reserved cores outside the node's available set"
                                             : s->cores_unsup_allocs;
}

// Base record, device usage and Preemptor device fields of one row from the
// row's non-terminal allocs (slots h_node_alloc_off[r] .. [r + 1]); returns
// the row's kRow* flags. `slots_changed` collects the Preemptor slots whose
// device fields were rewritten (null: not needed).
static uint8_t alloc_row(pe_stack* s, uint32_t r, std::vector<uint32_t>* slots_changed) {
    uint8_t flags = 0;
    pe::NodeRec rec = s->h_node_rec[r];
    const uint32_t ng = s->dev_ix.n(r), g0 = s->dev_ix.b(r);
    int64_t used[pe::kMaxDevGroups + 1] = {0};
    std::vector<int64_t> used_big(ng > pe::kMaxDevGroups ? ng : 0, 0);
    int64_t* du = ng > pe::kMaxDevGroups ? used_big.data() : used;
    const uint32_t sb = r + 1 < s->h_node_alloc_off.size() ? s->h_node_alloc_off[r] : 0;
    const uint32_t se = r + 1 < s->h_node_alloc_off.size() ? s->h_node_alloc_off[r + 1] : 0;
    for (uint32_t slot = sb; slot < se; slot++) {
        const HostAlloc& a = s->allocs[s->h_palloc_index[slot]];
        rec.used_cpu += a.cpu;
        rec.used_mem += a.mem;
        rec.used_disk += a.disk;
        // UsedBandwidth of the NodeRec's device (the node's first); allocs on
        // another device make the node a multi-device one (build_md)
        if (on_first_dev(s, a)) rec.used_mbits += a.mbits;
        rec.used_dyn += a.dyn;
        pe::PreemptAlloc& x = s->h_palloc[slot];
        x.dev_g = x.dev_c = 0;
        x.n_dev = 0;
        for (uint32_t k = a.dev_begin; k < a.dev_end; k++) {
            const uint32_t g = s->alloc_dev[k].first, c = s->alloc_dev[k].second;
            if (g >= ng) continue;   // the group is no longer fingerprinted (devices.go:88-99)
            du[g] += c;
            if (x.n_dev >= 4 || g >= 4 || c > 255) { flags |= kRowDevEnt; continue; }
            x.dev_g |= g << (8 * x.n_dev);
            x.dev_c |= c << (8 * x.n_dev);
            x.n_dev++;
        }
        if (slots_changed) slots_changed->push_back(slot);
    }
    s->h_base_rec[r] = rec;
    uint32_t packed = 0;
    for (uint32_t k = 0; k < ng; k++) {
        const int64_t healthy = (int64_t)s->dev_groups[g0 + k].healthy;
        if (du[k] > healthy) flags |= kRowOverheld;
        if (s->dev_packable) packed |= (uint32_t)std::max<int64_t>(0, healthy - du[k]) << (8 * k);
    }
    s->h_dev_free[r] = packed;
    const uint64_t* u = &s->h_core_base[4 * (size_t)r];
    const uint64_t* av = r < s->h_core_avail.size() / 4 ? &s->h_core_avail[4 * (size_t)r] : nullptr;
    if (av && (av[0] | av[1] | av[2] | av[3]))
        for (int w = 0; w < 4; w++)
            if (u[w] & ~av[w]) flags |= kRowCoreOut;
    return flags;
}

static void count_row_flags(pe_stack* s, uint8_t f, int sign) {
    s->n_row_overheld += sign * ((f & kRowOverheld) != 0);
    s->n_row_devent += sign * ((f & kRowDevEnt) != 0);
    s->n_row_core_out += sign * ((f & kRowCoreOut) != 0);
}

// Everything derived from the snapshot's allocations: base proposed usage,
// device free counts, the Preemptor's per-node candidate lists.
int build_alloc_state(pe_stack* s) {
    const uint32_t n = (uint32_t)s->nodes.size();
    s->alloc_state_ok = false;
    {
        // compact the device-entry pool to the live allocs' ranges: entries
        // overwritten by pe_update_allocs leave dead ranges behind
        std::vector<std::pair<uint32_t, uint32_t>> live;
        live.reserve(s->alloc_dev.size());
        for (HostAlloc& a : s->allocs) {
            const uint32_t b = (uint32_t)live.size();
            for (uint32_t k = a.dev_begin; k < a.dev_end; k++) live.push_back(s->alloc_dev[k]);
            a.dev_begin = b;
            a.dev_end = (uint32_t)live.size();
        }
        s->alloc_dev.swap(live);
        std::vector<std::pair<uint32_t, int32_t>> lp;
        lp.reserve(s->alloc_ports.size());
        for (HostAlloc& a : s->allocs) {
            const uint32_t b = (uint32_t)lp.size();
            for (uint32_t k = a.port_begin; k < a.port_end; k++) lp.push_back(s->alloc_ports[k]);
            a.port_begin = b;
            a.port_end = (uint32_t)lp.size();
        }
        s->alloc_ports.swap(lp);
    }
    // non-terminal allocs per job (SetJob and the collision / property counts
    // touch only the job's own allocs)
    s->job_allocs.clear();
    for (uint32_t i = 0; i < (uint32_t)s->allocs.size(); i++)
        if (!s->allocs[i].terminal) s->job_allocs[s->allocs[i].job].push_back(i);
    // reserved cores held by the snapshot's allocs. Overlapping sets, or cores
    // outside a node's AllocsFit-available set, fail every AllocsFit on that
    // node ("cores", funcs.go:158-180): not modelled on the device.
    s->cores_unsup_allocs.clear();
    s->h_core_base.assign(4 * (size_t)n, 0);
    s->any_alloc_cores = false;
    for (const HostAlloc& a : s->allocs) {
        if (a.terminal) continue;
        if (a.cores_beyond) s->cores_unsup_allocs = "allocs holding core ids >= 256";
        uint64_t* u = &s->h_core_base[4 * (size_t)a.row];
        for (int w = 0; w < 4; w++) {
            if (!a.cores[w]) continue;
            s->any_alloc_cores = true;
            if (u[w] & a.cores[w]) s->cores_unsup_allocs = "allocs holding overlapping reserved cores";
            u[w] |= a.cores[w];
        }
    }
    // Preemptor inputs (preemption.go:96-154): non-terminal allocs per node in table order
    s->job_keys.clear();
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> jtg;
    std::vector<uint32_t> cnt(n + 1, 0);
    for (auto& a : s->allocs) if (!a.terminal) cnt[a.row + 1]++;
    s->h_node_alloc_off.assign(n + 1, 0);
    for (uint32_t i = 0; i < n; i++) s->h_node_alloc_off[i + 1] = s->h_node_alloc_off[i] + cnt[i + 1];
    const uint32_t m = s->h_node_alloc_off[n];
    s->h_palloc.assign(std::max<uint32_t>(m, 1), pe::PreemptAlloc{});
    std::memset(s->h_palloc.data(), 0, sizeof(pe::PreemptAlloc) * s->h_palloc.size());
    s->h_palloc_index.assign(m, 0);
    s->alloc_slot.assign(s->allocs.size(), PE_NONE);
    {
        std::vector<uint32_t> fill(s->h_node_alloc_off.begin(), s->h_node_alloc_off.end() - 1);
        uint32_t max_m = 0;
        for (uint32_t i = 0; i < n; i++) max_m = std::max(max_m, cnt[i + 1]);
        s->evict_words = max_m <= 32u ? 1u : max_m <= 256u ? 8u : 32u;
        s->evict_too_many = max_m > pe::kEvictMaxAllocs;
        for (uint32_t i = 0; i < s->allocs.size(); i++) {
            const HostAlloc& a = s->allocs[i];
            if (a.terminal) continue;
            const uint32_t slot = fill[a.row]++;
            s->h_palloc_index[slot] = i;
            s->alloc_slot[i] = slot;
            pe::PreemptAlloc& x = s->h_palloc[slot];
            x.cpu = a.cpu; x.mem = a.mem; x.disk = a.disk;
            x.priority = a.priority; x.max_parallel = a.max_parallel;
            x.job_key = s->job_keys.emplace(std::make_pair(a.job, a.ns), (uint32_t)s->job_keys.size()).first->second;
            x.jtg_key = jtg.emplace(std::make_tuple(a.job, a.ns, a.tg), (uint32_t)jtg.size()).first->second;
            // what a stop or eviction gives back to the NodeRec's device (the
            // node's first); other devices' bandwidth is the host's (build_md)
            x.mbits = on_first_dev(s, a) ? a.mbits : 0;
            x.dyn = a.dyn;
            x.state_index = i | (a.has_net ? pe::kAllocHasNet : 0u);
        }
    }
    // per row: base record, device free counts (DeviceAccounter, devices.go:25-100,
    // packed 4 x u8 per node), the Preemptor's device fields, the row reasons
    s->h_base_rec = s->h_node_rec;
    s->h_dev_free.assign(n, 0);
    s->row_flags.assign(n, 0);
    s->n_row_overheld = s->n_row_devent = s->n_row_core_out = 0;
    for (uint32_t r = 0; r < n; r++) {
        s->row_flags[r] = alloc_row(s, r, nullptr);
        count_row_flags(s, s->row_flags[r], +1);
    }
    alloc_state_reasons(s);
    HIP_TRY(s, upload_s(s, s->d_base_rec, s->h_base_rec));
    HIP_TRY(s, upload_s(s, s->d_rec, s->h_base_rec));
    HIP_TRY(s, upload_s(s, s->d_dev_free_base, s->h_dev_free));
    HIP_TRY(s, upload_s(s, s->d_dev_free, s->h_dev_free));
    s->n_jtg_keys = (uint32_t)jtg.size();
    s->h_preempted.assign(std::max<uint32_t>(m, 1), 0);
    HIP_TRY(s, upload_s(s, s->d_node_alloc_off, s->h_node_alloc_off));
    HIP_TRY(s, upload_s(s, s->d_palloc, s->h_palloc));
    HIP_TRY(s, upload_s(s, s->d_preempted, s->h_preempted));
    HIP_TRY(s, upload_s(s, s->d_pcount, std::vector<uint32_t>(std::max<uint32_t>(s->n_jtg_keys, 1), 0)));
    std::vector<uint32_t> zeros(n, 0);
    HIP_TRY(s, upload_s(s, s->d_coll_job, zeros));
    s->h_core_used = s->h_core_base;
    if (s->has_cores || s->any_alloc_cores) {
        if (!s->has_cores) {   // core sets on allocs only: empty reservable masks
            s->h_core_rsvable.assign(4 * (size_t)n, 0);
            s->h_core_avail.assign(4 * (size_t)n, 0);
            s->h_core_spc.assign(n, 0);
            s->has_cores = true;
        }
        HIP_TRY(s, upload_s(s, s->d_core_rsvable, s->h_core_rsvable));
        HIP_TRY(s, upload_s(s, s->d_core_avail, s->h_core_avail));
        HIP_TRY(s, upload_s(s, s->d_core_spc, s->h_core_spc));
        HIP_TRY(s, upload_s(s, s->d_core_base, s->h_core_base));
        HIP_TRY(s, upload_s(s, s->d_core_used, s->h_core_base));
        std::vector<uint64_t> pc(4 * (size_t)std::max<uint32_t>(m, 1), 0);
        for (uint32_t slot = 0; slot < m; slot++)
            for (int w = 0; w < 4; w++) pc[4 * (size_t)slot + w] = s->allocs[s->h_palloc_index[slot]].cores[w];
        HIP_TRY(s, upload_s(s, s->d_palloc_cores, pc));
    }
    s->alloc_state_ok = true;
    return PE_OK;
}

// Rows `rows` of a device array from its host mirror `h` (row_elems
// elements of T per row): one k_scatter_rows launch reading the staging ring,
// or the whole array when the payload does not fit the ring.
template <class T>
int patch_rows(pe_stack* s, DevMem& d, const std::vector<T>& h, const std::vector<uint32_t>& rows, size_t row_elems) {
    static_assert(sizeof(T) % 4 == 0, "rows of whole 4-byte words");
    if (rows.empty()) return PE_OK;
    const uint32_t words = (uint32_t)(row_elems * sizeof(T) / 4);
    std::vector<uint32_t> payload(rows.size() * (1 + (size_t)words));
    std::memcpy(payload.data(), rows.data(), rows.size() * 4);
    uint32_t* dst = payload.data() + rows.size();
    for (size_t i = 0; i < rows.size(); i++)
        std::memcpy(dst + i * words, &h[(size_t)rows[i] * row_elems], (size_t)words * 4);
    const unsigned char* staged = stage_only(s, payload);
    if (!staged) {
        HIP_TRY(s, upload_s(s, d, h));
        return PE_OK;
    }
    HIP_TRY(s, pe_launch_scatter_rows(d.p, words, staged, (uint32_t)rows.size(), s->stream));
    return PE_OK;
}

// pe_update_nodes' share of build_alloc_state. The snapshot's allocations did
// not change: only the changed rows and the appended ones (which hold no
// allocs yet) get their base records, device free counts, Preemptor device
// fields and row reasons recomputed, and the device arrays are grown (content
// kept) and patched row by row; the plan then resets as after ResetPlan. A
// property of the whole snapshot that changed with the update (the packed
// device column, reserved cores appearing or leaving) takes the full build.
int refresh_node_rows(pe_stack* s, std::vector<uint32_t> rows, uint32_t n_old, bool packable_before,
                      bool cores_before) {
    const uint32_t n = (uint32_t)s->nodes.size();
    s->has_cores = s->has_cores || s->any_alloc_cores;
    static const bool force_full = getenv("PE_UPDATE_FULL") != nullptr;   // A/B against the full build
    if (force_full || !s->alloc_state_ok || s->h_node_alloc_off.size() != (size_t)n_old + 1 ||
        s->dev_packable != packable_before || s->has_cores != cores_before)
        return build_alloc_state(s);
    for (uint32_t r = n_old; r < n; r++) rows.push_back(r);
    std::sort(rows.begin(), rows.end());
    const uint32_t m = s->h_node_alloc_off[n_old];
    s->h_node_alloc_off.resize((size_t)n + 1, m);
    s->h_base_rec.resize(n);
    s->h_dev_free.resize(n, 0);
    s->row_flags.resize(n, 0);
    s->h_core_base.resize(4 * (size_t)n, 0);
    std::vector<uint32_t> slots;
    for (uint32_t r : rows) {
        count_row_flags(s, s->row_flags[r], -1);
        s->row_flags[r] = alloc_row(s, r, &slots);
        count_row_flags(s, s->row_flags[r], +1);
    }
    alloc_state_reasons(s);
    auto grow = [&](DevMem& d, size_t row_bytes, size_t extra) {
        return d.grow(row_bytes * n + extra, row_bytes * n_old + extra, s->stream);
    };
    HIP_TRY(s, grow(s->d_base_rec, sizeof(pe::NodeRec), 0));
    HIP_TRY(s, grow(s->d_rec, sizeof(pe::NodeRec), 0));
    HIP_TRY(s, grow(s->d_dev_free_base, 4, 0));
    HIP_TRY(s, grow(s->d_dev_free, 4, 0));
    HIP_TRY(s, grow(s->d_node_alloc_off, 4, 4));
    HIP_TRY(s, grow(s->d_coll_job, 4, 0));
    int rc;
    // the working copies too: a launch that reads node fields (class, capacity)
    // may run before the deferred reset copy lands
    if ((rc = patch_rows(s, s->d_base_rec, s->h_base_rec, rows, 1))) return rc;
    if ((rc = patch_rows(s, s->d_rec, s->h_base_rec, rows, 1))) return rc;
    if ((rc = patch_rows(s, s->d_dev_free_base, s->h_dev_free, rows, 1))) return rc;
    if ((rc = patch_rows(s, s->d_dev_free, s->h_dev_free, rows, 1))) return rc;
    if ((rc = patch_rows(s, s->d_palloc, s->h_palloc, slots, 1))) return rc;
    std::vector<uint32_t> tail;   // node_alloc_off entries of the appended rows
    for (uint32_t r = n_old; r < n; r++) tail.push_back(r + 1);
    if ((rc = patch_rows(s, s->d_node_alloc_off, s->h_node_alloc_off, tail, 1))) return rc;
    HIP_TRY(s, hipMemsetAsync(s->d_coll_job.p, 0, 4 * (size_t)n, s->stream));
    if (s->has_cores) {
        HIP_TRY(s, grow(s->d_core_rsvable, 32, 0));
        HIP_TRY(s, grow(s->d_core_avail, 32, 0));
        HIP_TRY(s, grow(s->d_core_spc, 8, 0));
        HIP_TRY(s, grow(s->d_core_base, 32, 0));
        HIP_TRY(s, grow(s->d_core_used, 32, 0));
        if ((rc = patch_rows(s, s->d_core_rsvable, s->h_core_rsvable, rows, 4))) return rc;
        if ((rc = patch_rows(s, s->d_core_avail, s->h_core_avail, rows, 4))) return rc;
        if ((rc = patch_rows(s, s->d_core_spc, s->h_core_spc, rows, 1))) return rc;
        std::vector<uint32_t> app(rows.end() - (n - n_old), rows.end());
        if ((rc = patch_rows(s, s->d_core_base, s->h_core_base, app, 4))) return rc;
        s->h_core_used = s->h_core_base;
        HIP_TRY(s, hipMemcpyAsync(s->d_core_used.p, s->d_core_base.p, 32 * (size_t)n, hipMemcpyDeviceToDevice, s->stream));
    }
    // a new evaluation context: the deferred ResetPlan copy (rec <- base,
    // free counts <- base, preempted / pcount zero) runs before the next launch
    std::fill(s->h_preempted.begin(), s->h_preempted.end(), 0);
    s->reset_pending = true;
    s->offer_row = -1;
    return PE_OK;
}

// Task groups of the previous job go to a small pool; a new one takes a
// retired group's device buffers (same stream: later uploads are ordered after
// the kernels that read them).
void retire_tgs(pe_stack* s) {
    for (auto& g : s->tgs)
        if (s->tg_pool.size() < 16) s->tg_pool.push_back(std::move(g));
    s->tgs.clear();
}

std::unique_ptr<TgPlan> new_tg(pe_stack* s) {
    auto g = std::make_unique<TgPlan>();
    if (s->tg_pool.empty()) return g;
    std::unique_ptr<TgPlan> old = std::move(s->tg_pool.back());
    s->tg_pool.pop_back();
    auto take = [](DevMem& dst, DevMem& src) { std::swap(dst.p, src.p); std::swap(dst.bytes, src.bytes); };
    take(g->class_ok, old->class_ok);
    take(g->node_ok, old->node_ok);
    take(g->class_aff, old->class_aff);
    take(g->node_aff, old->node_aff);
    take(g->alias_ok, old->alias_ok);
    g->alias_for = old->alias_for;
    g->alias_gen = old->alias_gen;
    take(g->coll_tg, old->coll_tg);
    take(g->dev_cls, old->dev_cls);
    take(g->class_ok_batch, old->class_ok_batch);
    take(g->node_feas, old->node_feas);
    take(g->node_aux, old->node_aux);
    take(g->aff_vals, old->aff_vals);
    take(g->aff_idx, old->aff_idx);
    take(g->static_gate, old->static_gate);
    take(g->static_blocked, old->static_blocked);
    return g;
}

// Why the group's static ports cannot go on `row` under the current plan
// (AssignPorts, network.go:317-363; the reference's error text in *why), or
// false when they fit. The used ports of an address: the node's reservations
// for its IP, ReservedHostPorts, the ports the proposed snapshot allocs hold
// on it (plan stops and preemptions excluded).
bool static_port_reason(pe_stack* s, const TgPlan& g, uint32_t row, std::string* why, uint32_t excl = 0) {
    const HostAddr* ad = nullptr;
    if (row < s->node_addrs.size())
        for (const HostAddr& a : s->node_addrs[row]) if (a.alias == g.net_host) { ad = &a; break; }
    for (const auto& rp : g.rports) {
        if (!ad) {
            if (why) *why = "no addresses available for \"" + s->S(g.net_host) + "\" network";
            return true;
        }
        if (rp.first < 0 || rp.first >= 65536) {
            if (why) *why = "invalid port " + std::to_string(rp.first) + " (out of range)";
            return true;
        }
        bool used = false;
        for (const HostAddr& a : s->node_addrs[row])
            if (a.ip == ad->ip) used = used || std::binary_search(a.reserved.begin(), a.reserved.end(), rp.first);
        if (row < s->node_rhp.size())
            used = used || std::binary_search(s->node_rhp[row].begin(), s->node_rhp[row].end(), rp.first);
        for (uint32_t k = s->h_node_alloc_off[row]; k < s->h_node_alloc_off[row + 1] && !used; k++) {
            if (s->h_preempted[k]) continue;   // a plan stop (2) or preemption (1)
            const uint32_t rel = k - s->h_node_alloc_off[row];
            if (rel < 32 && ((excl >> rel) & 1u)) continue;   // preempted by the Select being evaluated
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            for (uint32_t q = a.port_begin; q < a.port_end; q++)
                used = used || (s->alloc_ports[q].first == ad->ip && s->alloc_ports[q].second == rp.first);
        }
        if (used) {
            if (why) *why = "reserved port collision " + (rp.second == PE_NONE ? std::string() : s->S(rp.second)) + "=" +
                            std::to_string(rp.first);
            return true;
        }
    }
    return false;
}

// The collision text when the group's own placement holds the ports (its first static port).
std::string static_port_collision(pe_stack* s, const TgPlan& g) {
    const auto& ports = g.rports.empty() ? g.trports : g.rports;
    if (ports.empty()) return "reserved port collision";
    const auto& rp = ports.front();
    return "reserved port collision " + (rp.second == PE_NONE ? std::string() : s->S(rp.second)) + "=" +
           std::to_string(rp.first);
}

// AssignNetwork's ReservedPorts check (network.go:407-442) for the task
// network's static ports on the node's one device network: the address yieldIP
// gives from its CIDR. UsedPorts[ip] holds the ReservedPorts of node addresses
// with that IP, ReservedHostPorts when the IP is a key SetNode created (the
// network's IP field or an address, network.go:92-141, 238-265), and the ports
// the proposed allocs hold on it (minus `excl`, CSR-relative).
bool task_port_reason(pe_stack* s, const TgPlan& g, uint32_t row, std::string* why, uint32_t excl = 0) {
    const HostNode& h = s->nodes[row];
    if (h.n_device_nets == 0 || g.trports.empty()) return false;   // "no networks available" is the device's
    const uint32_t ip = h.first_yield;
    bool keyed = ip == h.first_ipfield;
    if (row < s->node_addrs.size())
        for (const HostAddr& a : s->node_addrs[row]) keyed = keyed || a.ip == ip;
    for (const auto& rp : g.trports) {
        if (rp.first < 0 || rp.first >= 65536) {
            if (why) *why = "invalid port " + std::to_string(rp.first) + " (out of range)";
            return true;
        }
        bool used = false;
        if (row < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[row])
                if (a.ip == ip) used = used || std::binary_search(a.reserved.begin(), a.reserved.end(), rp.first);
        if (keyed && row < s->node_rhp.size())
            used = used || std::binary_search(s->node_rhp[row].begin(), s->node_rhp[row].end(), rp.first);
        for (uint32_t k = s->h_node_alloc_off[row]; k < s->h_node_alloc_off[row + 1] && !used; k++) {
            if (s->h_preempted[k]) continue;
            const uint32_t rel = k - s->h_node_alloc_off[row];
            if (rel < 32 && ((excl >> rel) & 1u)) continue;
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            for (uint32_t q = a.port_begin; q < a.port_end; q++)
                used = used || (s->alloc_ports[q].first == ip && s->alloc_ports[q].second == rp.first);
        }
        if (used) {
            if (why) *why = "reserved port collision " + (rp.second == PE_NONE ? std::string() : s->S(rp.second)) + "=" +
                            std::to_string(rp.first);
            return true;
        }
    }
    return false;
}

// PreemptForNetwork's reserved-port step (preemption.go:302-342) for the
// static ask of `g` on one node, as the device's preempt_for_network consumes
// it: candidates are the node's proposed state allocs outside the job;
// usedPortToAlloc maps every ReservedPorts value of a preemptible candidate with
// a network to its last holder in candidate order, filteredReservedPorts the
// values of the others with a network. Then whether the static ports still
// collide once the listed holders leave (node reservations, remaining allocs,
// this group's own placements).
// The static ports' blockers on the node for the retried offer: allocs of the
// node (CSR-relative bits) that hold a needed port on the address the ask
// takes, and whether anything that no preemption removes blocks one (a node
// reservation, an invalid port, no address, an alloc of the job itself).
// The blockers are returned as a list of up to 8 CSR-relative indices, one
// byte each (0xFF ends it); *overflow when more allocs block.
static uint64_t port_blockers(pe_stack* s, const TgPlan& g, uint32_t row, bool* permanent, bool* overflow) {
    *permanent = false;
    *overflow = false;
    const bool task = g.rports.empty();
    uint32_t ip = PE_NONE;
    bool keyed = true;   // ReservedHostPorts apply (always for an address)
    if (task) {
        const HostNode& h = s->nodes[row];
        if (h.n_device_nets == 0) return ~0ull;
        ip = h.first_yield;
        keyed = ip == h.first_ipfield;
        if (row < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[row]) keyed = keyed || a.ip == ip;
    } else {
        if (row < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[row]) if (a.alias == g.net_host) { ip = a.ip; break; }
        if (ip == PE_NONE) { *permanent = true; return ~0ull; }
    }
    const auto& ports = task ? g.trports : g.rports;
    const uint32_t b = s->h_node_alloc_off[row], e = s->h_node_alloc_off[row + 1];
    std::vector<uint32_t> blk;
    for (const auto& rp : ports) {
        if (rp.first < 0 || rp.first >= 65536) { *permanent = true; continue; }
        if (row < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[row])
                if (a.ip == ip && std::binary_search(a.reserved.begin(), a.reserved.end(), rp.first)) *permanent = true;
        if (keyed && row < s->node_rhp.size() &&
            std::binary_search(s->node_rhp[row].begin(), s->node_rhp[row].end(), rp.first))
            *permanent = true;
        for (uint32_t k = b; k < e; k++) {
            if (s->h_preempted[k]) continue;
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            bool holds = false;
            for (uint32_t q = a.port_begin; q < a.port_end; q++)
                holds = holds || (s->alloc_ports[q].first == ip && s->alloc_ports[q].second == rp.first);
            if (!holds) continue;
            if (a.job == s->job_id && a.ns == s->job_ns) *permanent = true;
            else if (std::find(blk.begin(), blk.end(), k - b) == blk.end()) blk.push_back(k - b);
        }
    }
    if (blk.size() > 8) {
        *overflow = true;
        return ~0ull;
    }
    std::sort(blk.begin(), blk.end());
    uint64_t list = ~0ull;
    for (size_t i = 0; i < blk.size(); i++) list = (list & ~(0xFFull << (8 * i))) | ((uint64_t)blk[i] << (8 * i));
    return list;
}

// ---- multi-device nodes (TgTables::md) -------------------------------------
// A task network ask on a snapshot where some node has several device
// networks, or allocs on a device other than its first: those nodes' outcome
// comes from the host (engine_types.h MdNet). The per-node dynamic-port count
// stays node-wide, as on every other node.
static inline bool tg_md(const pe_stack* s, const TgPlan& g) {
    return g.ask.has_task_net > 0 && (s->n_multi_net > 0 || s->net_other_dev > 0);
}

// A node's AvailNetworks (the device networks) in node order.
static void node_nets(const pe_stack* s, uint32_t r, std::vector<HostNet>& out) {
    out.clear();
    if (r < s->node_dnets.size() && !s->node_dnets[r].empty()) { out = s->node_dnets[r]; return; }
    const HostNode& h = s->nodes[r];
    if (h.n_device_nets) out.push_back(HostNet{h.first_dev, h.first_ipfield, h.first_yield, h.first_mbits});
}

static inline uint32_t canon(const pe_stack* s, uint32_t id) {
    if (id == PE_NONE) return PE_NONE;
    const uint32_t c = s->lookup(s->S(id));
    return c == PE_NONE ? id : c;
}

// One node's NetworkIndex for the group's AssignNetwork (network.go:92-230,
// 407-482): its AvailNetworks in node order, AvailBandwidth / UsedBandwidth
// per device, the node-wide dynamic-range count, and the ports the plan's
// placements hold; `removed` marks CSR-relative allocs PreemptForNetwork took
// out of the proposed list.
struct MdIndex {
    pe_stack* s = nullptr;
    const TgPlan* g = nullptr;
    uint32_t row = 0, b = 0, e = 0;
    std::vector<HostNet> nets;
    std::vector<uint32_t> dev;                          // canonical device of each network
    std::vector<std::pair<uint32_t, int32_t>> avail, used;
    int32_t dyn = 0;
    std::vector<std::pair<uint32_t, int32_t>> extra;    // (ip, port) held by plan placements
    std::vector<uint8_t> removed;
    uint32_t alias_ip = PE_NONE;                        // the group network's address (its static ports)

    int32_t& used_of(uint32_t d) {
        for (auto& u : used) if (u.first == d) return u.second;
        used.emplace_back(d, 0);
        return used.back().second;
    }
    int32_t avail_of(uint32_t d) const {
        for (auto& u : avail) if (u.first == d) return u.second;
        return 0;
    }
    uint32_t alloc_dev(const HostAlloc& a) const {
        return a.net_dev == PE_NONE ? canon(s, s->nodes[row].first_dev) : canon(s, a.net_dev);
    }
    // UsedPorts[ip] (network.go:54-70, 92-141, 238-293): address reservations
    // of that IP, ReservedHostPorts on the keys SetNode made (the networks' IP
    // fields and the addresses), the proposed allocs' ports, the plan's.
    bool port_used(uint32_t ip, int32_t v) const {
        bool keyed = false;
        for (const HostNet& nw : nets) keyed = keyed || nw.ipfield == ip;
        if (row < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[row])
                if (a.ip == ip) {
                    keyed = true;
                    if (std::binary_search(a.reserved.begin(), a.reserved.end(), v)) return true;
                }
        if (keyed && row < s->node_rhp.size() && std::binary_search(s->node_rhp[row].begin(), s->node_rhp[row].end(), v))
            return true;
        for (uint32_t k = b; k < e; k++) {
            if (s->h_preempted[k] || removed[k - b]) continue;
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            for (uint32_t q = a.port_begin; q < a.port_end; q++)
                if (s->alloc_ports[q].first == ip && s->alloc_ports[q].second == v) return true;
        }
        for (auto& x : extra) if (x.first == ip && x.second == v) return true;
        return false;
    }
    // One AssignNetwork (yieldIP over the networks, one address each):
    // bandwidth, the ask's ReservedPorts on the address, the dynamic ports.
    // The refusal is the last network's (err is overwritten per address).
    bool assign(int32_t idx_dyn, int* choice, uint32_t* code) const {
        const pe::Ask& a = g->ask;
        *code = pe::kTrNoNetworks;
        for (size_t i = 0; i < nets.size(); i++) {
            int32_t u = 0;
            for (auto& x : used) if (x.first == dev[i]) u = x.second;
            if (u + a.task_mbits > avail_of(dev[i])) { *code = pe::kTrBandwidth; continue; }
            bool bad = false;
            for (size_t q = 0; q < g->trports.size() && !bad; q++) {
                const int32_t v = g->trports[q].first;
                if (v < 0 || v >= 65536) {
                    *code = pe::kTrTaskStatic | pe::kMdCoded | pe::kMdInvalidPort | ((uint32_t)q << 8);
                    bad = true;
                } else if (port_used(nets[i].yield, v)) {
                    *code = pe::kTrTaskStatic | pe::kMdCoded | ((uint32_t)q << 8);
                    bad = true;
                }
            }
            if (bad) continue;
            if (pe::kDynPortCapacity - idx_dyn < a.task_dyn) { *code = pe::kTrTaskDyn; continue; }
            *choice = (int)i;
            return true;
        }
        return false;
    }
    // What one placement of the group leaves in the index for the next
    // (NetworkIndex.AddAllocs of the placed alloc, network.go:144-193): the
    // group ports when the group network has ports, else the task network's
    // bandwidth and ports on the device it took.
    void apply(int choice) {
        const pe::Ask& a = g->ask;
        const bool shared = g->has_network && g->net_ports > 0;
        if (a.commit_mbits) used_of(dev[(size_t)choice]) += a.commit_mbits;
        dyn += a.commit_dyn;
        if (!shared) {
            for (auto& rp : g->trports) extra.emplace_back(nets[(size_t)choice].yield, rp.first);
        } else {
            for (auto& rp : g->rports) extra.emplace_back(alias_ip, rp.first);
        }
    }
};

// Whether `row` is a multi-device node: several device networks, or an alloc
// with bandwidth held on a device other than the first.
static bool md_node(const pe_stack* s, uint32_t row) {
    if (s->nodes[row].n_device_nets > 1) return true;
    if (!s->net_other_dev) return false;
    const uint32_t first = canon(s, s->nodes[row].first_dev);
    for (uint32_t k = s->h_node_alloc_off[row]; k < s->h_node_alloc_off[row + 1]; k++) {
        if (s->h_preempted[k]) continue;
        const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
        if (a.has_net && a.net_dev != PE_NONE && canon(s, a.net_dev) != first) return true;
    }
    return false;
}

// Go 1.16 sort.Slice over CSR-relative indices by a precomputed key.
static void go_sort_by(std::vector<uint32_t>& v, const std::vector<double>& key) {
    struct Less {
        const double* k;
        bool operator()(uint32_t x, uint32_t y) const { return k[x] < k[y]; }
    };
    if (!v.empty()) pe::go_sort(v.data(), (int)v.size(), Less{key.data()});
}

// PreemptForNetwork (preemption.go:270-455) for the task network's ask on a
// multi-device node, then the retried AssignNetwork; the same steps as the
// device's preempt_for_network (evict.inc), with the candidates grouped by
// device. Fills the MdNet's ev / pre and *choice (kMdPre).
static void md_preempt(const MdIndex& x0, const std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int>& pcount,
                       pe::MdNet* m, int* choice) {
    pe_stack* s = x0.s;
    const TgPlan& g = *x0.g;
    const int32_t needed = g.ask.task_mbits;
    std::vector<uint32_t> lst;
    std::map<uint32_t, std::set<int32_t>> filtered;
    std::set<uint32_t> devs;
    for (uint32_t k = x0.b; k < x0.e; k++) {
        if (s->h_preempted[k]) continue;
        const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
        if ((a.job == s->job_id && a.ns == s->job_ns) || !a.has_net) continue;   // SetCandidates; Networks[0]
        const uint32_t d = x0.alloc_dev(a);
        if (s->job_priority - a.priority < 10) {
            for (uint32_t q = a.port_begin; q < a.port_end; q++) filtered[d].insert(s->alloc_ports[q].second);
            continue;
        }
        devs.insert(d);
        lst.push_back(k - x0.b);
    }
    m->ev = pe::kMdSkip;
    if (devs.empty()) return;
    if (devs.size() > 1) { m->ev = pe::kMdUnsup; return; }   // deviceToAllocs in Go map order
    const uint32_t D = *devs.begin();
    const int32_t total = x0.avail_of(D);
    if (total < needed) return;
    int32_t used_d = 0;
    for (auto& u : x0.used) if (u.first == D) used_d = u.second;
    const int32_t free_bw = total - used_d;
    auto al = [&](uint32_t rel) -> const HostAlloc& { return s->allocs[s->h_palloc_index[x0.b + rel]]; };
    std::vector<uint32_t> pre;
    int32_t pbw = 0;
    if (!g.trports.empty()) {   // the reserved ports first (preemption.go:309-342)
        std::map<int32_t, uint32_t> holder;
        for (uint32_t rel : lst) {
            const HostAlloc& a = al(rel);
            for (uint32_t q = a.port_begin; q < a.port_end; q++) holder[s->alloc_ports[q].second] = rel;
        }
        for (auto& rp : g.trports) {
            auto it = holder.find(rp.first);
            if (it != holder.end()) {
                if (std::find(pre.begin(), pre.end(), it->second) != pre.end()) { m->ev = pe::kMdUnsup; return; }
                pbw += al(it->second).mbits;
                pre.push_back(it->second);
            } else if (filtered[D].count(rp.first)) {
                return;   // a higher-priority alloc holds it: the next device, and there is none
            }
        }
        size_t n = lst.size();   // RemoveAllocs: swap with the last
        for (size_t i = 0; i < n; i++)
            if (std::find(pre.begin(), pre.end(), lst[i]) != pre.end()) { lst[i] = lst[n - 1]; i--; n--; }
        lst.resize(n);
    }
    std::vector<double> key(x0.e - x0.b, 0.0);
    const double dn = (double)needed;
    auto dist = [&](uint32_t rel) { return std::fabs((double)((int64_t)needed - al(rel).mbits) / dn); };
    bool met = pbw + free_bw >= needed;
    for (int64_t after = INT64_MIN; !met;) {   // filterAndGroupPreemptibleAllocs: priorities ascending
        int64_t pr = INT64_MAX;
        for (uint32_t rel : lst) if (al(rel).priority > after && al(rel).priority < pr) pr = al(rel).priority;
        if (pr == INT64_MAX) break;
        after = pr;
        std::vector<uint32_t> v;
        for (uint32_t rel : lst) if (al(rel).priority == pr) v.push_back(rel);
        for (uint32_t rel : v) {   // scoreForNetwork (preemption.go:653-660)
            const HostAlloc& a = al(rel);
            auto it = pcount.find(std::make_tuple(a.job, a.ns, a.tg));
            const int num = it == pcount.end() ? 0 : it->second;
            double pen = 0.0;
            if (a.max_parallel > 0 && num >= a.max_parallel) pen = (double)((num + 1) - a.max_parallel) * 50.0;
            key[rel] = dist(rel) + pen;
        }
        go_sort_by(v, key);
        for (uint32_t rel : v) {
            pbw += al(rel).mbits;
            pre.push_back(rel);
            if (pbw + free_bw >= needed) { met = true; break; }
        }
    }
    if (!met || pre.empty()) return;
    for (uint32_t rel : pre) key[rel] = -dist(rel);   // filterSuperset: distance descending
    go_sort_by(pre, key);
    int32_t avail = free_bw;
    std::vector<uint32_t> out;
    for (uint32_t rel : pre) {
        out.push_back(rel);
        avail += al(rel).mbits;
        if (avail != 0 && needed != 0 && avail >= needed) break;
    }
    if (out.size() > 8 || *std::max_element(out.begin(), out.end()) > 254u) { m->ev = pe::kMdUnsup; return; }
    // the retried AssignNetwork on a fresh index of the remaining allocs: the
    // group's port offer is not in it (rank.go:362-371)
    MdIndex x1 = x0;
    for (uint32_t rel : out) {
        const HostAlloc& a = al(rel);
        x1.removed[rel] = 1;
        if (a.mbits) x1.used_of(x1.alloc_dev(a)) -= a.mbits;
        x1.dyn -= a.dyn;
    }
    uint32_t code;
    if (!x1.assign(x1.dyn, choice, &code)) return;
    m->ev = pe::kMdPre;
    m->n_pre = (uint8_t)out.size();
    m->pre = ~0ull;
    for (size_t i = 0; i < out.size(); i++) m->pre = (m->pre & ~(0xFFull << (8 * i))) | ((uint64_t)out[i] << (8 * i));
}

// The group's MdNet per node (TgTables::md) from the host mirror: the plan's
// placements of the group replayed onto the devices they took (md_hist),
// then first fit for the admitted count, the first refusal's reason, and the
// Preempt Select's verdict.
static int build_md(pe_stack* s, TgPlan& g) {
    const uint32_t n = (uint32_t)s->nodes.size();
    std::vector<pe::MdNet> md(n);
    for (auto& m : md) { std::memset(&m, 0, sizeof(m)); m.lim = ~0u; }
    std::unordered_map<uint32_t, uint32_t> own;                 // row -> the group's plan placements
    std::unordered_map<uint32_t, int32_t> other_dyn;            // row -> other groups' placements' ports
    g.md_other = 0;
    for (auto& p : plan_of(s)) {
        if (p.second >= n) continue;
        if (p.first == g.name) { own[p.second]++; continue; }
        g.md_other++;
        for (auto& t : s->tgs)
            if (t->name == p.first) { other_dyn[p.second] += t->ask.commit_dyn; break; }
    }
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int> pcount;   // Plan.NodePreemptions per job / group
    for (size_t k = 0; k < s->h_preempted.size() && k < s->h_palloc_index.size(); k++)
        if (s->h_preempted[k] == 1) {
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            pcount[std::make_tuple(a.job, a.ns, a.tg)]++;
        }
    std::unordered_map<uint32_t, uint8_t> vdev;
    vdev.swap(g.md_vdev);
    for (auto it = g.md_hist.begin(); it != g.md_hist.end();) {   // popped or reset plans
        auto o = own.find(it->first);
        const size_t keep = o == own.end() ? 0 : o->second;
        if (it->second.size() > keep) it->second.resize(keep);
        if (it->second.empty()) it = g.md_hist.erase(it);
        else ++it;
    }
    const int32_t tg_part = g.ask.tg_dyn > 0 ? g.ask.tg_dyn + g.ask.static_dyn : 0;
    const bool changes = g.ask.commit_mbits != 0 || g.ask.commit_dyn != 0 ||
                         (g.has_network && g.net_ports > 0 ? !g.rports.empty() : !g.trports.empty());
    for (uint32_t r = 0; r < n; r++) {
        if (!md_node(s, r)) continue;
        MdIndex x;
        x.s = s;
        x.g = &g;
        x.row = r;
        x.b = s->h_node_alloc_off[r];
        x.e = s->h_node_alloc_off[r + 1];
        x.removed.assign(x.e - x.b, 0);
        node_nets(s, r, x.nets);
        for (const HostNet& nw : x.nets) {
            const uint32_t d = canon(s, nw.dev);
            x.dev.push_back(d);
            bool found = false;   // AvailBandwidth[device]: the last network naming it
            for (auto& a : x.avail) if (a.first == d) { a.second = nw.mbits; found = true; }
            if (!found) x.avail.emplace_back(d, nw.mbits);
        }
        if (r < s->node_addrs.size())
            for (const HostAddr& a : s->node_addrs[r]) if (a.alias == g.net_host) { x.alias_ip = a.ip; break; }
        x.dyn = s->h_base_rec[r].used_dyn;
        for (uint32_t k = x.b; k < x.e; k++) {
            const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
            if (s->h_preempted[k]) { x.dyn -= a.dyn; continue; }
            if (a.mbits) x.used_of(x.alloc_dev(a)) += a.mbits;
        }
        {
            auto od = other_dyn.find(r);
            if (od != other_dyn.end()) x.dyn += od->second;
        }
        // the group's placements on the node, in plan order, on the devices they took
        auto o = own.find(r);
        const uint32_t placed = o == own.end() ? 0u : o->second;
        std::vector<uint8_t>& hist = g.md_hist[r];
        for (uint32_t j = 0; j < placed; j++) {
            if (j == hist.size()) {
                int ch = -1;
                uint32_t code;
                auto v = vdev.find(r);
                if (v != vdev.end() && v->second < x.nets.size()) { ch = v->second; vdev.erase(v); }
                else if (!x.assign(x.dyn + tg_part, &ch, &code)) ch = -1;
                if (ch < 0) return s->fail(PE_EUNSUPPORTED, "a placement's network device on a multi-device node is unknown");
                hist.push_back((uint8_t)ch);
            }
            x.apply(hist[j]);
        }
        if (hist.empty()) g.md_hist.erase(r);
        pe::MdNet& m = md[r];
        // the Preempt Select's verdict (built on this state; the Select rebuilds)
        int ch0 = -1;
        uint32_t code0 = 0;
        if (x.assign(x.dyn + tg_part, &ch0, &code0)) {
            m.ev = pe::kMdFit;
            g.md_vdev[r] = (uint8_t)ch0;
        } else {
            int chp = -1;
            md_preempt(x, pcount, &m, &chp);
            if (m.ev == pe::kMdPre) g.md_vdev[r] = (uint8_t)chp;
        }
        // first fit for the plain Selects: placements admitted, the refusal after
        uint32_t slots = 0, code = 0;
        MdIndex y = x;
        for (;;) {
            int ch;
            if (!y.assign(y.dyn + tg_part, &ch, &code)) break;
            if (!changes || slots + 1 >= pe::kMdUnbounded - 1) { slots = pe::kMdUnbounded; break; }
            slots++;
            y.apply(ch);
        }
        m.lim = slots;
        m.code = code;
    }
    HIP_TRY(s, upload_s(s, g.md_dev, md));
    HIP_TRY_STATE(s, pe_launch_md_gate(g.md_dev.as<pe::MdNet>(), g.coll_tg.as<uint32_t>(), n, s->stream));
    g.md_on = true;
    return PE_OK;
}

static void port_step(pe_stack* s, const TgPlan& g, uint32_t row, bool own_placed, uint64_t* list, uint8_t* info,
                      uint64_t* blockers) {
    *list = ~0ull;
    *info = 0;
    *blockers = ~0ull;
    const auto& ports = g.rports.empty() ? g.trports : g.rports;
    const uint32_t b = s->h_node_alloc_off[row], e = s->h_node_alloc_off[row + 1];
    // the holder and blocker lists hold one-byte CSR-relative indices (the
    // widest eviction width covers 256 allocs)
    if (e - b > 255u) { *info = pe::kPortUnsup; return; }
    std::map<int32_t, uint32_t> holder;
    std::set<int32_t> filtered;
    for (uint32_t k = b; k < e; k++) {
        if (s->h_preempted[k]) continue;
        const HostAlloc& a = s->allocs[s->h_palloc_index[k]];
        if ((a.job == s->job_id && a.ns == s->job_ns) || !a.has_net) continue;
        const bool pre = s->job_priority - a.priority >= 10;
        for (uint32_t q = a.port_begin; q < a.port_end; q++) {
            if (pre) holder[s->alloc_ports[q].second] = k - b;
            else filtered.insert(s->alloc_ports[q].second);
        }
    }
    uint32_t n = 0;
    std::vector<bool> listed(e - b, false);
    for (const auto& rp : ports) {
        auto it = holder.find(rp.first);
        if (it != holder.end()) {
            if (listed[it->second] || n >= 8) { *info = pe::kPortUnsup; return; }
            listed[it->second] = true;
            *list = (*list & ~(0xFFull << (8 * n))) | ((uint64_t)it->second << (8 * n));
            n++;
        } else if (filtered.count(rp.first)) {
            *info = pe::kPortFail;
            return;
        }
    }
    bool permanent = false, overflow = false;
    *blockers = port_blockers(s, g, row, &permanent, &overflow);
    if (overflow) { *info = pe::kPortUnsup; return; }
    *info = (uint8_t)(n | ((own_placed || permanent) ? pe::kPortBlocked : 0u));
}

// Static port gates follow ProposedAllocs: stops and evictions free ports.
void invalidate_static(pe_stack* s) {
    for (auto& g : s->tgs) if (has_static(*g) || g->md_on) g->tables_valid = false;
}

pe::NodeSoA soa_of(pe_stack* s) {
    pe::NodeSoA a;
    a.n = (uint32_t)s->nodes.size();
    a.rec = s->d_rec.as<pe::NodeRec>();
    a.coll_job = s->d_coll_job.as<uint32_t>();
    a.core_rsvable = s->has_cores ? s->d_core_rsvable.as<uint64_t>() : nullptr;
    a.core_avail = s->has_cores ? s->d_core_avail.as<uint64_t>() : nullptr;
    a.core_used = s->has_cores ? s->d_core_used.as<uint64_t>() : nullptr;
    a.core_spc = s->has_cores ? s->d_core_spc.as<int64_t>() : nullptr;
    return a;
}

// Reserved cores the next placement of the group takes on `row` (the lowest
// free ones, rank.go:437-466), from the host mirror of the plan's used sets;
// with `take` they become used (Plan.AppendAlloc).
void core_record(pe_stack* s, const TgPlan& g, int32_t row, bool take, uint64_t out[4]) {
    for (int w = 0; w < 4; w++) out[w] = 0;
    if (g.ask.cores <= 0 || !s->has_cores || row < 0 || (size_t)row >= s->nodes.size()) return;
    uint32_t need = (uint32_t)g.ask.cores;
    for (int w = 0; w < 4 && need; w++) {
        uint64_t f = s->h_core_rsvable[4 * (size_t)row + w] & ~s->h_core_used[4 * (size_t)row + w];
        for (; f && need; need--) { out[w] |= f & (~f + 1); f &= f - 1; }
        if (take) s->h_core_used[4 * (size_t)row + w] |= out[w];
    }
}

// A snapshot alloc's reserved cores leave (hold = false: plan stop or
// preemption) or rejoin (PopUpdate) its node's used set in the host mirror.
void core_hold(pe_stack* s, uint32_t alloc, bool hold) {
    if (!s->has_cores || alloc >= s->allocs.size()) return;
    const HostAlloc& a = s->allocs[alloc];
    for (int w = 0; w < 4; w++) {
        uint64_t& u = s->h_core_used[4 * (size_t)a.row + w];
        u = hold ? (u | a.cores[w]) : (u & ~a.cores[w]);
    }
}

// Job-dependent per-node collision counts from the snapshot + the plan, and
// with `own` the job's own proposed state allocs per node (ProposedAllocs
// minus plan placements and plan stops). The counts are mostly zero (a new
// job, a short plan): the nonzero ones go up as a sorted sparse list and one
// launch rewrites every array, instead of one dense upload per array.
static pe::ResetArgs reset_args(pe_stack* s) {
    pe::ResetArgs R;
    R.rec = s->d_rec.as<pe::NodeRec>();
    R.base_rec = s->d_base_rec.as<pe::NodeRec>();
    R.dev_free = s->d_dev_free.as<uint32_t>();
    R.dev_free_base = s->d_dev_free_base.as<uint32_t>();
    R.n = (uint32_t)s->nodes.size();
    R.preempted = s->d_preempted.as<uint8_t>();
    R.m = (uint32_t)s->h_preempted.size();
    R.pcount = s->d_pcount.as<uint32_t>();
    R.keys = std::max<uint32_t>(s->n_jtg_keys, 1);
    return R;
}

// A pending fold (pe_stack::fold_pending) as its own launch.
static int flush_counts(pe_stack* s) {
    if (!s->counts_pending) return PE_OK;
    const pe::CountArgs C = s->pending_counts;
    HIP_TRY(s, pe_launch_counts(&C.D, C.nd, C.n, C.ents, C.m, C.R.rec ? &C.R : nullptr, s->stream));
    s->counts_pending = false;
    return PE_OK;
}

static int flush_fold(pe_stack* s) {
    if (!s->fold_pending) return PE_OK;
    const pe::FoldArgs F = s->pending_fold;
    const pe::NodeSoA soa = soa_of(s);
    HIP_TRY(s, pe_launch_fold_feas_staged(&soa, F.class_src, F.class_dst, F.ncls, F.node_ok, F.feas, s->stream));
    s->fold_pending = false;   // only a launched fold clears the flag (as flush_reset)
    return PE_OK;
}

// The deferred ResetPlan launch, before any other device work of the handle.
static int flush_reset(pe_stack* s) {
    if (s->fold_pending) {
        const int rc = flush_fold(s);
        if (rc) return rc;
    }
    if (!s->reset_pending) return PE_OK;
    HIP_TRY(s, hipSetDevice(s->device));
    const pe::ResetArgs R = reset_args(s);
    HIP_TRY(s, pe_launch_reset_plan(R.rec, R.base_rec, R.dev_free, R.dev_free_base, R.n, R.preempted, R.m, R.pcount,
                                    R.keys, s->stream));
    // only a launched copy clears the flag: a failed launch is retried by the
    // next entry point instead of leaving the previous evaluation's state
    s->reset_pending = false;
    return PE_OK;
}


void invalidate_job_distinct(pe_stack* s, uint32_t tgi);

// ---- the served-Select view (pe_spec_view) ----------------------------------
// The records of the active run, published for the caller; its counters mirror
// sp.served / sp.confirmed. What the caller served or confirmed from the view
// is taken over exactly as spec_serve / commit_one would have done it.
static const pe::EmitRec& spec_rec(const pe_stack::Spec& sp, uint32_t k) {
    return sp.compact ? sp.crecs[k] : sp.vrecs[k];
}

static void sys_view_take(pe_stack* s);

// Record k's row, and its PreemptedAllocs (evicting runs; none otherwise).
static inline int32_t spec_rec_row(const pe_stack::Spec& sp, uint32_t k) {
    return sp.compact ? sp.crecs[k].row : sp.recs[k].row;
}
static inline uint32_t spec_rec_npre(const pe_stack::Spec& sp, uint32_t k) {
    return sp.evict ? sp.pre_off[k + 1] - sp.pre_off[k] : 0u;
}
static inline const uint32_t* spec_rec_pre(const pe_stack::Spec& sp, uint32_t k) {
    return sp.evict ? sp.pre_list.data() + sp.pre_off[k] : nullptr;
}

// A served nil needs no Commit: it is settled as soon as it is served.
static void spec_settle(pe_stack::Spec& sp) {
    if (sp.served == sp.confirmed + 1 && spec_rec_row(sp, sp.served - 1) < 0) sp.confirmed = sp.served;
    sp.pending = sp.served > sp.confirmed;
}

// Record k's Commit named its row: Plan.AppendAlloc (+ AppendPreemptedAlloc)
// in the host mirror, as commit_one's predicted branch; `kids` logs it for the
// replicas as pe_commit / pe_commit_preempt would.
static void spec_confirm_rec(pe_stack* s, uint32_t k, bool kids) {
    pe_stack::Spec& sp = s->spec;
    const int32_t row = spec_rec_row(sp, k);
    if (row < 0) return;
    s->gen++;
    plan_of(s).emplace_back(s->tgs[sp.tgi]->name, (uint32_t)row);
    invalidate_job_distinct(s, sp.tgi);
    if (kids && !s->kids.empty()) {
        const uint32_t np = spec_rec_npre(sp, k);
        kid_log(s, np ? 1 : 0, sp.tgi, row, np ? spec_rec_pre(sp, k) : nullptr, np);
    }
}

// pe_last_metrics after record k was served.
static void spec_metrics_served(pe_stack* s, uint32_t k) {
    const pe_stack::Spec& sp = s->spec;
    if (!sp.metrics || k + 1 >= sp.mcounts_off.size()) return;
    s->m_counts.assign(sp.mcounts.begin() + sp.mcounts_off[k], sp.mcounts.begin() + sp.mcounts_off[k + 1]);
    s->m_scores.assign(sp.mscores.begin() + sp.mscores_off[k], sp.mscores.begin() + sp.mscores_off[k + 1]);
    s->metrics_text_ok = false;
    s->metrics_valid = true;
}

static void view_take(pe_stack* s) {
    sys_view_take(s);
    pe_spec_view& v = s->sview;
    pe_stack::Spec& sp = s->spec;
    if (!v.n_rec || !sp.active) return;
    if (v.served == sp.served && v.confirmed == sp.confirmed) return;
    const uint32_t served = std::min(std::max(v.served, sp.served), sp.n_rec);
    const uint32_t confirmed = std::min(std::max(v.confirmed, sp.confirmed), served);
    // a record pe_select served (spec_start / spec_serve) whose Commit the
    // caller confirmed through the view
    if (sp.pending && confirmed >= sp.served) spec_confirm_rec(s, sp.served - 1, true);
    for (uint32_t k = sp.served; k < served; k++) {   // spec_serve of record k, then its commit
        const pe::EmitRec& r = spec_rec(sp, k);
        s->gen++;
        elig_log_span(s, sp.tgi, s->offset, r.nodes_evaluated);
        s->offset = r.new_offset;
        s->metrics_valid = false;
        s->spec_stats[1]++;
        if (k < confirmed) spec_confirm_rec(s, k, true);
    }
    if (served > sp.served) spec_metrics_served(s, served - 1);
    sp.served = served;
    sp.confirmed = confirmed;
    spec_settle(sp);
    s->offer_row = -1;
    v.served = sp.served;
    v.confirmed = sp.confirmed;
}

static void view_publish(pe_stack* s) {
    pe_stack::Spec& sp = s->spec;
    pe_spec_view& v = s->sview;
    if (!sp.compact) {   // served Selects carry no reserved cores: the leading fields
        sp.vrecs.resize(sp.n_rec);
        for (uint32_t k = 0; k < sp.n_rec; k++) {
            const pe_ranked_node& r = sp.recs[k];
            pe::EmitRec& e = sp.vrecs[k];
            std::memset(&e, 0, sizeof(e));
            std::memcpy(&e, &r, offsetof(pe::EmitRec, n_device_offers));
            e.n_device_offers = r.n_device_offers;
            for (int q = 0; q < PE_MAX_DEVICE_REQ; q++) e.device_offer_group[q] = (uint16_t)r.device_offer_group[q];
            e.flags = sp.evict ? sp.rflags[k] : 0u;
        }
    }
    v.epoch++;
    v.tg_index = sp.tgi;
    v.recs = sp.compact ? sp.crecs.data() : sp.vrecs.data();
    v.pre_off = sp.evict ? sp.pre_off.data() : nullptr;
    v.pre_allocs = sp.evict ? sp.pre_list.data() : nullptr;
    v.mcounts = sp.metrics ? sp.mcounts.data() : nullptr;
    v.mcounts_off = sp.metrics ? sp.mcounts_off.data() : nullptr;
    v.mscores = sp.metrics ? sp.mscores.data() : nullptr;
    v.mscores_off = sp.metrics ? sp.mscores_off.data() : nullptr;
    v.served = sp.served;
    v.confirmed = sp.confirmed;
    v.n_rec = (s->metrics_on && !sp.metrics) ? 0u : sp.n_rec;
}

static void view_withdraw(pe_stack* s) {
    pe_spec_view& v = s->sview;
    if (!v.n_rec && !v.recs) return;
    v.epoch++;
    v.n_rec = 0;
    v.recs = nullptr;
    v.pre_off = v.pre_allocs = nullptr;
    v.mcounts = nullptr;
    v.mcounts_off = nullptr;
    v.mscores = nullptr;
    v.mscores_off = nullptr;
    v.served = v.confirmed = 0;
}

// ---- the served system-Select view (pe_system_view) --------------------------
// The per-row cache of the active k_system pass and a log the caller writes
// for every SetNodes([row]) + Select (+ Commit) it answered from it; taken over
// exactly as pe_set_nodes' per-node path, sys_serve and commit_one would have
// done it.
constexpr uint64_t kSysNaNBits = 0x7FF8000000000000ull;
constexpr uint64_t kSysStale = kSysNaNBits | 3u;
static_assert(kSysStale == PE_SYS_STALE, "the view's stale marker is the cache's");

// The caller's log entries [k0, upto) with AllocMetric on: the memo of failing
// classes as the sequential Selects left it (the engine's copy, then the
// caller's array and the reference memo), and the last Select's maps.
static void sys_view_take_metrics(pe_stack* s, uint32_t k0, uint32_t upto) {
    pe_system_view& v = s->sysview;
    pe_stack::SysSpec& y = s->sys;
    const uint64_t* cache = s->h_sys_cache.as<uint64_t>();
    const uint32_t nn = (uint32_t)s->nodes.size(), ncls = s->ncls;
    for (uint32_t k = k0; k < upto; k++) {
        const uint32_t e = v.log[k];
        const uint32_t row = e & PE_SYS_ROW_MASK;
        if (row >= nn) continue;
        uint32_t code = 0;
        bool before = false;
        if (e & PE_SYS_NIL) {
            code = (uint32_t)(cache[row] & 3u);
            const uint32_t mc = y.mclass[row];
            if (code == 1 && mc != PE_NONE) {
                before = y.mfailed_eng[mc] != 0;
                y.mfailed_eng[mc] = 1;
            }
        }
        if (k + 1 == upto) metrics_set_last_sys(s, row, code, before);
    }
    std::memcpy(y.mfailed.data(), y.mfailed_eng.data(), y.mfailed.size());
    auto& rt = s->ref_tg_memo[s->tgs[y.tgi]->name];
    if (s->ref_job_memo.size() != ncls) s->ref_job_memo.assign(ncls, -1);
    if (rt.size() != ncls) rt.assign(ncls, -1);
    for (uint32_t c = 0; c < ncls; c++) {
        if (y.mfailed_eng[c]) s->ref_job_memo[c] = 0;
        if (y.mfailed_eng[ncls + c]) rt[c] = 0;
    }
}

static void sys_view_take(pe_stack* s) {
    pe_system_view& v = s->sysview;
    if (!v.n_rows || v.n_log == s->sys_taken) return;
    plan_settle(s);   // the take-over moves the list
    ApiScope prof_(s, "sys_view_take");
    pe_stack::SysSpec& y = s->sys;
    const uint32_t upto = std::min(v.n_log, v.log_cap);
    if (!y.active || y.tgi >= s->tgs.size() || s->visit.size() != 1) { s->sys_taken = upto; return; }
    const auto name = s->tgs[y.tgi]->name;
    uint64_t* cache = s->h_sys_cache.as<uint64_t>();
    auto take_fast = [&](uint32_t k0) {
        // nothing for EvalEligibility to log: the per-node SetNodes / Select
        // bookkeeping leaves the last entry's state, and only the commits
        // need one step each
        uint32_t last = PE_NONE;
        bool last_nil = true;
        uint32_t cnt = 0;
        // one branch-light pass: the committed rows compacted into the queue
        // (the caller marked their outcome stale, nomad_pe.h), then the plan
        // entries from them
        const size_t p0 = y.pending.size();
        y.pending.resize(p0 + (upto - k0));
        uint32_t* q = y.pending.data() + p0;
        size_t c = 0;
        const uint32_t nn = (uint32_t)s->nodes.size();
        for (uint32_t k = k0; k < upto; k++) {
            const uint32_t e = v.log[k];
            const uint32_t row = e & PE_SYS_ROW_MASK;
            if (row >= nn) continue;
            cnt++;
            last = row;
            last_nil = (e & PE_SYS_NIL) != 0;
            q[c] = row;
            c += (!last_nil && (e & PE_SYS_COMMITTED)) ? 1u : 0u;
        }
        y.pending.resize(p0 + c);
        const size_t l0 = plan_of(s).size();
        plan_of(s).resize(l0 + c);
        for (size_t i = 0; i < c; i++) plan_of(s)[l0 + i] = std::make_pair(name, q[i]);
        if (cnt) {
            const uint32_t le = v.log[upto - 1];
            const bool committed = !last_nil && (le & PE_SYS_COMMITTED) && (le & PE_SYS_ROW_MASK) == last;
            s->gen += cnt;   // one per SetNodes, as the per-node path counts
            s->visit[0] = last;
            s->d_visit_is_visit = false;
            s->rank_of_valid = false;
            s->visit_unique = true;
            s->offset = 0;
            s->limit = 2;
            y.served += cnt;
            y.served_row = (last_nil || committed) ? -1 : (int32_t)last;
            s->offer_row = y.served_row;
            s->offers = 0xFFFFFFFFu;
            s->metrics_valid = false;
        }
    };
    // entry by entry while EvalEligibility still learns classes, then the
    // rest at once
    uint32_t k = s->sys_taken;
    for (; k < upto; k++) {
        if (s->elig_log.empty() && (s->elig_mute || s->tgs[y.tgi]->elig_complete)) break;
        const uint32_t e = v.log[k];
        const uint32_t row = e & PE_SYS_ROW_MASK;
        if (row >= s->nodes.size()) continue;
        // SetNodes([row]): the per-node path of pe_set_nodes
        if (!s->elig_log.empty()) elig_resolve(s);
        s->gen++;
        s->visit[0] = row;
        s->d_visit_is_visit = false;
        s->rank_of_valid = false;
        s->visit_unique = true;
        s->offset = 0;
        s->limit = 2;
        // Select: sys_serve
        const bool nil = (e & PE_SYS_NIL) != 0;
        y.served_row = nil ? -1 : (int32_t)row;
        y.served++;
        s->offer_row = y.served_row;
        s->offers = 0xFFFFFFFFu;
        s->metrics_valid = false;
        elig_log_span(s, y.tgi, 0, 1);
        // Commit: commit_one's served branch
        if (!nil && (e & PE_SYS_COMMITTED)) {
            y.served_row = -1;
            y.pending.push_back(row);
            cache[row] = kSysStale;
            plan_of(s).emplace_back(name, row);
            s->offer_row = -1;
        }
    }
    if (k < upto) take_fast(k);
    if (s->metrics_on && y.mready && v.mfailed) sys_view_take_metrics(s, s->sys_taken, upto);
    s->sys_taken = upto;
}

static void sys_view_publish(pe_stack* s) {
    pe_system_view& v = s->sysview;
    const uint32_t n = (uint32_t)s->nodes.size();
    v.epoch++;
    v.tg_index = s->sys.tgi;
    s->sys_log.resize(std::max<uint32_t>(n, 1));
    v.log = s->sys_log.data();
    v.log_cap = n;
    v.n_log = 0;
    s->sys_taken = 0;
    v.outcome = s->h_sys_cache.as<uint64_t>();
    v.preempt = s->cfg.preempt ? 1u : 0u;
    const bool m = s->metrics_on && s->sys.mready;
    v.mkey = m ? s->sys.mkey.data() : nullptr;
    v.mclass = m ? s->sys.mclass.data() : nullptr;
    v.mfailed = m ? s->sys.mfailed.data() : nullptr;
    v.mscore = m ? s->sys.mscore.data() : nullptr;
    v.mnode_class = m ? s->sys.mnode_class.data() : nullptr;
    v.mkey_ineligible = s->mkey_p("computed class ineligible");
    v.n_rows = ((s->metrics_on && !m) || !s->kids.empty()) ? 0u : n;
}

static void sys_view_withdraw(pe_stack* s) {
    pe_system_view& v = s->sysview;
    if (!v.n_rows && !v.outcome) return;
    v.epoch++;
    v.n_rows = 0;
    v.outcome = nullptr;
    v.n_log = 0;
    s->sys_taken = 0;
}

static void sys_deactivate(pe_stack* s) {
    s->sys.active = false;
    sys_view_withdraw(s);
}

// Every entry point first takes over the Selects / Commits the caller served
// from the views, then launches a deferred ResetPlan copy.
#define PE_FLUSH_RESET(s)                             \
    do {                                              \
        if (s) plan_settle(s);                        \
        if (s) view_take(s);                          \
        if ((s) && ((s)->reset_pending || (s)->fold_pending)) { \
            const int frc_ = flush_reset(s);          \
            if (frc_) return frc_;                    \
        }                                             \
    } while (0)

// `defer` (SetJob): the counts may wait for the next launch (counts_pending).
int build_collisions(pe_stack* s, bool own = false, bool defer = false) {
    if (s->counts_pending) {   // an earlier SetJob's counts first: launches keep their order
        const int frc = flush_counts(s);
        if (frc) return frc;
    }
    const size_t n = s->nodes.size();
    const uint32_t ntg = (uint32_t)s->tgs.size();
    const uint32_t nd = ntg + 2;   // dst 0: own, 1: job, 2 + g: task group g
    if (nd > (uint32_t)pe::kMaxCountDst || n >= (size_t(1) << 27)) {
        PE_FLUSH_RESET(s);
        std::vector<uint32_t> job(n, 0), mine(own ? n : 0, 0);
        std::vector<std::vector<uint32_t>> tg(ntg, std::vector<uint32_t>(n, 0));
        auto add = [&](uint32_t row, uint32_t tgname) {
            job[row]++;
            for (uint32_t g = 0; g < ntg; g++) if (s->tgs[g]->name == tgname) tg[g][row]++;
        };
        for (uint32_t i : s->own_allocs())
            if (!s->stopped(i)) { add(s->allocs[i].row, s->allocs[i].tg); if (own) mine[s->allocs[i].row]++; }
        for (auto& p : plan_of(s)) add(p.second, p.first);
        if (own) HIP_TRY(s, upload_s(s, s->d_own_existing, mine));
        HIP_TRY(s, upload_s(s, s->d_coll_job, job));
        for (uint32_t g = 0; g < ntg; g++) HIP_TRY(s, upload_s(s, s->tgs[g]->coll_tg, tg[g]));
        return PE_OK;
    }
    std::vector<uint32_t> keys;
    auto add = [&](uint32_t row, uint32_t tgname, bool is_own) {
        const uint32_t base = row << 5;
        if (is_own) keys.push_back(base);
        keys.push_back(base | 1u);
        for (uint32_t g = 0; g < ntg; g++) if (s->tgs[g]->name == tgname) keys.push_back(base | (2u + g));
    };
    for (uint32_t i : s->own_allocs())
        if (!s->stopped(i)) add(s->allocs[i].row, s->allocs[i].tg, own);   // ProposedAllocs drops plan stops
    for (auto& p : plan_of(s)) add(p.second, p.first, false);
    std::sort(keys.begin(), keys.end());
    std::vector<uint2> ents;
    for (size_t i = 0; i < keys.size();) {
        size_t j = i;
        while (j < keys.size() && keys[j] == keys[i]) j++;
        ents.push_back(make_uint2(keys[i], (uint32_t)(j - i)));
        i = j;
    }
    pe::CountDsts D;
    std::memset(&D, 0, sizeof(D));
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(uint32_t);
    if (own) {
        HIP_TRY(s, s->d_own_existing.ensure(bytes));
        D.d[0] = s->d_own_existing.as<uint32_t>();
    }
    HIP_TRY(s, s->d_coll_job.ensure(bytes));
    D.d[1] = s->d_coll_job.as<uint32_t>();
    for (uint32_t g = 0; g < ntg; g++) {
        HIP_TRY(s, s->tgs[g]->coll_tg.ensure(bytes));
        D.d[2 + g] = s->tgs[g]->coll_tg.as<uint32_t>();
    }
    const pe::ResetArgs R = s->reset_pending ? reset_args(s) : pe::ResetArgs{};
    // only where the next launch can be a fused k_chain (a short list): else
    // the counts launch now and run while the host prepares the first Select
    if (defer && s->counts_defer_ok && n <= pe_chain_fused_max_n()) {
        // the entries stay in the mapped staging ring: the launch that carries
        // them reads them from there
        const uint2* staged = ents.empty() ? nullptr : reinterpret_cast<const uint2*>(stage_only(s, ents));
        if (ents.empty() || staged) {
            pe::CountArgs& C = s->pending_counts;
            C.D = D;
            C.nd = nd;
            C.n = (uint32_t)n;
            C.ents = staged;
            C.m = (uint32_t)ents.size();
            C.R = R;
            s->counts_pending = true;
            s->reset_pending = false;   // the copy rides with the counts
            return PE_OK;
        }
    }
    if (!ents.empty()) HIP_TRY(s, upload_s(s, s->d_count_ents, ents));
    HIP_TRY(s, pe_launch_counts(&D, nd, (uint32_t)n, ents.empty() ? nullptr : s->d_count_ents.as<uint2>(),
                                (uint32_t)ents.size(), R.rec ? &R : nullptr, s->stream));
    s->reset_pending = false;   // the copy rode in this launch (cleared only once it launched)
    return PE_OK;
}

int build_job_counts(pe_stack* s, bool defer = false) { return build_collisions(s, true, defer); }

// propertySet cleared values (propertyset.go:159-209): the plan's stopped allocs
// of the job (terminal ones included, filterAllocs(stopping, false)), less one
// for every value the proposed allocs also use when more than one is cleared.
// `node_val` maps a row to the set's value index; `tg_filter` limits to a group.
template <class F>
std::vector<uint32_t> cleared_counts(pe_stack* s, size_t nvals, F node_val, bool job_level, uint32_t tg_name) {
    std::vector<uint32_t> cleared(nvals, 0);
    bool any = false;
    for (auto& kv : s->node_update)
        for (uint32_t ai : kv.second) {
            const HostAlloc& a = s->allocs[ai];
            if (a.job != s->job_id || a.ns != s->job_ns || (!job_level && a.tg != tg_name)) continue;
            const uint32_t v = node_val(a.row);
            if (v != pe::kMissing) { cleared[v]++; any = true; }
        }
    if (!any) return {};
    std::vector<uint8_t> prop(nvals, 0);
    for (auto& p : plan_of(s))
        if (job_level || p.first == tg_name) {
            const uint32_t v = node_val(p.second);
            if (v != pe::kMissing) prop[v] = 1;
        }
    for (size_t v = 0; v < nvals; v++)
        if (prop[v] && cleared[v] > 1) cleared[v]--;
    return cleared;
}

// Spread property sets for a task group (spread.go:76-104, propertyset.go).
static void cls_cache_sync(pe_stack* s);

int build_psets(pe_stack* s, TgPlan& g) {
    g.psets.clear();
    g.psets_dynamic = false;
    std::vector<const SpreadSpec*> specs;
    for (auto& sp : s->job_spreads) specs.push_back(&sp);
    for (auto& sp : g.spreads) specs.push_back(&sp);
    if (specs.size() > (size_t)pe::kMaxPsets) { g.unsupported = "more than 16 spread stanzas"; return PE_OK; }
    // computeSpreadInfo once per task group name; weights accumulate (spread.go:254)
    if (!s->spread_info_done.count(g.name)) {
        s->spread_info_done.insert(g.name);
        const int32_t before = s->sum_spread_weights;
        for (auto& sp : g.spreads) s->sum_spread_weights += (int32_t)(int8_t)sp.weight;
        for (auto& sp : s->job_spreads) s->sum_spread_weights += (int32_t)(int8_t)sp.weight;
        // SpreadIterator.Next divides by the running sum (spread.go:157): the
        // other groups' spread weights change with it
        if (s->sum_spread_weights != before)
            for (auto& o : s->tgs)
                if (o.get() != &g) o->psets_built = false;
    }
    // combined list for desired counts: tg spreads then job spreads, keyed by attribute
    std::map<uint32_t, const SpreadSpec*> info;
    for (auto& sp : g.spreads) info[sp.attribute] = &sp;
    for (auto& sp : s->job_spreads) info[sp.attribute] = &sp;
    const size_t n = s->nodes.size();
    for (const SpreadSpec* sp : specs) {
        auto ps = std::make_unique<PsetDev>();
        ps->target = parse_target(s, s->S(sp->attribute));
        ps->per_node = ps->target.escapes || ps->target.kind == T_ID || ps->target.kind == T_NAME;
        auto value_of = [&](const NodeView& nd) -> uint32_t {
            uint32_t vid;
            Target t = resolve(s, ps->target, nd, &vid);
            if (!t.found || t.nil) return pe::kMissing;
            if (vid == PE_NONE) vid = s->lookup(t.value);   // literal attribute target
            auto it = ps->value_index.find(vid);
            if (it == ps->value_index.end()) {
                it = ps->value_index.emplace(vid, (uint32_t)ps->value_str.size()).first;
                ps->value_str.push_back(vid);
            }
            return it->second;
        };
        std::vector<uint32_t> by_class(s->ncls, pe::kMissing), by_node;
        if (ps->per_node) {
            by_node.resize(n);
            for (size_t i = 0; i < n; i++) by_node[i] = value_of(s->view((uint32_t)i));
        } else {
            // the values per class, from the cache when the target was spread on before
            const std::string vk = s->S(sp->attribute);
            cls_cache_sync(s);
            auto cv = s->cc_val.find(vk);
            if (cv != s->cc_val.end() && cv->second.second.size() == s->ncls) {
                ps->value_str = cv->second.first;
                for (uint32_t i = 0; i < (uint32_t)ps->value_str.size(); i++) ps->value_index.emplace(ps->value_str[i], i);
                by_class = cv->second.second;
            } else {
                for (uint32_t c = 0; c < s->ncls; c++) by_class[c] = value_of(s->view(s->class_rep[c]));
                s->cc_val[vk] = std::make_pair(ps->value_str, by_class);
            }
        }
        // existing allocs of this job and task group (populateExisting) + plan allocs
        auto node_val = [&](uint32_t row) {
            return ps->per_node ? by_node[row] : by_class[s->nodes[row].cls];
        };
        ps->h_counts.assign(ps->value_str.size(), 0);
        for (uint32_t ai : s->own_allocs())
            if (const HostAlloc& a = s->allocs[ai]; a.ns == s->job_ns && a.tg == g.name) {
                uint32_t v = node_val(a.row);
                if (v != pe::kMissing) ps->h_counts[v]++;
            }
        for (auto& p : plan_of(s))
            if (p.first == g.name) {
                uint32_t v = node_val(p.second);
                if (v != pe::kMissing) ps->h_counts[v]++;
            }
        {   // GetCombinedUseMap: existing + proposed - cleared, not below 0
            const auto cl = cleared_counts(s, ps->value_str.size(), node_val, false, g.name);
            for (size_t v = 0; v < cl.size(); v++) {
                ps->h_counts[v] = ps->h_counts[v] >= cl[v] ? ps->h_counts[v] - cl[v] : 0u;
                if (cl[v]) g.psets_dynamic = true;
            }
        }
        const SpreadSpec* si = info[sp->attribute];
        const double total = (double)g.count;
        std::map<uint32_t, double> desired;
        double sum = 0.0;
        for (auto& t : si->targets) {
            double d = ((double)t.second / (double)100) * total;
            desired[t.first] = d;
            sum += d;
        }
        bool has_star = false;
        double star = 0;
        const uint32_t star_id = s->lookup("*");
        if (star_id != PE_NONE && desired.count(star_id)) { has_star = true; star = desired[star_id]; }
        if (sum > 0 && sum < total) { has_star = true; star = total - sum; }   // implicitTarget
        ps->even = si->targets.empty();
        ps->h_desired.assign(ps->value_str.size(), std::nan(""));
        for (size_t v = 0; v < ps->value_str.size(); v++) {
            auto it = desired.find(ps->value_str[v]);
            if (it != desired.end()) ps->h_desired[v] = it->second;
            else if (has_star) ps->h_desired[v] = star;
        }
        ps->weight_frac = (double)(int8_t)si->weight / (double)s->sum_spread_weights;
        HIP_TRY(s, upload_s(s, ps->val_class, by_class));
        if (ps->per_node) HIP_TRY(s, upload_s(s, ps->val_node, by_node));
        ps->h_val_class = std::move(by_class);   // host copies (the batched metrics trace's counts)
        ps->h_val_node = std::move(by_node);
        std::vector<uint32_t> cnt = ps->h_counts;
        if (cnt.empty()) cnt.push_back(0);
        HIP_TRY(s, upload_s(s, ps->counts, cnt));
        std::vector<double> des = ps->h_desired;
        if (des.empty()) des.push_back(0);
        HIP_TRY(s, upload_s(s, ps->desired, des));
        g.psets.push_back(std::move(ps));
    }
    g.n_spread = (int)g.psets.size();
    // distinct_property sets (propertyset.go:14-355): job-level ones count every
    // alloc of the job, task-group ones only the group's (filterAllocs)
    std::vector<std::pair<const ParsedConstraint*, bool>> dps;
    for (auto& c : s->job_constraints) if (c.op == "distinct_property") dps.emplace_back(&c, true);
    for (auto& c : g.distinct_props) dps.emplace_back(&c, false);
    if (g.psets.size() + dps.size() > (size_t)pe::kMaxPsets) {
        g.unsupported = "more than 16 spread and distinct_property sets";
        return PE_OK;
    }
    for (auto& dp : dps) {
        const ParsedConstraint& c = *dp.first;
        const bool job_level = dp.second;
        auto ps = std::make_unique<PsetDev>();
        ps->distinct = true;
        ps->target = c.l;
        ps->target_text = c.ltext;
        ps->per_node = ps->target.escapes || ps->target.kind == T_ID || ps->target.kind == T_NAME;
        // RTarget: strconv.ParseUint, default 1; unparsable -> every node filtered
        ps->allowed = 1;
        if (c.r.kind == T_LITERAL && !c.r.literal.empty()) {
            unsigned long long v = 0;
            bool okp = true;
            for (char ch : c.r.literal) {
                if (ch < '0' || ch > '9' || v > (UINT64_MAX - 9) / 10) { okp = false; break; }
                v = v * 10 + (unsigned)(ch - '0');
            }
            ps->allowed = okp ? (uint32_t)std::min<unsigned long long>(v, 0xFFFFFFFFull) : 0u;
        } else if (c.r.kind != T_LITERAL) {
            ps->allowed = 0;   // an interpolated RTarget does not parse as a count
        }
        auto value_of = [&](const NodeView& nd) -> uint32_t {
            uint32_t vid;
            Target t = resolve(s, ps->target, nd, &vid);
            if (!t.found || t.nil) return pe::kMissing;
            if (vid == PE_NONE) vid = s->lookup(t.value);
            auto it = ps->value_index.find(vid);
            if (it == ps->value_index.end()) {
                it = ps->value_index.emplace(vid, (uint32_t)ps->value_str.size()).first;
                ps->value_str.push_back(vid);
            }
            return it->second;
        };
        std::vector<uint32_t> by_class(s->ncls, pe::kMissing), by_node;
        if (ps->per_node) {
            by_node.resize(n);
            for (size_t i = 0; i < n; i++) by_node[i] = value_of(s->view((uint32_t)i));
        } else {
            for (uint32_t c2 = 0; c2 < s->ncls; c2++) by_class[c2] = value_of(s->view(s->class_rep[c2]));
        }
        auto node_val = [&](uint32_t row) { return ps->per_node ? by_node[row] : by_class[s->nodes[row].cls]; };
        ps->h_val_class = by_class;
        ps->h_val_node = by_node;
        ps->h_counts.assign(ps->value_str.size(), 0);
        for (uint32_t ai : s->own_allocs())
            if (const HostAlloc& a = s->allocs[ai]; a.ns == s->job_ns && (job_level || a.tg == g.name)) {
                const uint32_t v = node_val(a.row);
                if (v != pe::kMissing) ps->h_counts[v]++;
            }
        for (auto& p : plan_of(s))
            if (job_level || p.first == g.name) {
                const uint32_t v = node_val(p.second);
                if (v != pe::kMissing) ps->h_counts[v]++;
            }
        {
            const auto cl = cleared_counts(s, ps->value_str.size(), node_val, job_level, g.name);
            for (size_t v = 0; v < cl.size(); v++) {
                ps->h_counts[v] = ps->h_counts[v] >= cl[v] ? ps->h_counts[v] - cl[v] : 0u;
                if (cl[v]) g.psets_dynamic = true;
            }
        }
        HIP_TRY(s, upload_s(s, ps->val_class, by_class));
        if (ps->per_node) HIP_TRY(s, upload_s(s, ps->val_node, by_node));
        std::vector<uint32_t> cnt = ps->h_counts;
        if (cnt.empty()) cnt.push_back(0);
        HIP_TRY(s, upload_s(s, ps->counts, cnt));
        HIP_TRY(s, upload_s(s, ps->desired, std::vector<double>(1, 0.0)));
        g.psets.push_back(std::move(ps));
    }
    g.psets_built = true;
    return PE_OK;
}

// The checker caches hold for one node table (nodes_gen); a handful of
// distinct jobs at most.
static void cls_cache_sync(pe_stack* s) {
    if (s->cc_gen == s->nodes_gen && s->cc_job.size() + s->cc_sig.size() + s->cc_aff.size() + s->cc_val.size() < 96)
        return;
    s->cc_gen = s->nodes_gen;
    s->cc_job.clear();
    s->cc_sig.clear();
    s->cc_aff.clear();
    s->cc_val.clear();
}

// The inputs of job_fail: the job constraints (Constraint.String() holds all
// three fields).
static std::string job_checker_key(const pe_stack* s) {
    std::string k;
    for (auto& c : s->job_constraints) { k += c.text; k += '\x1f'; }
    return k;
}

// The inputs of tg_fail (drivers, constraints, host volumes, network mode,
// port host network), or "" when not cached (device requests).
static std::string tg_checker_key(const pe_stack* s, const TgPlan& g) {
    if (!g.dev_reqs.empty()) return std::string();
    std::string k = "D";
    for (uint32_t d : g.drivers) { k += s->S(d); k += '\x1f'; }
    k += "C";
    for (auto& c : g.constraints) { k += c.text; k += '\x1f'; }
    k += "V";
    for (auto& v : g.volumes) { k += s->S(v.first); k += v.second ? "+ro\x1f" : "+rw\x1f"; }
    k += "N";
    k += s->S(g.net_mode);
    k += '\x1f';
    k += g.net_ports > 0 ? "P" + s->S(g.net_host) : std::string("-");
    return k;
}

// Task-group checker verdict per signature and, per class, whether every
// signature of the class agrees ("uniform": the memo outcome does not depend
// on which member is visited first).
void classify_classes(pe_stack* s, TgPlan& g, pe::ConstraintEvaluator& ev) {
    if (!g.sig_tg.empty()) return;
    cls_cache_sync(s);
    const std::string tk = tg_checker_key(s, g);
    auto ct = tk.empty() ? s->cc_sig.end() : s->cc_sig.find(tk);
    if (ct != s->cc_sig.end() && ct->second.size() == s->sig_rep.size()) {
        g.sig_tg = ct->second;
    } else {
        g.sig_tg.assign(s->sig_rep.size(), 0);
        for (size_t sg = 0; sg < s->sig_rep.size(); sg++)
            g.sig_tg[sg] = tg_feasible(s, ev, g, s->view(s->sig_rep[sg])) ? 1 : 0;
        if (!tk.empty()) s->cc_sig[tk] = g.sig_tg;
    }
    g.class_uniform.assign(s->ncls, 1);
    g.class_verdict.assign(s->ncls, 0);
    if (s->job_memo.size() != s->ncls) s->job_memo.assign(s->ncls, -1);
    if (!s->job_escaped) {   // job_feasible per class, from the cache when the job was set before
        const std::string jk = job_checker_key(s);
        auto cj = s->cc_job.find(jk);
        if (cj == s->cc_job.end() || cj->second.size() != s->ncls) {
            std::vector<int8_t> v(s->ncls);
            for (uint32_t c = 0; c < s->ncls; c++) v[c] = job_feasible(s, ev, s->view(s->class_rep[c])) ? 1 : 0;
            cj = s->cc_job.insert_or_assign(jk, std::move(v)).first;
        }
        for (uint32_t c = 0; c < s->ncls; c++)
            if (s->job_memo[c] == -1) s->job_memo[c] = cj->second[c];
    }
    for (uint32_t c = 0; c < s->ncls; c++) {
        const auto& sigs = s->class_sigs[c];
        g.class_verdict[c] = sigs.empty() ? 0 : g.sig_tg[sigs[0]];   // a class left without members: no node reads it
        for (uint32_t sg : sigs) if (g.sig_tg[sg] != g.class_verdict[c]) g.class_uniform[c] = 0;
    }
    g.nonuniform.clear();
    for (uint32_t c = 0; c < s->ncls; c++) if (!g.class_uniform[c]) g.nonuniform.push_back(c);
}

// EvalEligibility memo emulation: the first node of a
// class that passes the job checks, in visit order from the cursor, decides
// the task group's verdict for the class. Uniform classes are decided by any
// member; only non-uniform ones need the scan.
void decide_classes(pe_stack* s, TgPlan& g, pe::ConstraintEvaluator& ev, std::vector<int8_t>& memo,
                    const uint32_t* order, size_t m, uint32_t start) {
    (void)ev;
    size_t pending = 0;
    for (uint32_t c = 0; c < s->ncls; c++) {
        if (memo[c] != -1) continue;
        if (g.class_uniform[c]) memo[c] = g.class_verdict[c];
        else pending++;
    }
    for (size_t k = 0; k < m && pending; k++) {
        const uint32_t row = order[(start + k) % m];
        const HostNode& nd = s->nodes[row];
        const uint32_t c = nd.cls;
        if (memo[c] != -1) continue;
        const bool jr = s->job_escaped ? g.job_ok_node[row] != 0 : s->job_memo[c] == 1;
        if (!jr) continue;
        memo[c] = g.sig_tg[nd.sig];
        pending--;
    }
}

std::vector<uint8_t> class_verdicts(pe_stack* s, TgPlan& g, const std::vector<int8_t>& memo) {
    std::vector<uint8_t> ok(s->ncls, 0);
    for (uint32_t c = 0; c < s->ncls; c++) ok[c] = memo[c] == 1 && (s->job_escaped || s->job_memo[c] == 1);
    return ok;
}

// FeasibilityWrapper + EvalEligibility memo emulation for one task group over a
// scan order (the visit order from the cursor). See SURVEY.md Appendix A3.
int build_tables(pe_stack* s, TgPlan& g, const std::vector<uint32_t>& order, uint32_t start) {
    pe::ConstraintEvaluator ev;
    const size_t n = s->nodes.size();
    auto& memo = s->tg_memo[g.name];
    if (memo.size() != s->ncls) memo.assign(s->ncls, -1);
    if (s->job_memo.size() != s->ncls) s->job_memo.assign(s->ncls, -1);
    std::vector<uint8_t> class_ok(s->ncls, 0), node_ok;
    const bool tg_escaped = g.escaped;
    if (tg_escaped) {
        // no memo for the task group: every node runs every check
        node_ok.assign(n, 0);
        for (uint32_t row = 0; row < n; row++)
            node_ok[row] = job_feasible(s, ev, s->view(row)) && tg_feasible(s, ev, g, s->view(row));
        std::fill(class_ok.begin(), class_ok.end(), 1);
    } else {
        if (s->job_escaped) {
            g.job_ok_node.assign(n, 0);
            for (uint32_t row = 0; row < n; row++) g.job_ok_node[row] = job_feasible(s, ev, s->view(row));
        } else {
            g.job_ok_node.clear();
        }
        {
            ApiScope prof_c_(s, "tables.classify");
            classify_classes(s, g, ev);
        }
        {
            ApiScope prof_d_(s, "tables.decide");
            decide_classes(s, g, ev, memo, order.data(), order.size(), start);
        }
        {
            ApiScope prof_v_(s, "tables.verdicts");
            class_ok = class_verdicts(s, g, memo);
        }
        if (s->job_escaped) node_ok = g.job_ok_node;
    }
    g.node_ok_used = !node_ok.empty();
    if (g.node_ok_used) HIP_TRY(s, upload_s(s, g.node_ok, node_ok));
    {
        // fold the class verdict into one byte per node (single round trip per
        // node); the class table goes up with the same launch when every
        // workgroup's pull of it over the bus stays small (blocks x classes
        // bytes, at most kStagedFoldBusBytes), else one upload + k_fold_feas
        pe::NodeSoA soa = soa_of(s);
        HIP_TRY(s, g.node_feas.ensure(std::max<size_t>(n, 1)));
        HIP_TRY(s, g.class_ok.ensure(std::max<size_t>(class_ok.size(), 1)));
        constexpr size_t kStagedFoldBusBytes = 256 * 1024;
        const size_t fold_blocks = std::min<size_t>(4096, std::max<size_t>(1, ((size_t)n + 255) / 256));
        const unsigned char* staged = class_ok.size() <= pe_fold_feas_max_classes() &&
                                              class_ok.size() * fold_blocks <= kStagedFoldBusBytes
                                          ? stage_only(s, class_ok)
                                          : nullptr;
        {
            const int rc = flush_fold(s);   // an earlier table's fold first (stream order)
            if (rc) return rc;
        }
        if (staged) {
            pe::FoldArgs F;
            F.class_src = staged;
            F.class_dst = g.class_ok.as<uint8_t>();
            F.ncls = (uint32_t)class_ok.size();
            F.node_ok = g.node_ok_used ? g.node_ok.as<uint8_t>() : nullptr;
            F.feas = g.node_feas.as<uint8_t>();
            s->pending_fold = F;
            s->fold_pending = true;
            if (!s->fold_defer_ok) {
                const int rc = flush_fold(s);
                if (rc) return rc;
            }
        } else {
            HIP_TRY(s, upload_s(s, g.class_ok, class_ok));
            HIP_TRY(s, pe_launch_fold_feas(&soa, g.class_ok.as<uint8_t>(),
                                           g.node_ok_used ? g.node_ok.as<uint8_t>() : nullptr,
                                           g.node_feas.as<uint8_t>(), s->stream));
        }
    }

    ApiScope prof_aff_(s, "tables.affinity+rest");
    // NodeAffinityIterator score per class (rank.go:698-725)
    g.has_aff_table = !g.affinities.empty();
    g.node_aff_used = false;
    if (g.has_aff_table) {
        bool escapes = false;
        for (auto& a : g.affinities)
            escapes = escapes || a.c.escapes || a.c.l.kind == T_ID || a.c.l.kind == T_NAME ||
                      a.c.r.kind == T_ID || a.c.r.kind == T_NAME;
        auto score = [&](const NodeView& nd) {
            double sum_w = 0.0;
            for (auto& a : g.affinities) sum_w += std::fabs((double)a.weight);
            double total = 0.0;
            for (auto& a : g.affinities) if (meets(s, ev, a.c, nd)) total += (double)a.weight;
            const double norm = total / sum_w;
            return total != 0.0 ? norm : 0.0;
        };
        if (escapes) {
            std::vector<double> na(n);
            for (size_t i = 0; i < n; i++) na[i] = score(s->view((uint32_t)i));
            HIP_TRY(s, upload_s(s, g.node_aff, na));
            g.node_aff_used = true;
            g.h_aff_node = std::move(na);
            g.h_aff_class.clear();
        } else {
            std::string ak;   // the affinities' texts and weights: the per-class scores' inputs
            for (auto& a : g.affinities) { ak += a.c.text; ak += '\x1f'; ak += std::to_string(a.weight); ak += '\x1f'; }
            cls_cache_sync(s);
            auto ct = s->cc_aff.find(ak);
            if (ct == s->cc_aff.end() || ct->second.size() != s->ncls) {
                std::vector<double> v(s->ncls);
                for (uint32_t c = 0; c < s->ncls; c++) v[c] = score(s->view(s->class_rep[c]));
                ct = s->cc_aff.insert_or_assign(ak, std::move(v)).first;
            }
            std::vector<double> ca = ct->second;
            HIP_TRY(s, upload_s(s, g.class_aff, ca));
            g.h_aff_class = std::move(ca);
            g.h_aff_node.clear();
        }
    } else {
        g.h_aff_class.clear();
        g.h_aff_node.clear();
    }
    g.aux_valid = false;
    // AssignPorts needs an address of the ports' host network on the node
    g.alias_used = false;
    if (g.ask.tg_dyn > 0) {
        const uint32_t want = g.net_host;
        // a property of the node table alone: a recycled plan's buffer built for
        // the same host network on the same node table is reused (no upload)
        if (g.alias_for != want || g.alias_gen != s->nodes_gen || g.alias_ok.bytes < n) {
            std::vector<uint8_t> al(n, 0);
            for (size_t i = 0; i < n; i++) {
                const auto a = s->view((uint32_t)i).aliases;
                al[i] = std::find(a.begin(), a.end(), want) != a.end();
            }
            HIP_TRY(s, upload_s(s, g.alias_ok, al));
            g.alias_for = want;
            g.alias_gen = s->nodes_gen;
        }
        g.alias_used = true;
    }
    if (has_static(g)) {
        // AssignPorts' static ports (network.go:317-363) or the task network's
        // (AssignNetwork, :407-442) on the current plan: a node is blocked when a
        // port is invalid, its host network has no address, or the port is used
        // on that address (the node's reservations, ReservedHostPorts, the
        // proposed snapshot allocs, this group's placements). The device adds
        // the group's later placements (gate).
        std::vector<uint8_t> own(n, 0), blocked(n, 0);
        for (auto& p : plan_of(s))
            if (p.first == g.name && p.second < n) own[p.second] = 1;
        const bool task = g.rports.empty();
        for (uint32_t r = 0; r < (uint32_t)n; r++)
            blocked[r] = (own[r] || (task ? task_port_reason(s, g, r, nullptr) : static_port_reason(s, g, r, nullptr)))
                             ? 1 : 0;
        DevMem& gate = task ? g.task_gate : g.static_gate;
        DevMem& bl = task ? g.task_blocked : g.static_blocked;
        HIP_TRY(s, upload_s(s, bl, blocked));
        HIP_TRY(s, gate.ensure(sizeof(uint32_t) * std::max<size_t>(n, 1)));
        HIP_TRY_STATE(s, pe_launch_static_gate(bl.as<uint8_t>(), g.coll_tg.as<uint32_t>(), gate.as<uint32_t>(), (uint32_t)n,
                                         s->stream));
        // PreemptForNetwork's reserved-port step per node, for Selects with Preempt
        std::vector<uint64_t> plist(n);
        std::vector<uint8_t> pinfo(n);
        std::vector<uint64_t> pblock(n);
        for (uint32_t r = 0; r < (uint32_t)n; r++) port_step(s, g, r, own[r] != 0, &plist[r], &pinfo[r], &pblock[r]);
        HIP_TRY(s, upload_s(s, g.port_list, plist));
        HIP_TRY(s, upload_s(s, g.port_info, pinfo));
        HIP_TRY(s, upload_s(s, g.port_block, pblock));
    }
    g.md_on = false;
    if (tg_md(s, g)) {   // task network on multi-device nodes: the host's first fit and verdicts
        const int rc = build_md(s, g);
        if (rc) return rc;
    }
    g.tables_valid = true;
    return PE_OK;
}

pe::TgTables tables_of(TgPlan& g) {
    pe::TgTables t;
    std::memset(&t, 0, sizeof(t));
    t.class_ok = g.class_ok.as<uint8_t>();
    t.node_ok = g.node_ok_used ? g.node_ok.as<uint8_t>() : nullptr;
    t.node_feas = g.node_feas.as<uint8_t>();
    t.class_aff = (g.has_aff_table && !g.node_aff_used) ? g.class_aff.as<double>() : nullptr;
    t.node_aff = g.node_aff_used ? g.node_aff.as<double>() : nullptr;
    t.alias_ok = g.alias_used ? g.alias_ok.as<uint8_t>() : nullptr;
    t.static_gate = g.rports.empty() ? nullptr : g.static_gate.as<uint32_t>();
    t.task_gate = g.trports.empty() ? nullptr : g.task_gate.as<uint32_t>();
    t.port_list = has_static(g) ? g.port_list.as<uint64_t>() : nullptr;
    t.port_info = has_static(g) ? g.port_info.as<uint8_t>() : nullptr;
    t.port_block = has_static(g) ? g.port_block.as<uint64_t>() : nullptr;
    t.md = g.md_on ? g.md_dev.as<pe::MdNet>() : nullptr;
    t.coll_tg = g.coll_tg.as<uint32_t>();
    if (!g.dev_reqs.empty()) {
        t.dev_free = g.dev_free;
        t.dev_cls = g.dev_cls.as<pe::DevClass>();
    }
    t.n_psets = (int)g.psets.size();
    t.n_spread = g.n_spread;
    for (int p = 0; p < t.n_psets; p++) {
        PsetDev& ps = *g.psets[p];
        t.pset_allowed[p] = ps.allowed;
        t.pset_val_class[p] = ps.val_class.as<uint32_t>();
        t.pset_val_node[p] = ps.per_node ? ps.val_node.as<uint32_t>() : nullptr;
        t.pset_counts[p] = ps.counts.as<uint32_t>();
        t.pset_desired[p] = ps.desired.as<double>();
        t.pset_nvals[p] = (int)ps.value_str.size();
        t.pset_even[p] = ps.even ? 1 : 0;
        t.pset_weight_frac[p] = ps.weight_frac;
        // per-value tables set after set (one spare boost entry per set)
        t.pset_tab_off[p] = t.pset_tab_total;
        t.pset_cnt_off[p] = t.pset_cnt_total;
        t.pset_tab_total += (uint32_t)t.pset_nvals[p] + 1u;
        t.pset_cnt_total += (uint32_t)t.pset_nvals[p];
    }
    return t;
}

// Bytes of a task group's spread boost table in HBM (the pset_tab_off layout).
size_t spread_tab_bytes(const TgPlan& g) {
    size_t v = 0;
    for (auto& ps : g.psets) v += ps->value_str.size() + 1;
    return sizeof(double) * std::max<size_t>(v, 1);
}

// Bytes of the fused count loop's per-value tables (spread boosts + use
// counts) in LDS, or 0 when they are kept in HBM instead (beyond the budget).
constexpr size_t kPsetLdsBudget = 48 * 1024;
size_t pset_lds_bytes(const pe::TgTables& t) {
    const size_t b = (sizeof(double) * t.pset_tab_total + 4u * t.pset_cnt_total + 15u) & ~(size_t)15u;
    return b <= kPsetLdsBudget ? b : 0u;
}

int prepare_tg(pe_stack* s, uint32_t tgi, const std::vector<uint32_t>& order, uint32_t start) {
    ApiScope prof_(s, "prepare_tg");
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    if (!s->have_job) return s->fail(PE_ESTATE, "pe_set_job not called");
    if (tgi >= s->tgs.size()) return s->fail(PE_EINVAL, "task group index out of range");
    TgPlan& g = *s->tgs[tgi];
    if (!g.unsupported.empty()) return s->fail(PE_EUNSUPPORTED, g.unsupported);
    if (!s->cores_unsupported.empty()) return s->fail(PE_EUNSUPPORTED, s->cores_unsupported);
    if (g.ask.cores > 0 && !s->cores_tg_unsupported.empty()) return s->fail(PE_EUNSUPPORTED, s->cores_tg_unsupported);
    if (!g.psets_built) {
        ApiScope prof_p_(s, "prepare_tg.psets");
        int rc = build_psets(s, g);
        if (rc) return rc;
        if (!g.unsupported.empty()) return s->fail(PE_EUNSUPPORTED, g.unsupported);
    }
    if (g.tables_valid && g.md_on) {   // another group's placements moved the nodes' dynamic ports
        size_t other = 0;
        for (auto& p : plan_of(s)) other += p.first != g.name;
        if (other != g.md_other) g.tables_valid = false;
    }
    if (!g.tables_valid) {
        ApiScope prof_t_(s, "prepare_tg.tables");
        int rc = build_tables(s, g, order, start);
        if (rc) return rc;
    }
    return PE_OK;
}

pe::Ask ask_for(pe_stack* s, TgPlan& g) {
    pe::Ask a = g.ask;
    const bool generic = s->cfg.stack_kind == PE_STACK_GENERIC;
    if (!generic) { a.distinct_job = 0; a.distinct_tg = 0; a.desired_count = 0; }
    a.algo_spread = s->cfg.algorithm == PE_ALGO_SPREAD;
    a.anti_aff = generic ? 1 : 0;
    return a;
}

// Job-level distinct_property counts every task group's allocs: after a commit
// of one group the other groups' value counts are rebuilt from the plan.
void invalidate_job_distinct(pe_stack* s, uint32_t tgi) {
    bool job_distinct = false;
    for (auto& c : s->job_constraints) job_distinct = job_distinct || c.op == "distinct_property";
    if (!job_distinct) return;
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi) s->tgs[k]->psets_built = false;
}

void invalidate_tables(pe_stack* s) {
    for (auto& g : s->tgs) g->tables_valid = false;
}

// Largest overlay (log2 entries) that fits the LDS budget of one workgroup.
// Where a FULL k_place keeps its per-value tables: dynamic LDS (A.pset_lds
// bytes) while they fit the budget, else one HBM set per evaluation.
int place_pset_tables(pe_stack* s, pe::BatchArgs& A, uint32_t n_evals, DevMem& buf) {
    A.pset_g_tab = nullptr;
    A.pset_g_cnt = nullptr;
    A.pset_lds = (uint32_t)pset_lds_bytes(A.tg);
    if (A.pset_lds || A.tg.n_psets == 0) return PE_OK;
    const size_t tb = sizeof(double) * A.tg.pset_tab_total * (size_t)n_evals;
    const size_t cb = 4u * A.tg.pset_cnt_total * (size_t)n_evals;
    HIP_TRY(s, buf.ensure(tb + cb));
    A.pset_g_tab = buf.as<double>();
    A.pset_g_cnt = reinterpret_cast<uint32_t*>(buf.as<unsigned char>() + tb);
    return PE_OK;
}

int max_hash_bits(bool full, size_t pset_bytes) {
    int bits = 12;
    while (bits > 6 && pe_place_lds_bytes(full, bits, false, pset_bytes) > 96 * 1024) bits--;
    return bits;
}

int hash_bits_for(uint32_t count, bool full, size_t pset_bytes) {
    int bits = 6;
    while (bits < 30 && (1u << bits) < 2u * std::max<uint32_t>(count, 1)) bits++;
    return std::min(bits, max_hash_bits(full, pset_bytes));
}

// Count bits of a packed windowed-kernel overlay entry (row << kbits | k), or 0
// when the rows or `max_k` placements per node do not fit in 32 bits. Rows stay
// below 2^rowbits - 1 so no entry equals the empty marker.
int packed_kbits(const pe_stack* s, uint32_t max_k, bool full) {
    if (full) return 0;
    int rowbits = 1;
    while (rowbits < 32 && ((uint64_t)1 << rowbits) <= (uint64_t)s->nodes.size()) rowbits++;
    const int kbits = 32 - rowbits;
    if (kbits < 2 || (uint64_t)max_k > ((uint64_t)1 << kbits) - 1) return 0;
    return kbits;
}

pe::BatchArgs batch_args(pe_stack* s, TgPlan& g) {
    pe::BatchArgs A;
    std::memset(&A, 0, sizeof(A));
    A.soa = soa_of(s);
    A.tg = tables_of(g);
    A.ask = ask_for(s, g);
    A.limit = s->limit;
    A.log10 = s->log10;
    A.net_overlay = (g.ask.tg_dyn > 0 || g.ask.has_task_net) ? 1 : 0;
    return A;
}

// Fold the sweep's per-node inputs into one u32 per node (SweepArgs::node_aux)
// when they fit: at most kAuxPsets spread properties of at most 255 values and
// at most kAuxValues distinct affinity scores. Otherwise the sweep resolves
// them through the class tables.
int build_aux(pe_stack* s, TgPlan& g, const pe::TgTables& t) {
    g.aux_valid = true;
    g.aux_ok = false;
    if (t.n_psets > pe::kAuxPsets) return PE_OK;
    for (int p = 0; p < t.n_psets; p++)
        if (t.pset_nvals[p] > (int)pe::kAuxMissing) return PE_OK;
    // intern the affinity scores: index 0 is 0.0 (no score appended)
    std::vector<double> vals{0.0};
    std::map<uint64_t, uint8_t> index{{0, 0}};
    const std::vector<double>& src = g.h_aff_node.empty() ? g.h_aff_class : g.h_aff_node;
    std::vector<uint8_t> idx(src.size(), 0);
    for (size_t i = 0; i < src.size(); i++) {
        uint64_t bits;
        std::memcpy(&bits, &src[i], 8);
        auto it = index.find(bits);
        if (it == index.end()) {
            if (vals.size() >= (size_t)pe::kAuxValues) return PE_OK;
            it = index.emplace(bits, (uint8_t)vals.size()).first;
            vals.push_back(src[i]);
        }
        idx[i] = it->second;
    }
    vals.resize(pe::kAuxValues, 0.0);
    HIP_TRY(s, upload_s(s, g.aff_vals, vals));
    if (!idx.empty()) HIP_TRY(s, upload_s(s, g.aff_idx, idx));
    const size_t n = s->nodes.size();
    HIP_TRY(s, g.node_aux.ensure(sizeof(uint32_t) * std::max<size_t>(n, 1)));
    pe::NodeSoA soa = soa_of(s);
    const uint8_t* per_class = (!idx.empty() && g.h_aff_node.empty()) ? g.aff_idx.as<uint8_t>() : nullptr;
    const uint8_t* per_node = (!idx.empty() && !g.h_aff_node.empty()) ? g.aff_idx.as<uint8_t>() : nullptr;
    HIP_TRY(s, pe_launch_fold_aux(&soa, &t, per_class, per_node, g.node_aux.as<uint32_t>(), s->stream));
    g.aux_ok = true;
    return PE_OK;
}

bool full_scan_kernel(pe_stack* s, TgPlan& g, uint32_t n) {
    return !g.psets.empty() || s->limit >= n;
}

// Full-scan Select (limit >= n) as a multi-CU sweep: every workgroup reduces
// its rows to a SweepRec, one merge yields the winner.
// Visit position of every row (PE_NONE: not listed) for the sweep paths.
int ensure_rank_of(pe_stack* s) {
    if (s->rank_of_valid) return PE_OK;
    std::vector<uint32_t> rank_of(s->nodes.size(), PE_NONE);
    for (uint32_t i = 0; i < (uint32_t)s->visit.size(); i++) rank_of[s->visit[i]] = i;
    HIP_TRY(s, upload_s(s, s->d_rank_of, rank_of));
    s->rank_of_valid = true;
    return PE_OK;
}

// The sweep over snapshot rows [row_begin, row_end) (one GPU's shard, or all
// rows): per-workgroup SweepRec records merged into *rec.
// SweepArgs and grid of one full-pass Select over rows [row_begin, row_end)
// (tables, aux fold, penalty bits); no launch.
int sweep_setup(pe_stack* s, TgPlan& g, const pe_select_options* opts, uint32_t row_begin, uint32_t row_end,
                pe::SweepArgs* args, uint32_t* blocks_out) {
    const uint32_t n = (uint32_t)s->visit.size();
    pe::SweepArgs& A = *args;
    std::memset(&A, 0, sizeof(A));
    A.soa = soa_of(s);
    A.tg = tables_of(g);
    A.ask = ask_for(s, g);
    {
        const int rc = ensure_rank_of(s);
        if (rc) return rc;
    }
    A.rank_of = s->d_rank_of.as<uint32_t>();
    A.n_visit = n;
    A.offset = s->offset;
    A.row_begin = row_begin;
    A.row_end = row_end;
    A.log10 = s->log10;
    if (opts && opts->penalty_count > 0) {
        std::vector<uint32_t> bits((s->nodes.size() + 31) / 32, 0);
        for (uint32_t i = 0; i < opts->penalty_count; i++) {
            uint32_t r = opts->penalty_rows[i];
            if (r < s->nodes.size()) bits[r >> 5] |= 1u << (r & 31);
        }
        HIP_TRY(s, upload_s(s, s->d_penalty, bits));
        A.penalty_bits = s->d_penalty.as<uint32_t>();
    }
    if (!g.psets.empty()) {
        HIP_TRY(s, s->d_spread_tab.ensure(spread_tab_bytes(g)));
        A.spread_tab = s->d_spread_tab.as<double>();
    }
    if (!g.aux_valid) {
        ApiScope prof_a_(s, "sweep.build_aux");
        int rc = build_aux(s, g, A.tg);
        if (rc) return rc;
    }
    bool use_aux = g.aux_ok;
    if (const char* e = std::getenv("PE_SWEEP_AUX")) use_aux = use_aux && std::atoi(e) != 0;
    if (use_aux) {
        A.node_aux = g.node_aux.as<uint32_t>();
        A.aff_vals = g.aff_vals.as<double>();
    }
    s->last_sweep_bytes = use_aux ? 76u : 73u;
    // exactly one round of resident workgroups: a grid-stride pass with no
    // tail, and few records for the merge
    uint32_t blocks = (A.row_end - A.row_begin + 256 * 8 - 1) / (256 * 8);
    uint32_t per_cu = (uint32_t)(use_aux ? s->sweep_per_cu_aux : s->sweep_per_cu);
    if (const char* e = std::getenv("PE_SWEEP_BPC")) per_cu = (uint32_t)std::max(1, std::atoi(e));
    blocks = std::max<uint32_t>(1, std::min<uint32_t>(blocks, (uint32_t)s->n_cu * per_cu));
    HIP_TRY(s, s->d_sweep_recs.ensure(sizeof(pe::SweepRec) * blocks));
    HIP_TRY(s, s->d_sweep_merged.ensure(sizeof(pe::SweepRec)));
    HIP_TRY(s, s->d_record.ensure(sizeof(pe_ranked_node)));
    A.recs = s->d_sweep_recs.as<pe::SweepRec>();
    *blocks_out = blocks;
    return PE_OK;
}

int sweep_partial(pe_stack* s, TgPlan& g, const pe_select_options* opts, uint32_t row_begin, uint32_t row_end,
                  pe::SweepArgs* args, pe::SweepRec* rec) {
    pe::SweepArgs& A = *args;
    uint32_t blocks = 0;
    int rc = sweep_setup(s, g, opts, row_begin, row_end, args, &blocks);
    if (rc) return rc;
    if (A.spread_tab) HIP_TRY(s, pe_launch_spread_table(&A.tg, s->d_spread_tab.as<double>(), s->stream));
    if (row_end <= row_begin) {   // an empty shard contributes the identity record
        pe_rec_init(rec);
        s->last_ms = s->last_sweep_ms = 0;
        s->last_ms_pending = false;
        return PE_OK;
    }
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    HIP_TRY_STATE(s, pe_launch_sweep(&A, blocks, s->d_sweep_merged.as<pe::SweepRec>(), s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    HIP_TRY(s, hipMemcpyAsync(rec, s->d_sweep_merged.p, sizeof(*rec), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    s->last_sweep_ms = ms;
    return PE_OK;
}

// Resolve a merged record into the Select result (winner record from the
// resident snapshot; a full pass leaves the cursor unchanged).
int sweep_finish(pe_stack* s, pe::SweepArgs& A, const pe::SweepRec& rec, pe_ranked_node* out) {
    const uint32_t n = (uint32_t)s->visit.size();
    std::memset(out, 0, sizeof(*out));
    const uint32_t rank = pe_rec_winner(&rec);
    out->row = -1;
    out->nodes_evaluated = n;   // every node is pulled: the stream is exhausted
    out->nodes_filtered = rec.filtered;
    out->nodes_exhausted = rec.exhausted;
    out->new_offset = s->offset;   // a full pass leaves the cursor unchanged
    if (rank != PE_NONE) {
        uint32_t pos = s->offset + rank;
        if (pos >= n) pos -= n;
        const uint32_t row = s->visit[pos];
        HIP_TRY_STATE(s, pe_launch_node_record(&A, row, s->d_record.as<pe_ranked_node>(), s->stream));
        pe_ranked_node rr;
        HIP_TRY(s, hipMemcpyAsync(&rr, s->d_record.p, sizeof(rr), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        out->row = (int32_t)row;
        out->final_score = rr.final_score;
        out->n_scores = rr.n_scores;
        std::memcpy(out->scores, rr.scores, sizeof(out->scores));
        out->n_device_offers = rr.n_device_offers;
        std::memcpy(out->device_offer_group, rr.device_offer_group, sizeof(out->device_offer_group));
    }
    return PE_OK;
}

int run_sweep_select(pe_stack* s, TgPlan& g, const pe_select_options* opts, pe_ranked_node* out) {
    pe::SweepArgs A;
    pe::SweepRec rec;
    int rc = sweep_partial(s, g, opts, 0, (uint32_t)s->nodes.size(), &A, &rec);
    if (rc) return rc;
    return sweep_finish(s, A, rec, out);
}

// Options / filtered / exhausted over the current visit list (k_census).
int census(pe_stack* s, TgPlan& g, uint32_t* cnt) {
    pe::BatchArgs A = batch_args(s, g);
    HIP_TRY(s, upload_visit(s, s->visit));
    A.perms = s->d_visit.as<uint32_t>();
    A.n_visit = (uint32_t)s->visit.size();
    HIP_TRY(s, s->d_ev_out.ensure(16));
    HIP_TRY(s, hipMemsetAsync(s->d_ev_out.p, 0, 16, s->stream));
    HIP_TRY_STATE(s, pe_launch_census(&A, s->d_ev_out.as<uint32_t>(), nullptr, nullptr, s->stream));
    HIP_TRY(s, hipMemcpyAsync(cnt, s->d_ev_out.p, 3 * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    return PE_OK;
}

constexpr uint32_t kParallelMinNodes = 4096;   // lists shorter than this keep the fused loop
constexpr uint64_t kParallelWalk = 4096;        // expected positions per windowed Select

// A plain Select over the visit list from the cursor with every position
// evaluated in parallel (k_census with outcomes) and LimitIterator +
// MaxScoreIterator resolved on the device (k_evict_resolve).
int run_parallel_select(pe_stack* s, TgPlan& g, pe_ranked_node* out, uint32_t* new_offset);

// Preemptor inputs on the device for the current job / task group.
pe::PreemptArgs preempt_args(pe_stack* s, TgPlan& g) {
    pe::PreemptArgs P;
    std::memset(&P, 0, sizeof(P));
    P.soa = soa_of(s);
    P.tg = tables_of(g);
    P.ask = ask_for(s, g);
    P.node_alloc_off = s->d_node_alloc_off.as<uint32_t>();
    P.allocs = s->d_palloc.as<pe::PreemptAlloc>();
    P.preempted = s->d_preempted.as<uint8_t>();
    P.pcount = s->d_pcount.as<uint32_t>();
    P.own_existing = s->d_own_existing.as<uint32_t>();
    P.job_key = s->job_key;
    P.job_priority = s->job_priority;
    P.log10 = s->log10;
    P.score_preemption = s->cfg.stack_kind == PE_STACK_GENERIC ? 1 : 0;
    P.palloc_cores = s->has_cores ? s->d_palloc_cores.as<uint64_t>() : nullptr;
    P.mask_words = s->evict_words;
    return P;
}

// The next wider eviction width after a launch flagged kEvictWider (a node's
// ProposedAllocs outgrew it), or 0 when none is left.
static uint32_t wider_words(uint32_t w) {
    for (uint32_t x : pe::kEvictWidths)
        if (x > w) return x;
    return 0;
}

// Record `o`'s PreemptedAllocs from the preempted set of its node (`mask`, W
// words over the node's CSR slots): inline up to PE_MAX_PREEMPT, the full
// list kept under record index `rec` beyond that (pe_preempted_of). With
// `commit` the allocs also join the host mirror of Plan.NodePreemptions (the
// device loop already applied them).
static void set_preempted(pe_stack* s, pe_ranked_node& o, uint32_t rec, uint32_t row, const uint32_t* mask,
                          uint32_t words, bool commit) {
    const uint32_t b = s->h_node_alloc_off[row], m = s->h_node_alloc_off[row + 1] - b;
    o.n_preempted = 0;
    std::vector<uint32_t> full;
    for (uint32_t i = 0; i < m && i < 32u * words; i++) {
        if (!((mask[i >> 5] >> (i & 31u)) & 1u)) continue;
        const uint32_t a = s->h_palloc_index[b + i];
        if (o.n_preempted < PE_MAX_PREEMPT) o.preempted[o.n_preempted] = a;
        o.n_preempted++;
        full.push_back(a);
        if (commit) {
            s->h_preempted[b + i] = 1;
            core_hold(s, a, false);
            invalidate_static(s);
        }
    }
    if (o.n_preempted > PE_MAX_PREEMPT) {
        for (auto& e : s->pre_overflow)
            if (e.first == rec) { e.second = std::move(full); return; }
        s->pre_overflow.emplace_back(rec, std::move(full));
    }
}

// The full PreemptedAllocs of record `rec` of the current call.
static const uint32_t* preempted_list(const pe_stack* s, uint32_t rec, const pe_ranked_node& o) {
    if (o.n_preempted <= PE_MAX_PREEMPT) return o.preempted;
    for (auto& e : s->pre_overflow)
        if (e.first == rec && e.second.size() == o.n_preempted) return e.second.data();
    return nullptr;
}

int run_parallel_select(pe_stack* s, TgPlan& g, pe_ranked_node* out, uint32_t* new_offset) {
    std::memset(out, 0, sizeof(*out));
    out->row = -1;
    const uint32_t n = (uint32_t)s->visit.size();
    *new_offset = n ? s->offset % n : 0;
    if (n == 0) return PE_OK;
    pe::BatchArgs A = batch_args(s, g);
    HIP_TRY(s, upload_visit(s, s->visit));
    A.perms = s->d_visit.as<uint32_t>();
    A.n_visit = n;
    HIP_TRY(s, s->d_ev_status.ensure(n));
    HIP_TRY(s, s->d_ev_score.ensure(sizeof(double) * n));
    HIP_TRY(s, s->d_ev_out.ensure(16));
    HIP_TRY(s, s->d_ev_mask.ensure(sizeof(uint32_t) * (pe::kEvictMaxWords + 1)));
    HIP_TRY(s, s->d_ev_flags.ensure(16));
    HIP_TRY(s, s->d_record.ensure(sizeof(pe_ranked_node)));
    HIP_TRY(s, hipMemsetAsync(s->d_ev_out.p, 0, 16, s->stream));
    HIP_TRY_STATE(s, pe_launch_census(&A, s->d_ev_out.as<uint32_t>(), s->d_ev_status.as<uint8_t>(),
                                s->d_ev_score.as<double>(), s->stream));
    pe::EvictResolveArgs R;
    R.status = s->d_ev_status.as<uint8_t>();
    R.score = s->d_ev_score.as<double>();
    R.n = n;
    R.offset = s->offset % n;
    R.limit = s->limit;
    R.out = s->d_ev_out.as<int32_t>();
    HIP_TRY_STATE(s, pe_launch_resolve(&R, s->stream));
    int32_t res[4];
    HIP_TRY(s, hipMemcpyAsync(res, R.out, sizeof(res), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    const uint32_t consumed = (uint32_t)res[1];
    out->nodes_evaluated = consumed;
    out->nodes_filtered = (uint32_t)res[2];
    out->nodes_exhausted = (uint32_t)res[3];
    *new_offset = (uint32_t)(((uint64_t)(s->offset % n) + consumed) % n);
    out->new_offset = *new_offset;
    if (res[0] >= 0) {
        // the option's record: BinPack with evict gives the plain result on a
        // node that fits (no preemption, no preemption score)
        const uint32_t row = s->visit[(uint32_t)(((uint64_t)(s->offset % n) + (uint32_t)res[0]) % n)];
        pe::PreemptArgs P = preempt_args(s, g);
        P.visit = s->d_visit.as<uint32_t>();
        P.n_visit = n;
        P.flags = s->d_ev_flags.as<uint32_t>();
        pe_ranked_node rr;
        for (;;) {   // the node's ProposedAllocs may have outgrown the width: the record wider
            HIP_TRY_STATE(s, pe_launch_evict_record(&P, row, s->d_record.as<pe_ranked_node>(),
                                                    s->d_ev_mask.as<uint32_t>(), s->stream));
            uint32_t fl = 0;
            HIP_TRY(s, hipMemcpyAsync(&rr, s->d_record.p, sizeof(rr), hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(s, hipMemcpyAsync(&fl, s->d_ev_mask.as<uint32_t>() + P.mask_words, sizeof(fl),
                                      hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(s, hipStreamSynchronize(s->stream));
            if (!(fl & pe::kEvictWider)) break;
            P.mask_words = wider_words(P.mask_words);
            if (!P.mask_words) return s->fail(PE_EUNSUPPORTED, "preemption: a node's proposed allocs exceed the "
                                                                "widest eviction width");
        }
        out->row = (int32_t)row;
        out->final_score = rr.final_score;
        out->n_scores = rr.n_scores;
        std::memcpy(out->scores, rr.scores, sizeof(out->scores));
        out->n_device_offers = rr.n_device_offers;
        std::memcpy(out->device_offer_group, rr.device_offer_group, sizeof(out->device_offer_group));
    }
    return PE_OK;
}

// Select with Preempt=true (BinPack evict, rank.go:193-527 + PreemptionScoringIterator)
// over `order` from cursor `offset`: every position evaluated in parallel, then
// the LimitIterator window resolved on the device.
int run_evict_select(pe_stack* s, TgPlan& g, const std::vector<uint32_t>& order, uint32_t offset,
                     const pe_select_options* opts, pe_ranked_node* out, uint32_t* new_offset, uint32_t rec = 0,
                     uint32_t words = 0) {
    std::memset(out, 0, sizeof(*out));
    out->row = -1;
    const uint32_t n = (uint32_t)order.size();
    *new_offset = n ? offset % n : 0;
    if (!s->preempt_unsupported.empty()) return s->fail(PE_EUNSUPPORTED, "preemption: " + s->preempt_unsupported);
    if (g.ask.cores > 0) return s->fail(PE_EUNSUPPORTED, "reserved cores with preemption");
    if (n == 0) return PE_OK;
    pe::PreemptArgs P = preempt_args(s, g);
    if (words) P.mask_words = words;
    HIP_TRY(s, upload_visit(s, order));
    P.visit = s->d_visit.as<uint32_t>();
    P.n_visit = n;
    if (opts && opts->penalty_count > 0) {
        std::vector<uint32_t> bits((s->nodes.size() + 31) / 32, 0);
        for (uint32_t i = 0; i < opts->penalty_count; i++) {
            uint32_t r = opts->penalty_rows[i];
            if (r < s->nodes.size()) bits[r >> 5] |= 1u << (r & 31);
        }
        HIP_TRY(s, upload_s(s, s->d_penalty, bits));
        P.penalty_bits = s->d_penalty.as<uint32_t>();
    }
    if (!g.psets.empty()) {
        HIP_TRY(s, s->d_spread_tab.ensure(spread_tab_bytes(g)));
        HIP_TRY(s, pe_launch_spread_table(&P.tg, s->d_spread_tab.as<double>(), s->stream));
        P.spread_tab = s->d_spread_tab.as<double>();
    }
    HIP_TRY(s, s->d_ev_status.ensure(n));
    HIP_TRY(s, s->d_ev_score.ensure(sizeof(double) * n));
    HIP_TRY(s, s->d_ev_flags.ensure(16));
    HIP_TRY(s, s->d_ev_out.ensure(16));
    HIP_TRY(s, s->d_ev_mask.ensure(sizeof(uint32_t) * (pe::kEvictMaxWords + 1)));
    HIP_TRY(s, s->d_record.ensure(sizeof(pe_ranked_node)));
    HIP_TRY(s, hipMemsetAsync(s->d_ev_flags.p, 0, 16, s->stream));
    P.status = s->d_ev_status.as<uint8_t>();
    P.score = s->d_ev_score.as<double>();
    P.flags = s->d_ev_flags.as<uint32_t>();
    pe::EvictResolveArgs R;
    R.status = P.status;
    R.score = P.score;
    R.n = n;
    R.offset = offset % n;
    R.limit = s->limit;
    R.out = s->d_ev_out.as<int32_t>();
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    HIP_TRY_STATE(s, pe_launch_evict(&P, &R, s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    int32_t res[4];
    uint32_t flags = 0;
    HIP_TRY(s, hipMemcpyAsync(res, R.out, sizeof(res), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipMemcpyAsync(&flags, P.flags, sizeof(flags), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    if (flags & pe::kEvictUnsup)
        return s->fail(PE_EUNSUPPORTED, "preemption: a node outside the device path (several network devices, "
                                        "static ports on a node of more than 32 allocs, reserved cores)");
    if (flags & pe::kEvictWider) {   // a node's ProposedAllocs outgrew the width: the same Select wider
        const uint32_t w = wider_words(P.mask_words);
        if (!w) return s->fail(PE_EUNSUPPORTED, "preemption: a node's proposed allocs exceed the widest eviction width");
        return run_evict_select(s, g, order, offset, opts, out, new_offset, rec, w);
    }
    const uint32_t consumed = (uint32_t)res[1];
    out->nodes_evaluated = consumed;
    out->nodes_filtered = (uint32_t)res[2];
    out->nodes_exhausted = (uint32_t)res[3];
    *new_offset = (uint32_t)(((uint64_t)(offset % n) + consumed) % n);
    out->new_offset = *new_offset;
    if (res[0] >= 0) {
        const uint32_t row = order[(uint32_t)(((uint64_t)(offset % n) + (uint32_t)res[0]) % n)];
        HIP_TRY_STATE(s, pe_launch_evict_record(&P, row, s->d_record.as<pe_ranked_node>(), s->d_ev_mask.as<uint32_t>(),
                                          s->stream));
        pe_ranked_node rr;
        uint32_t mask[pe::kEvictMaxWords + 1];
        HIP_TRY(s, hipMemcpyAsync(&rr, s->d_record.p, sizeof(rr), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipMemcpyAsync(mask, s->d_ev_mask.p, sizeof(uint32_t) * (P.mask_words + 1), hipMemcpyDeviceToHost,
                                  s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        out->row = (int32_t)row;
        out->final_score = rr.final_score;
        out->n_scores = rr.n_scores;
        std::memcpy(out->scores, rr.scores, sizeof(out->scores));
        out->n_device_offers = rr.n_device_offers;
        std::memcpy(out->device_offer_group, rr.device_offer_group, sizeof(out->device_offer_group));
        set_preempted(s, *out, rec, row, mask, P.mask_words, false);
    }
    return PE_OK;
}

// A compact chain record as the full RankedNode (the leading fields are
// byte-identical; no preemptions or reserved cores on the chain path).
static inline void widen_rec(const pe::EmitRec& e, pe_ranked_node* o) {
    std::memcpy(o, &e, offsetof(pe::EmitRec, n_device_offers));
    std::memset(reinterpret_cast<char*>(o) + offsetof(pe_ranked_node, n_preempted), 0,
                sizeof(pe_ranked_node) - offsetof(pe_ranked_node, n_preempted));
    o->n_device_offers = e.n_device_offers;
    for (int q = 0; q < PE_MAX_DEVICE_REQ; q++) o->device_offer_group[q] = e.device_offer_group[q];
}

// One evaluation on the stack's plan (pe_select / pe_place): the fused count
// loop in launches of at most H/2 placements, each merging its overlay back
// into the HBM SoA so the plan persists.
int run_place(pe_stack* s, uint32_t tgi, uint32_t count, int commit, const std::vector<uint32_t>& order,
              uint32_t offset, const pe_select_options* opts, pe_ranked_node* out, uint32_t* placed,
              uint32_t* new_offset) {
    TgPlan& g = *s->tgs[tgi];
    *placed = 0;
    *new_offset = offset;
    if (order.empty()) {
        if (count) { std::memset(&out[0], 0, sizeof(out[0])); out[0].row = -1; }
        *new_offset = 0;
        return PE_OK;
    }
    const uint32_t n = (uint32_t)order.size();
    const bool full = full_scan_kernel(s, g, n);
    std::vector<pe::EmitRec>* sink = s->emit_sink;
    pe::BatchArgs A = batch_args(s, g);
    if (opts && opts->penalty_count > 0) {
        std::vector<uint32_t> bits((s->nodes.size() + 31) / 32, 0);
        for (uint32_t i = 0; i < opts->penalty_count; i++) {
            uint32_t r = opts->penalty_rows[i];
            if (r < s->nodes.size()) bits[r >> 5] |= 1u << (r & 31);
        }
        HIP_TRY(s, upload_s(s, s->d_penalty, bits));
        A.penalty_bits = s->d_penalty.as<uint32_t>();
    }
    if (full) {
        const int rc = place_pset_tables(s, A, 1, s->d_pset_g);
        if (rc) return rc;
    }
    A.hash_bits = hash_bits_for(count, full, A.pset_lds);
    A.packed_overlay = packed_kbits(s, 1u << A.hash_bits, full);
    bool chain = false;
    // the phase-static chain is compiled without reserved cores (k_chain's registers)
    if (!full && s->use_base && count > 1 && A.limit <= pe_chain_max_limit() && g.ask.cores == 0) {
        // count loop over one rotation at a time (k_base + k_chain): needs a
        // visit list without repeated rows
        chain = true;
        if (&order == &s->visit) {
            chain = s->visit_unique;   // checked once per SetNodes
        } else {
            std::vector<uint8_t> seen(s->nodes.size(), 0);
            for (uint32_t r : order) {
                if (seen[r]) { chain = false; break; }
                seen[r] = 1;
            }
        }
        if (chain) {
            // one evaluation: values in visit order (coalesced window reads)
            // PE_BASE_BY_ROW=1: the values by row instead (k_base reads the
            // records in row order, k_chain gathers the values through the list)
            static const bool by_row = std::getenv("PE_BASE_BY_ROW") != nullptr;
            HIP_TRY(s, s->d_base.ensure(sizeof(double) * std::max<size_t>(std::max<size_t>(s->nodes.size(), n), 1)));
            A.base = s->d_base.as<double>();
            A.base_by_pos = by_row ? 0 : 1;
            HIP_TRY(s, s->d_base1.ensure(sizeof(double) * std::max<size_t>(by_row ? s->nodes.size() : n, 1)));
            A.base1 = s->d_base1.as<double>();
            HIP_TRY(s, s->d_chain_vs.ensure(sizeof(double) * (size_t)pe_chain_max_n()));
            A.chain_vs = s->d_chain_vs.as<double>();
            if (std::getenv("PE_CHAIN_PROF")) {
                HIP_TRY(s, s->d_prof.ensure(32 * sizeof(unsigned long long)));
                HIP_TRY(s, hipMemset(s->d_prof.p, 0, 32 * sizeof(unsigned long long)));
                A.prof = s->d_prof.as<unsigned long long>();
            }
        }
    }
    bool staged_is_visit = false;
    {
        // the visit order: k_base of the chain reads a new list straight from
        // the staging ring and stores it to d_visit itself (no copy launch)
        ApiScope prof_up_(s, "run_place.upload_visit");
        const bool is_visit = &order == &s->visit;
        const unsigned char* src = nullptr;
        if (chain && A.base_by_pos && !(is_visit && s->d_visit_is_visit)) {
            HIP_TRY(s, s->d_visit.ensure(sizeof(uint32_t) * (size_t)n));
            src = stage_only(s, order);
        }
        if (src) {
            A.perm_src = reinterpret_cast<const uint32_t*>(src);
            A.perm_dst = s->d_visit.as<uint32_t>();
            s->d_visit_is_visit = false;   // until the launch that stores it is queued
            staged_is_visit = is_visit;
        } else {
            HIP_TRY(s, upload_visit(s, order));
        }
    }
    A.perms = s->d_visit.as<uint32_t>();
    A.n_visit = n;
    const uint32_t chunk = std::max<uint32_t>(1, (1u << A.hash_bits) / 2);
    // records and status land in mapped page-locked memory: the kernel writes
    // them over PCIe while it runs, one stream sync per launch
    HIP_TRY(s, s->h_place_out.ensure(sizeof(pe_ranked_node) * std::min(count, chunk)));
    HIP_TRY(s, s->h_place_status.ensure(16));
    A.commit = commit;
    A.writeback = commit;
    A.full_out = s->h_place_out.dev<pe_ranked_node>();
    A.eval_status = s->h_place_status.dev<uint32_t>();
    if (!A.full_out || !A.eval_status) return s->fail(PE_EHIP, "mapped result buffers unavailable");
    // the table build's pending fold: carried by the chain's first launch
    // (k_base pulls the class table into LDS per workgroup while that stays
    // small on the bus, the fused k_chain for short lists), else its own launch
    bool fused = false;
    // pending work this call's first launch carries: handed back when that
    // launch fails, so the next entry point still launches it
    bool fold_taken = false, counts_taken = false;
    const pe::FoldArgs fold_saved = s->pending_fold;
    const pe::CountArgs counts_saved = s->pending_counts;
    if (chain) {
        const uint32_t base_blocks = (2u * (uint32_t)n + 63u) / 64u;
        fused = A.base_by_pos && (uint32_t)n <= pe_chain_fused_max_n() && pe_chain_shape(n) <= 4 &&
                count <= pe_chain_fused_max_count() && count <= chunk &&
                s->nodes.size() <= 16384 && std::getenv("PE_CHAIN_FUSED") == nullptr;
        if (fused && s->fold_pending && s->pending_fold.ncls > pe_chain_fused_max_classes()) fused = false;
        if (s->fold_pending && (fused || (size_t)s->pending_fold.ncls * base_blocks <= 256u * 1024u)) {
            A.fold = s->pending_fold;
            s->fold_pending = false;
            fold_taken = true;
        }
    }
    {
        const int frc = flush_fold(s);
        if (frc) return frc;
    }
    if (chain) {
        // k_chain writes one compact entry per Select; k_emit (many workgroups)
        // builds the full records and writes the placements back (or, fused,
        // k_chain itself)
        if (fused) {
            A.fused = 1;
            A.base1 = nullptr;   // later phases re-evaluate rows holding placements
            HIP_TRY(s, s->d_fused_parts.ensure(sizeof(double) * PE_MAX_SCORES * std::max<size_t>(n, 1)));
            HIP_TRY(s, s->d_fused_nparts.ensure(std::max<size_t>(n, 1)));
            A.fused_parts = s->d_fused_parts.as<double>();
            A.fused_nparts = s->d_fused_nparts.as<uint8_t>();
            if (s->counts_pending) {   // SetJob's counts ride in this launch
                A.counts = s->pending_counts;
                s->counts_pending = false;
                counts_taken = true;
            }
        }
        const size_t cap = std::min(count, chunk);
        HIP_TRY(s, s->d_emit.ensure(sizeof(pe::ChainEmit) * cap));
        HIP_TRY(s, s->d_emit_ov.ensure(sizeof(uint2) * cap));
        if (!s->d_emit_n.p) {
            HIP_TRY(s, s->d_emit_n.ensure(4 * sizeof(uint32_t)));
            HIP_TRY(s, hipMemsetAsync(s->d_emit_n.p, 0, 4 * sizeof(uint32_t), s->stream));
        }
        A.emit = s->d_emit.as<pe::ChainEmit>();
        A.emit_ov = s->d_emit_ov.as<uint2>();
        A.emit_n = s->d_emit_n.as<uint32_t>();
        HIP_TRY(s, s->h_emit_out.ensure(sizeof(pe::EmitRec) * cap));
        A.emit_out = s->h_emit_out.dev<pe::EmitRec>();
        if (!A.emit_out) return s->fail(PE_EHIP, "mapped result buffers unavailable");
        A.full_out = nullptr;
    }
    double total_ms = 0;
    uint32_t done = 0;
    const bool hprof = std::getenv("PE_PLACE_PROF") != nullptr;
    double h_launch = 0, h_sync = 0, h_copy = 0;
    // The chain path ends with k_emit (or the fused k_chain), each of whose
    // workgroups raises its own completion word in the mapped h_emit_done
    // block (sequence place_seq): the host spins on them instead of waking
    // from a stream synchronisation; the launch's event timing is resolved
    // when it is asked for (pe_last_kernel_ms).
    bool spin = chain && s->spin_wait;
    volatile uint32_t* flag = nullptr;
    if (spin) {
        const size_t fb = sizeof(uint32_t) * pe_emit_grid(chunk);
        if (s->h_emit_done.bytes < fb) {
            HIP_TRY(s, s->h_emit_done.ensure(fb));
            std::memset(s->h_emit_done.p, 0, s->h_emit_done.bytes);
        }
        flag = s->h_emit_done.as<uint32_t>();
        A.done_flag = s->h_emit_done.dev<uint32_t>();
        HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    }
    while (done < count) {
        const uint32_t c = std::min(chunk, count - done);
        A.count = c;
        A.offset0 = *new_offset;
        const double t0 = hprof ? now_us() : 0.0;
        if (spin) {
            A.done_seq = ++s->place_seq;
        } else {
            HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
        }
        {
            ApiScope prof_l_(s, "run_place.launch");
            if (chain) {
                hipEvent_t* split = nullptr;
                if (s->kernel_split) {
                    for (auto& ev : s->ev_split)
                        if (!ev) HIP_TRY(s, hipEventCreate(&ev));
                    split = s->ev_split;
                }
                HIP_TRY_STATE(s, hipSuccess);   // whatever is still pending launches first
                const hipError_t le = pe_launch_chain(&A, 1, 1, s->stream, split);
                if (le != hipSuccess && done == 0) {
                    if (fold_taken) { s->pending_fold = fold_saved; s->fold_pending = true; }
                    if (counts_taken) { s->pending_counts = counts_saved; s->counts_pending = true; }
                }
                HIP_TRY(s, le);
                s->split_valid = split != nullptr;
            } else {
                s->split_valid = false;
                HIP_TRY_STATE(s, pe_launch_place(&A, 1, full, s->stream));
            }
            if (A.perm_src) {   // d_visit now holds the list (stream order)
                s->d_visit_is_visit = staged_is_visit;
                A.perm_src = nullptr;
                A.perm_dst = nullptr;
            }
            A.fold = pe::FoldArgs{};   // the first launch carried it
            HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
        }
        const double t1 = hprof ? now_us() : 0.0;
        ApiScope prof_w_(s, "run_place.wait+copy");
        if (spin) {
            const double t_spin = now_us();
            const uint32_t nwg = A.fused ? 1u : pe_emit_grid(c);
            uint32_t w = 0;   // completion words seen so far (in order)
            while (w < nwg) {
                if (flag[w] == A.done_seq) { w++; continue; }
                if (now_us() - t_spin >= 2000.0) break;
                __builtin_ia32_pause();
            }
            if (w < nwg) {
                HIP_TRY(s, hipStreamSynchronize(s->stream));
                while (w < nwg && flag[w] == A.done_seq) w++;
                if (w < nwg) return s->fail(PE_EHIP, "k_emit completion word missing");
            }
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
        } else {
            HIP_TRY(s, hipStreamSynchronize(s->stream));
            float ms = 0;
            HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
            total_ms += ms;
        }
        const double t2 = hprof ? now_us() : 0.0;
        uint32_t st[2];
        std::memcpy(st, const_cast<const uint32_t*>(s->h_place_status.as<uint32_t>()), sizeof(st));
        const uint32_t got = std::min(c, st[0] + 1);   // placed + the failing Select
        if (chain) {
            const pe::EmitRec* er = s->h_emit_out.as<pe::EmitRec>();
            if (sink) {
                // the caller serves them one by one (speculation): stay compact
                if (sink->size() < done + got) sink->resize(done + got);
                std::memcpy(sink->data() + done, er, sizeof(pe::EmitRec) * got);
                s->emit_sunk = true;
            } else {
                for (uint32_t i = 0; i < got; i++) widen_rec(er[i], &out[done + i]);
            }
        } else {
            std::memcpy(out + done, s->h_place_out.as<pe_ranked_node>(), sizeof(pe_ranked_node) * got);
        }
        if (commit)
            for (uint32_t i = 0; i < st[0]; i++)
                plan_of(s).emplace_back(g.name, (uint32_t)(chain && sink ? (*sink)[done + i].row : out[done + i].row));
        if (hprof) {
            const double t3 = now_us();
            h_launch += t1 - t0;
            h_sync += t2 - t1;
            h_copy += t3 - t2;
        }
        if (chain && (st[1] & kChainErrFlag))
            return s->fail(PE_EINTERNAL, "k_chain: a bounds guard tripped (evaluation stopped)");
        *placed += st[0];
        *new_offset = st[1] & ~kStalledFlag;
        if (chain && (st[1] & kStalledFlag)) {
            // a Select needs more than the chain's window of a long list (sparse
            // options): the lazy per-position loop places the rest
            done += st[0];
            if (sink) {   // full records from here on: widen the compact ones
                for (uint32_t i = 0; i < done; i++) widen_rec((*sink)[i], &out[i]);
                s->emit_sunk = false;
                sink = nullptr;
            }
            chain = false;
            A.fused = 0;
            A.fused_parts = nullptr;
            A.fused_nparts = nullptr;
            A.base = nullptr;
            A.base1 = nullptr;
            A.base_by_pos = 0;
            A.emit = nullptr;
            A.emit_out = nullptr;
            A.full_out = s->h_place_out.dev<pe_ranked_node>();
            A.done_flag = nullptr;
            spin = false;
            continue;
        }
        done += c;
        if (st[0] < c) break;
    }
    s->last_ms_pending = false;
    if (spin) {
        s->last_ms_pending = true;   // ev0 .. ev1 bracket the loop's launches
        if (hprof || A.prof) {
            HIP_TRY(s, hipEventSynchronize(s->ev1));
            float ms = 0;
            HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
            total_ms = ms;
            s->last_ms_pending = false;
        }
    }
    if (hprof)
        std::fprintf(stderr, "run_place: launch %.1f us, sync %.1f us (kernels %.1f us), copy %.1f us\n", h_launch,
                     h_sync, total_ms * 1e3, h_copy);
    s->last_ms = total_ms;   // (pending when the spin path left it to the events)
    if (A.prof) {
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        unsigned long long pr[32];
        HIP_TRY(s, hipMemcpy(pr, A.prof, sizeof(pr), hipMemcpyDeviceToHost));
        for (int ph = 0; ph < 4; ph++) {
            const unsigned long long* p = pr + 8 * ph;
            if (!p[1]) continue;
            std::fprintf(stderr, "k_chain phase %d clocks: top %llu values %llu scan %llu index %llu select-bounds %llu "
                                 "argmax %llu emit+commit %llu\n", ph, p[0], p[1], p[2], p[3], p[4], p[5], p[6]);
        }
        std::fprintf(stderr, "k_chain kernels %.3f ms\n", total_ms);
    }
    return PE_OK;
}

}  // namespace

extern "C" {

// The row of placement i of the run (record i, or its record in an evicting run).
static inline int32_t spec_row(const pe_stack::Spec& sp, uint32_t i) {
    return spec_rec_row(sp, sp.evict ? sp.place_rec[i] : i);
}

// Placements among the run's settled records: what HBM must hold after a flush.
static uint32_t spec_conf_placed(const pe_stack::Spec& sp) {
    if (!sp.evict) return std::min(sp.confirmed, sp.placed);
    uint32_t c = 0;
    for (uint32_t k = 0; k < sp.confirmed && k < sp.n_rec; k++) c += sp.rec_place[k] != PE_NONE;
    return c;
}

static bool spec_serve(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out);
static bool spec_eligible(pe_stack* s, uint32_t tgi, const pe_select_options* opts);
static int spec_flush(pe_stack* s);
static int spec_start(pe_stack* s, uint32_t tgi, pe_ranked_node* out);
static void spec_drop(pe_stack* s);
static int sys_flush(pe_stack* s);
static bool sys_serve(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out, int* rc);
static void sys_touch(pe_stack* s, uint32_t row);

uint32_t pe_abi_version(void) { return PE_ABI_VERSION; }

const char* pe_comm_library(void) { return rccl().ok ? rccl().path.c_str() : ""; }

pe_stack* pe_stack_create(const pe_config* cfg) {
    if (!cfg) { g_error = "null config"; return nullptr; }
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev == 0) {
        g_error = "no HIP device available: the placement engine runs only on the GPU";
        return nullptr;
    }
    if (cfg->device_count > PE_MAX_DEVICES) { g_error = "device_count above PE_MAX_DEVICES"; return nullptr; }
    const int root_dev = cfg->device_count > 1 ? cfg->device_ids[0] : cfg->device;
    if (root_dev < 0 || root_dev >= ndev) { g_error = "device ordinal out of range"; return nullptr; }
    for (uint32_t k = 1; k < cfg->device_count; k++)
        if (cfg->device_ids[k] < 0 || cfg->device_ids[k] >= ndev) { g_error = "device ordinal out of range"; return nullptr; }
    auto* s = new pe_stack();
    s->cfg = *cfg;
    s->cfg.device = root_dev;
    s->cfg.device_count = 0;
    s->device = root_dev;
    if (hipSetDevice(s->device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&s->ev0) != hipSuccess || hipEventCreate(&s->ev1) != hipSuccess ||
        hipEventCreate(&s->ev2) != hipSuccess) {
        g_error = "HIP stream/event creation failed";
        delete s;
        return nullptr;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, s->device) == hipSuccess && cus > 0)
        s->n_cu = cus;
    s->sweep_per_cu = pe_sweep_blocks_per_cu(false);
    s->sweep_per_cu_aux = pe_sweep_blocks_per_cu(true);
    s->log10 = pe::gm::log_go(10.0);
    if (const char* e = std::getenv("PE_SWEEP_MIN")) s->sweep_min = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("PE_LOOP_SWEEP_MIN")) s->loop_sweep_min = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char* e = std::getenv("PE_RESULTS_VIA_COPY")) s->results_via_copy = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_WINDOW_LAZY")) s->use_base = std::atoi(e) == 0;
    if (const char* e = std::getenv("PE_SPECULATE")) s->spec_on = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_SPIN_WAIT")) s->spin_wait = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_COUNTS_DEFER")) s->counts_defer_ok = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_API_PROF")) s->api_prof = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_KERNEL_SPLIT")) s->kernel_split = std::atoi(e) != 0;
    if (const char* e = std::getenv("PE_TEST_FALLBACK_EVERY")) s->test_fallback_every = std::strtoull(e, nullptr, 10);
    if (cfg->device_count > 1) {
        // replicas on the other devices, and the communicators of the group
        bool same = true;
        for (uint32_t k = 1; k < cfg->device_count; k++) {
            pe_config kc = s->cfg;
            kc.device = cfg->device_ids[k];
            pe_stack* kid = pe_stack_create(&kc);
            if (!kid) { pe_stack_destroy(s); return nullptr; }
            kid->test_fallback_every = 0;
            s->kids.push_back(kid);
            same = same && cfg->device_ids[k] == root_dev;
        }
        s->loopback = same;
        if (!same) {
            std::vector<int> devs(cfg->device_ids, cfg->device_ids + cfg->device_count);
            s->group_comms.assign(devs.size(), nullptr);
            const ncclResult_t r = rc_CommInitAll(s->group_comms.data(), (int)devs.size(), devs.data());
            if (r != ncclSuccess) {
                g_error = std::string("ncclCommInitAll: ") + rc_GetErrorString(r);
                s->group_comms.clear();
                pe_stack_destroy(s);
                return nullptr;
            }
        }
        (void)hipSetDevice(s->device);
    }
    return s;
}

void pe_stack_destroy(pe_stack* s) {
    if (!s) return;
    for (pe_stack* k : s->kids) pe_stack_destroy(k);
    for (ncclComm_t c : s->group_comms)
        if (c) (void)rc_CommDestroy(c);
    if (s->api_prof)
        for (auto& kv : s->api_acc)
            std::fprintf(stderr, "api %-28s %10.1f us total %8llu calls %8.2f us/call\n", kv.first.c_str(),
                         kv.second.first, (unsigned long long)kv.second.second,
                         kv.second.first / std::max<uint64_t>(kv.second.second, 1));
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->comm) (void)rc_CommDestroy(s->comm);
    if (s->h_xbuf) (void)hipHostFree(s->h_xbuf);
    if (s->ev_x0) (void)hipEventDestroy(s->ev_x0);
    if (s->ev_x1) (void)hipEventDestroy(s->ev_x1);
    for (hipEvent_t ev : s->ev_xs)
        if (ev) (void)hipEventDestroy(ev);
    retire_tgs(s);
    for (hipEvent_t ev : s->ev_split)
        if (ev) (void)hipEventDestroy(ev);
    if (s->ev0) (void)hipEventDestroy(s->ev0);
    if (s->ev1) (void)hipEventDestroy(s->ev1);
    if (s->ev2) (void)hipEventDestroy(s->ev2);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    delete s;
}

const char* pe_last_error(const pe_stack* s) { return s ? s->err.c_str() : g_error.c_str(); }

double pe_last_kernel_ms(const pe_stack* s) {
    if (!s) return 0.0;
    if (s->last_ms_pending) {
        pe_stack* m = const_cast<pe_stack*>(s);
        float ms = 0;
        if (hipEventSynchronize(m->ev1) == hipSuccess && hipEventElapsedTime(&ms, m->ev0, m->ev1) == hipSuccess)
            m->last_ms = ms;
        m->last_ms_pending = false;
    }
    return s->last_ms;
}

int pe_set_kernel_split(pe_stack* s, int on) {
    if (!s) return PE_EINVAL;
    s->kernel_split = on != 0;
    s->split_valid = false;
    return PE_OK;
}

int pe_last_kernel_split(const pe_stack* s, double* ms4) {
    if (!s || !ms4) return PE_EINVAL;
    if (!s->split_valid) return PE_ESTATE;
    pe_stack* m = const_cast<pe_stack*>(s);
    if (hipEventSynchronize(m->ev_split[4]) != hipSuccess) return m->fail(PE_EHIP, "kernel split events");
    for (int k = 0; k < 4; k++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, m->ev_split[k], m->ev_split[k + 1]) != hipSuccess)
            return m->fail(PE_EHIP, "kernel split events");
        ms4[k] = ms;
    }
    return PE_OK;
}

uint32_t pe_last_sweep_bytes(const pe_stack* s) { return s ? s->last_sweep_bytes : 0u; }

int pe_check_constraint(const char* op, const char* l, int ls, const char* r, int rs) {
    pe::ConstraintEvaluator ev;
    pe::Target lt, rt;
    lt.nil = ls == 0; lt.found = ls == 1; lt.value = (ls == 1 && l) ? l : "";
    rt.nil = rs == 0; rt.found = rs == 1; rt.value = (rs == 1 && r) ? r : "";
    return ev.check(op ? op : "", lt, rt) ? 1 : 0;
}

// ---- EvalEligibility export (context.go:190-356) ---------------------------

static void elig_reset(pe_stack* s) {
    s->elig_log.clear();
    s->ex_job.clear();
    s->ex_job_seen.clear();
    s->ex_job_unseen = 0;
    s->ex_tg.clear();
    s->ex_tg_escaped.clear();
    s->ex_dirty.clear();
    s->cls_str.clear();
}

static void elig_size(pe_stack* s) {
    if (s->ex_job.size() != s->ncls) {
        s->ex_job.assign(s->ncls, -1);
        s->ex_job_seen.assign(s->ncls, 0);
        s->ex_job_unseen = s->ncls;
    }
}

static pe_stack::ExTg& elig_tg(pe_stack* s, uint32_t name) {
    pe_stack::ExTg& e = s->ex_tg[name];
    if (e.st.size() != s->ncls) {
        e.st.assign(s->ncls, -1);
        e.seen.assign(s->ncls, 0);
        e.unseen = s->ncls;
    }
    return e;
}

static void elig_set(pe_stack* s, uint32_t map, std::vector<int8_t>& st, uint32_t c, int8_t v) {
    if (st[c] == v) return;
    st[c] = v;
    s->ex_dirty.emplace_back(map, c);
}

// One row the chain pulled for a Select of task group g, in visit order
// (FeasibilityWrapper.Next, feasible.go:1061-1153): the job-level entry of its
// class is written unless the job escaped; the task group's entry is decided
// by the first visited node of the class that passes the job checks.
static void elig_visit(pe_stack* s, TgPlan& g, pe::ConstraintEvaluator& ev, uint32_t row) {
    const HostNode& nd = s->nodes[row];
    const uint32_t c = nd.cls;
    bool jr;
    if (s->job_escaped) {
        jr = g.job_ok_node.size() == s->nodes.size() ? g.job_ok_node[row] != 0 : job_feasible(s, ev, s->view(row));
    } else {
        if (s->job_memo.size() != s->ncls) s->job_memo.assign(s->ncls, -1);
        if (s->job_memo[c] == -1) s->job_memo[c] = job_feasible(s, ev, s->view(row)) ? 1 : 0;
        jr = s->job_memo[c] == 1;
        if (!s->ex_job_seen[c]) { s->ex_job_seen[c] = 1; s->ex_job_unseen--; }
        elig_set(s, PE_NONE, s->ex_job, c, jr ? 1 : 0);
    }
    if (g.escaped) return;
    pe_stack::ExTg& e = elig_tg(s, g.name);
    if (e.seen[c]) return;
    if (!jr) {
        // a class-exact job failure: no node of the class reaches the tg checks
        if (!s->job_escaped) { e.seen[c] = 1; e.unseen--; }
        return;
    }
    e.seen[c] = 1;
    e.unseen--;
    if (g.sig_tg.size() != s->sig_rep.size()) {
        g.sig_tg.clear();
        classify_classes(s, g, ev);
    }
    elig_set(s, g.name, e.st, c, g.sig_tg[nd.sig] ? 1 : 0);
}

static void elig_walk(pe_stack* s, uint32_t tgi, const std::vector<uint32_t>& list, uint32_t begin, uint32_t len,
                      pe::ConstraintEvaluator& ev) {
    const size_t m = list.size();
    if (tgi >= s->tgs.size() || !m) return;
    TgPlan& g = *s->tgs[tgi];
    elig_size(s);
    pe_stack::ExTg* e = g.escaped ? nullptr : &elig_tg(s, g.name);
    len = (uint32_t)std::min<uint64_t>(len, m);
    for (uint32_t k = 0; k < len; k++) {
        if ((!e || e->unseen == 0) && (s->job_escaped || s->ex_job_unseen == 0)) {   // nothing left to learn
            g.elig_complete = true;
            break;
        }
        elig_visit(s, g, ev, list[(begin + k) % m]);
    }
}

static void elig_resolve(pe_stack* s) {
    if (s->elig_log.empty()) return;
    pe::ConstraintEvaluator ev;
    for (const auto& sp : s->elig_log) elig_walk(s, sp.tgi, s->visit, sp.begin, sp.len, ev);
    s->elig_log.clear();
}

// A Select of task group tgi pulled `len` rows of the SetNodes list from
// position `begin` (its StaticIterator window). Consecutive windows of one
// group merge, so the speculative count loop logs one span.
static void elig_log_span(pe_stack* s, uint32_t tgi, uint32_t begin, uint32_t len) {
    if (s->elig_mute || !len || (tgi < s->tgs.size() && s->tgs[tgi]->elig_complete)) return;
    const uint32_t m = (uint32_t)s->visit.size();
    if (!m) return;
    begin %= m;
    if (!s->elig_log.empty()) {
        pe_stack::EligSpan& last = s->elig_log.back();
        if (last.tgi == tgi && last.len < m && (uint32_t)(((uint64_t)last.begin + last.len) % m) == begin) {
            last.len = (uint32_t)std::min<uint64_t>((uint64_t)last.len + len, m);
            return;
        }
        if (last.tgi == tgi && last.len >= m) return;   // the whole list already
    }
    s->elig_log.push_back(pe_stack::EligSpan{tgi, begin, std::min(len, m)});
}

// A Select over another list (the preferred nodes): resolve in order now.
static void elig_visit_list(pe_stack* s, uint32_t tgi, const std::vector<uint32_t>& list, uint32_t len) {
    if (s->elig_mute || !len || (tgi < s->tgs.size() && s->tgs[tgi]->elig_complete)) return;
    elig_resolve(s);
    pe::ConstraintEvaluator ev;
    elig_walk(s, tgi, list, 0, len, ev);
}

static int set_state_one(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes, const pe_alloc_table* allocs) {
    if (s) plan_settle(s);   // the deferred entries index the current list
    if (s) s->jf.clear();   // node attributes change: the job checkers run again
    if (!s || !strs || !nodes) return PE_EINVAL;
    spec_drop(s);
    s->counts_pending = false;   // a new snapshot: its arrays are rebuilt (the job's counts by the next SetJob)
    s->node_update.clear();   // a new evaluation context: no plan stops
    s->stop_count.clear();
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    s->strs.clear();
    s->sid.clear();
    s->add_strings(strs);
    s->have_state = false;
    plan_of(s).clear();
    s->tg_memo.clear();
    s->job_memo.clear();
    s->ref_tg_memo.clear();
    s->ref_job_memo.clear();
    s->spread_info_done.clear();
    s->sum_spread_weights = 0;
    elig_reset(s);
    int rc = build_state(s, nodes, allocs);
    if (rc) return rc;
    s->have_state = true;
    s->have_job = false;
    s->have_job_version = false;
    retire_tgs(s);
    s->visit.clear();
    s->offset = 0;
    return PE_OK;
}

static int update_allocs_one(pe_stack* s, const pe_strtab* strs, const pe_alloc_table* allocs, const uint32_t* index) {
    if (s) plan_settle(s);   // the deferred entries index the current list
    if (!s || !allocs) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    spec_drop(s);
    {
        const int frc = flush_counts(s);   // before any array is resized
        if (frc) return frc;
    }
    s->node_update.clear();   // a new evaluation context: no plan stops
    s->stop_count.clear();
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    s->add_strings(strs);
    const size_t before = s->allocs.size();
    int rc = append_allocs(s, allocs, index);
    if (rc) {
        s->allocs.resize(before);
        s->have_state = false;   // partially applied: the caller must reload
        return rc;
    }
    rc = build_alloc_state(s);
    if (rc) { s->have_state = false; return rc; }
    // a new evaluation context, as after pe_set_state
    std::fill(s->h_preempted.begin(), s->h_preempted.end(), 0);
    s->offer_row = -1;
    plan_of(s).clear();
    s->tg_memo.clear();
    s->job_memo.clear();
    s->ref_tg_memo.clear();
    s->ref_job_memo.clear();
    s->spread_info_done.clear();
    s->sum_spread_weights = 0;
    elig_reset(s);
    s->have_job = false;
    s->have_job_version = false;
    retire_tgs(s);
    s->visit.clear();
    s->offset = 0;
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    return PE_OK;
}

static int update_nodes_one(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes, const uint32_t* index) {
    if (s) plan_settle(s);   // the deferred entries index the current list
    if (s) s->jf.clear();   // node attributes change: the job checkers run again
    if (!s || !nodes) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    spec_drop(s);
    {
        const int frc = flush_counts(s);   // before any array is resized
        if (frc) return frc;
    }
    s->node_update.clear();   // a new evaluation context: no plan stops
    s->stop_count.clear();
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    s->add_strings(strs);
    const uint32_t n_old = (uint32_t)s->nodes.size();
    std::vector<uint32_t> target(nodes->n);
    uint32_t n_new = n_old;
    for (uint32_t i = 0; i < nodes->n; i++) {
        const uint32_t r = index ? index[i] : PE_NONE;
        if (r != PE_NONE && r >= n_old) return s->fail(PE_EINVAL, "node index out of range");
        target[i] = r == PE_NONE ? n_new++ : r;
    }
    const bool packable_before = s->dev_packable, cores_before = s->has_cores;
    int rc = apply_nodes(s, nodes, target, n_new);
    if (rc) {   // the mirror may be half updated: a reload is required
        s->have_state = false;
        return rc;
    }
    std::vector<uint32_t> rows;
    for (uint32_t r : target)
        if (r < n_old) rows.push_back(r);
    plan_of(s).clear();
    s->tg_memo.clear();
    s->job_memo.clear();
    s->ref_tg_memo.clear();
    s->ref_job_memo.clear();
    s->spread_info_done.clear();
    s->sum_spread_weights = 0;
    elig_reset(s);
    s->have_job = false;
    s->have_job_version = false;
    retire_tgs(s);
    s->visit.clear();
    s->offset = 0;
    rc = refresh_node_rows(s, std::move(rows), n_old, packable_before, cores_before);
    if (rc) s->have_state = false;
    return rc;
}

// may_defer: a handle without child devices leaves the state copy to the next
// SetJob's k_counts launch (one launch less per evaluation)
static int reset_plan_one(pe_stack* s, bool may_defer) {
    if (!s) return PE_EINVAL;
    s->plan_defer.active = false;   // the plan is emptied below
    ApiScope prof_(s, "reset_plan");
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    spec_drop(s);
    s->node_update.clear();   // a new evaluation context: no plan stops
    s->stop_count.clear();
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    const size_t n = s->nodes.size();
    ApiScope prof_launch_(s, "reset_plan.launch");
    s->reset_pending = true;
    if (!may_defer) {
        const int frc = flush_reset(s);
        if (frc) return frc;
    }
    std::fill(s->h_preempted.begin(), s->h_preempted.end(), 0);
    if (s->has_cores) {   // reserved cores back to the snapshot's
        HIP_TRY(s, hipMemcpyAsync(s->d_core_used.p, s->d_core_base.p, sizeof(uint64_t) * 4 * n, hipMemcpyDeviceToDevice,
                                  s->stream));
        s->h_core_used = s->h_core_base;
    }
    s->node_update.clear();
    s->stop_count.assign(s->allocs.size(), 0);
    s->offer_row = -1;   // stream-ordered: later launches and uploads see the reset state
    plan_of(s).clear();
    s->tg_memo.clear();
    s->job_memo.clear();
    s->ref_tg_memo.clear();
    s->ref_job_memo.clear();
    s->spread_info_done.clear();
    s->sum_spread_weights = 0;
    elig_reset(s);
    s->have_job = false;
    s->have_job_version = false;
    retire_tgs(s);
    s->offset = 0;
    return PE_OK;
}

static int set_job_one(pe_stack* s, const pe_strtab* strs, const pe_job* j) {
    if (!s || !j) return PE_EINVAL;
    ApiScope prof_(s, "set_job");
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    s->add_strings(strs);
    const bool generic = s->cfg.stack_kind == PE_STACK_GENERIC;
    if (generic && s->have_job_version && s->job_version == j->version) return PE_OK;   // stack.go:94-96
    elig_resolve(s);   // the windows so far belong to the current job's task groups
    {
        const int frc = spec_flush(s);   // a different job: the plan so far goes to HBM first
        if (frc) return frc;
    }
    sys_deactivate(s);   // per-row outcomes of the previous job's groups
    s->sys.singles = 0;
    s->sys.singles_tgi = PE_NONE;
    s->have_job_version = true;
    s->job_version = j->version;
    s->job_id = j->id;
    s->job_ns = j->ns;
    s->job_priority = j->priority;
    s->job_constraints.clear();
    s->job_escaped = false;
    for (uint32_t i = 0; i < j->constraint_count; i++) {
        s->job_constraints.push_back(parse_constraint(s, j->constraints[j->constraint_off + i]));
        s->job_escaped = s->job_escaped || s->job_constraints.back().escapes;
    }
    {   // the per-row job checker outcomes hold for the same constraints (and
        // node table: SetState / UpdateNodes clear them)
        std::string key = job_checker_key(s);
        if (key != s->jf_key) {
            s->jf.clear();
            s->jf_key = std::move(key);
            s->jf_texts.clear();
            for (auto& c : s->job_constraints) s->jf_texts.push_back(c.text);
        }
    }
    bool job_distinct_hosts = false;
    for (auto& c : s->job_constraints) {
        if (c.op == "distinct_hosts") job_distinct_hosts = true;
    }
    s->job_affinities.clear();
    for (uint32_t i = 0; i < j->affinity_count; i++)
        s->job_affinities.push_back(ParsedAffinity{parse_constraint(s, *reinterpret_cast<const pe_constraint*>(&j->affinities[j->affinity_off + i])),
                                                   j->affinities[j->affinity_off + i].weight});
    auto conv_spreads = [&](uint32_t off, uint32_t cnt) {
        std::vector<SpreadSpec> out;
        for (uint32_t i = 0; i < cnt; i++) {
            const pe_spread& sp = j->spreads[off + i];
            SpreadSpec ss{sp.attribute, sp.weight, {}};
            for (uint32_t k = 0; k < sp.target_count; k++)
                ss.targets.emplace_back(j->spread_targets[sp.target_off + k].value, j->spread_targets[sp.target_off + k].percent);
            out.push_back(ss);
        }
        return out;
    };
    s->job_spreads = conv_spreads(j->spread_off, j->spread_count);
    std::string job_unsupported;

    retire_tgs(s);
    for (uint32_t gi = 0; gi < j->tg_count; gi++) {
        const pe_task_group& t = j->task_groups[gi];
        auto g = new_tg(s);
        g->name = t.name;
        g->count = t.count;
        g->unsupported = job_unsupported;
        tg_ask(j, t, &g->ask);
        g->ask.distinct_job = job_distinct_hosts ? 1 : 0;
        g->ask.distinct_tg = 0;
        for (uint32_t k = 0; k < t.constraint_count; k++) {
            g->constraints.push_back(parse_constraint(s, j->constraints[t.constraint_off + k]));
            if (g->constraints.back().op == "distinct_hosts") g->ask.distinct_tg = 1;
            if (g->constraints.back().op == "distinct_property") g->distinct_props.push_back(g->constraints.back());
        }
        for (uint32_t k = 0; k < t.task_count; k++) {
            const pe_task& x = j->tasks[t.task_off + k];
            g->drivers.insert(x.driver);
            for (uint32_t c = 0; c < x.constraint_count; c++) g->constraints.push_back(parse_constraint(s, j->constraints[x.constraint_off + c]));
            for (uint32_t d = 0; d < x.device_count; d++)
                g->dev_reqs.push_back(parse_dev_request(s, j, j->devices[x.device_off + d]));
            if (x.cores > 0 && x.lifecycle != PE_LC_MAIN) g->unsupported = "reserved cores on a lifecycle hook task";
            if (x.has_network && x.net_reserved_ports > 0) {
                if (!g->trports.empty()) g->unsupported = "static ports in several task networks";
                else if (!j->rport_value) g->unsupported = "task static ports without their values (pe_task.rport_off)";
                else
                    for (int32_t q = 0; q < x.net_reserved_ports; q++) {
                        const int32_t v = j->rport_value[x.rport_off + (uint32_t)q];
                        // a static port in the dynamic range shrinks the task's dynamic picks: not modelled
                        if (v >= 20000 && v <= 32000) g->unsupported = "task static ports in the dynamic port range";
                        g->trports.emplace_back(v, j->rport_label ? j->rport_label[x.rport_off + (uint32_t)q] : PE_NONE);
                    }
            }
        }
        if (g->ask.cores > 0)   // the per-node ask is Σ main tasks + SharesPerCore x cores (no max over hooks)
            for (uint32_t k = 0; k < t.task_count; k++) {
                const uint32_t lc = j->tasks[t.task_off + k].lifecycle;
                if (lc == PE_LC_PRESTART || lc == PE_LC_POSTSTOP) g->unsupported = "reserved cores beside prestart / poststop tasks";
            }
        for (auto& c : g->constraints) g->escaped = g->escaped || c.escapes;
        for (uint32_t k = 0; k < t.volume_count; k++)
            g->volumes.emplace_back(j->volume_source[t.volume_off + k], j->volume_read_only[t.volume_off + k] != 0);
        if (t.has_csi_volumes) g->unsupported = "CSI volumes";
        g->has_network = t.has_network != 0;
        g->net_mode = t.has_network ? t.net_mode : s->lookup("host");
        g->net_host = t.net_host_network;
        g->net_ports = t.net_dyn_ports + t.net_reserved_ports;
        for (uint32_t k = 0; t.has_network && j->rport_value && k < t.rport_count; k++)
            g->rports.emplace_back(j->rport_value[t.rport_off + k], j->rport_label ? j->rport_label[t.rport_off + k] : PE_NONE);
        if (t.has_network && (int64_t)g->rports.size() != (int64_t)t.net_reserved_ports)
            g->unsupported = "static port asks without their values (pe_task_group.rport_*)";
        if (!g->rports.empty() && !g->trports.empty())
            g->unsupported = "static ports in the task group network and a task network";
        // affinities: job, task group, tasks (rank.go:671-686)
        g->affinities = s->job_affinities;
        for (uint32_t k = 0; k < t.affinity_count; k++)
            g->affinities.push_back(ParsedAffinity{parse_constraint(s, *reinterpret_cast<const pe_constraint*>(&j->affinities[t.affinity_off + k])),
                                                   j->affinities[t.affinity_off + k].weight});
        for (uint32_t k = 0; k < t.task_count; k++) {
            const pe_task& x = j->tasks[t.task_off + k];
            for (uint32_t a = 0; a < x.affinity_count; a++)
                g->affinities.push_back(ParsedAffinity{parse_constraint(s, *reinterpret_cast<const pe_constraint*>(&j->affinities[x.affinity_off + a])),
                                                       j->affinities[x.affinity_off + a].weight});
        }
        if (!g->dev_reqs.empty()) {
            if (g->dev_reqs.size() > (size_t)pe::kMaxDevReq) g->unsupported = "more than 4 device requests";
            else if (!s->dev_packable) g->unsupported = "nodes with more than 4 device groups or 255 instances";
            g->ask.n_dev = (int32_t)g->dev_reqs.size();
            g->ask.dev_aff = 0;
            g->ask.dev_tw = 0.0;
            for (size_t q = 0; q < g->dev_reqs.size() && q < (size_t)pe::kMaxDevReq; q++) {
                const DevReqSpec& r = g->dev_reqs[q];
                if (r.count > 255) g->unsupported = "device request count above 255";
                g->ask.dev_cnt[q] = (int32_t)std::min<uint32_t>(r.count, 255);
                if (!r.affinities.empty()) {
                    g->ask.dev_aff |= 1u << q;
                    for (auto& a : r.affinities) g->ask.dev_tw += std::fabs((double)a.weight);
                }
            }
            if (g->unsupported.empty()) {
                int rc = build_dev_classes(s, *g);
                if (rc) return rc;
            }
        }
        g->spreads = conv_spreads(t.spread_off, t.spread_count);
        if (!generic && (!g->spreads.empty() || !s->job_spreads.empty())) g->spreads.clear();
        if (!generic) g->affinities.clear();
        s->tgs.push_back(std::move(g));
    }
    {   // static ports of one group only: a sibling's placements would hold them too
        int with_static = 0;
        for (auto& g : s->tgs) with_static += has_static(*g) ? 1 : 0;
        if (with_static > 1)
            for (auto& g : s->tgs)
                if (has_static(*g)) g->unsupported = "static port asks in several task groups of a job";
    }
    for (auto& g : s->tgs) {   // AssignNetwork's address: the network CIDR's one address on every node
        if (g->trports.empty()) continue;
        for (uint32_t r = 0; r < (uint32_t)s->nodes.size() && g->unsupported.empty(); r++) {
            const HostNode& nd = s->nodes[r];
            bool known = nd.n_device_nets == 0 || nd.yield_known;
            if (nd.n_device_nets > 1)
                for (const HostNet& nw : s->node_dnets[r]) known = known && nw.yield != PE_NONE;
            if (!known) g->unsupported = "task static ports on a network whose CIDR is not one known address";
        }
    }
    if (!generic) s->job_spreads.clear();
    // multi-device nodes (build_md) model one task network of one group: the
    // replay of the plan puts only that group's placements on the devices
    if (s->n_multi_net > 0 || s->net_other_dev > 0) {
        int with_net = 0;
        for (auto& g : s->tgs) with_net += g->ask.has_task_net > 0;
        for (auto& g : s->tgs) {
            if (g->ask.has_task_net > 1) g->unsupported = "several task networks in a group, with multi-device nodes";
            else if (g->ask.has_task_net && with_net > 1)
                g->unsupported = "task networks in several groups of a job, with multi-device nodes";
        }
    }
    s->have_job = true;
    for (auto& g : s->tgs) s->ex_tg_escaped[g->name] = g->escaped;   // EvalEligibility.SetJob (context.go:221-234)
    ApiScope prof_own_(s, "set_job.own+collisions");
    {
        auto it = s->job_keys.find(std::make_pair(s->job_id, s->job_ns));
        s->job_key = it == s->job_keys.end() ? PE_NONE : it->second;
    }
    s->offer_row = -1;
    return build_job_counts(s, true);
}

int pe_set_nodes(pe_stack* s, const uint32_t* rows, uint32_t n, uint32_t* limit_out) {
    if (!s) return PE_EINVAL;
    plan_settle(s);   // the deferred entries index the current list
    sys_view_take(s);   // the caller's served system Selects first
    if (n == 1 && rows && s->sys.active && s->visit.size() == 1 && rows[0] < s->nodes.size()) {
        // SystemScheduler's per-node SetNodes while the per-row cache answers:
        // the task group's tables do not depend on the list (every class's
        // memo verdict is uniform), so only the list changes
        if (!s->elig_log.empty()) elig_resolve(s);
        s->gen++;
        s->visit[0] = rows[0];
        s->d_visit_is_visit = false;
        s->rank_of_valid = false;
        s->visit_unique = true;
        s->offset = 0;
        s->limit = 2;
        if (limit_out) *limit_out = 2;
        return PE_OK;
    }
    ApiScope prof_(s, "set_nodes");
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    if (!rows && n) return s->fail(PE_EINVAL, "null rows");
    if (n > 1 && n == s->visit.size() && std::memcmp(rows, s->visit.data(), sizeof(uint32_t) * n) == 0) {
        // the same list again (a SystemScheduler evaluation over the same
        // ready nodes, a replayed evaluation): already validated, and its
        // device copy and visit ranks stay resident; the iterator restarts
        const int frc = spec_flush(s);
        if (frc) return frc;
        s->gen++;
        elig_resolve(s);
        s->offset = 0;
        uint32_t lim = 2;
        if (s->cfg.stack_kind == PE_STACK_GENERIC && !s->cfg.batch) {
            const uint32_t log_limit = (uint32_t)std::ceil(std::log2((double)n));
            if (log_limit > lim) lim = log_limit;
        }
        s->limit = lim;
        if (limit_out) *limit_out = lim;
        invalidate_tables(s);
        return PE_OK;
    }
    // validate before touching any state: a rejected list leaves the previous one
    // in place. The same pass finds repeated rows (the chain and sweep loops and
    // the system placement need a list without them).
    if (s->seen_stamp.size() != s->nodes.size()) {
        s->seen_stamp.assign(s->nodes.size(), 0);
        s->seen_gen = 0;
    }
    if (++s->seen_gen == 0) {
        std::fill(s->seen_stamp.begin(), s->seen_stamp.end(), 0);
        s->seen_gen = 1;
    }
    bool unique = true;
    {
        const uint32_t nn = (uint32_t)s->nodes.size(), gen = s->seen_gen;
        uint32_t* stamp = s->seen_stamp.data();
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t r = rows[i];
            if (r >= nn) return s->fail(PE_EINVAL, "row out of range");
            unique = unique && stamp[r] != gen;
            stamp[r] = gen;
        }
    }
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    s->gen++;
    elig_resolve(s);   // logged spans index the old list
    s->visit.assign(rows, rows + n);
    s->d_visit_is_visit = false;
    s->offset = 0;
    uint32_t lim = 2;
    if (s->cfg.stack_kind == PE_STACK_GENERIC && !s->cfg.batch && n > 0) {
        uint32_t log_limit = (uint32_t)std::ceil(std::log2((double)n));
        if (log_limit > lim) lim = log_limit;
    }
    s->limit = lim;
    if (limit_out) *limit_out = lim;
    invalidate_tables(s);
    // the visit position of every row (rank_of) is built when a sweep needs it
    s->visit_unique = unique;
    s->rank_of_valid = false;
    return PE_OK;
}

static bool tg_full_scan(pe_stack* s, TgPlan& g) {
    return !g.affinities.empty() || !g.spreads.empty() || !s->job_spreads.empty();
}

// Device offers of a Select result, one byte per request (~0u: none).
static uint32_t pack_offers(const pe_ranked_node* out) {
    if (out->row < 0 || out->n_device_offers == 0) return 0xFFFFFFFFu;
    uint32_t w = 0;
    for (uint32_t q = 0; q < out->n_device_offers && q < 4; q++) w |= (out->device_offer_group[q] & 255u) << (8 * q);
    return w;
}

static int select_impl(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out,
                       uint32_t rec = 0);

// AllocMetric maps of one plain Select (structs.go:9903-9937): the rows the
// chain pulled (visit order from the Select's cursor), FeasibilityWrapper
// reasons from the host-side checkers with the reference's memo transitions
// (feasible.go:1061-1153), every later reason from k_trace on the device.
// NodeScoreMeta (structs.go:10030-10035) and the top-K ScoreHeap
// (lib/kheap/score_heap.go) with Go's container/heap up/down, so ties keep the
// reference's order.
// The named scores of one option (at most 7 scorers: binpack, devices,
// job-anti-affinity, node-reschedule-penalty, node-affinity,
// allocation-spread, preemption) as PE_SCORER_* ids, so the heap moves PODs.
const char* const kScorerNames[7] = {"binpack", "devices", "job-anti-affinity", "node-reschedule-penalty",
                                     "node-affinity", "allocation-spread", "preemption"};
struct ScoreList {
    uint8_t name[8];
    double val[8];
    uint32_t n = 0;
    void emplace_back(uint32_t k, double v) {
        name[n] = (uint8_t)k;
        val[n] = v;
        n++;
    }
    uint32_t size() const { return n; }
};

struct ScoreMeta {
    uint32_t row;
    ScoreList scores;   // sorted by name on output
    double norm;
};

struct ScoreHeap {
    static constexpr uint32_t cap = 5;   // MaxRetainedNodeScores (structs.go:178)
    ScoreMeta items[cap];
    uint32_t len = 0;
    bool less(uint32_t i, uint32_t j) const { return items[i].norm < items[j].norm; }
    void up(uint32_t j) {
        while (j > 0) {
            const uint32_t i = (j - 1) / 2;
            if (!less(j, i)) break;
            std::swap(items[i], items[j]);
            j = i;
        }
    }
    bool down(uint32_t i0, uint32_t n) {
        uint32_t i = i0;
        for (;;) {
            const uint32_t j1 = 2 * i + 1;
            if (j1 >= n) break;
            uint32_t j = j1;
            if (j1 + 1 < n && less(j1 + 1, j1)) j = j1 + 1;
            if (!less(j, i)) break;
            std::swap(items[i], items[j]);
            i = j;
        }
        return i > i0;
    }
    // whether push(m) changes the heap: a full heap ignores an item not above
    // its minimum (and the closing up(len-1) of heap.Push is then a no-op, the
    // heap property holding)
    bool enters(double norm) const { return len < cap || norm > items[0].norm; }
    void push(const ScoreMeta& m) {   // heap.Push → ScoreHeap.Push (+ heap.Fix) then up(len-1)
        if (len < cap) {
            items[len++] = m;
        } else if (m.norm > items[0].norm) {
            items[0] = m;
            if (!down(0, len)) up(0);
        }
        up(len - 1);
    }
    // GetItemsReverse: heap.Pop until empty, into out[0 .. len) (descending)
    uint32_t reverse_items(ScoreMeta* out) {
        const uint32_t total = len;
        uint32_t i = total;
        while (len > 0) {
            const uint32_t n = len - 1;
            std::swap(items[0], items[n]);
            down(0, n);
            out[--i] = items[n];
            len--;
        }
        return total;
    }
};

// One AllocMetric map (key -> count) as it fills: a Select's maps hold a
// handful of keys, so a short vector searched in place
struct MetricCounts {
    static constexpr uint32_t kInline = 6;   // most maps: a few keys, no allocation
    std::pair<uint32_t, uint32_t> in[kInline];
    uint32_t n = 0;
    std::vector<std::pair<uint32_t, uint32_t>> more;
    void add(uint32_t k) {
        for (uint32_t i = 0; i < n; i++)
            if (in[i].first == k) {
                in[i].second++;
                return;
            }
        for (auto& e : more)
            if (e.first == k) {
                e.second++;
                return;
            }
        if (n < kInline) in[n++] = {k, 1u};
        else more.emplace_back(k, 1u);
    }
    void append(uint32_t kind, std::vector<pe_metric_count>& out) const {
        for (uint32_t i = 0; i < n; i++) out.push_back(pe_metric_count{kind, in[i].first, in[i].second});
        for (auto& e : more) out.push_back(pe_metric_count{kind, e.first, e.second});
    }
};

// The maps of one Select as they fill (FilterNode / ExhaustedNode, ScoreNode);
// keys are caller string ids (node classes) or engine strings (reasons).
struct MetricAcc {
    MetricCounts cf, kf, ce, de;
    ScoreHeap heap;
    void reset() {
        for (MetricCounts* c : {&cf, &kf, &ce, &de}) {
            c->n = 0;
            c->more.clear();
        }
        heap.len = 0;
    }
    // the row's node class key: the flat per-row copy (jf_ready) when current
    static uint32_t mclass(const pe_stack* s, uint32_t row) {
        if (row < s->jf_mclass.size() && s->jf.size() == s->nodes.size()) return s->jf_mclass[row];
        const uint32_t nc = s->nodes[row].node_class;
        return (nc != PE_NONE && !s->S(nc).empty()) ? nc : PE_NONE;
    }
    void filter(pe_stack* s, uint32_t row, uint32_t why) {
        const uint32_t nc = mclass(s, row);
        if (nc != PE_NONE) cf.add(nc);
        if (why != PE_NONE) kf.add(why);
    }
    void filter(pe_stack* s, uint32_t row, const std::string& why) { filter(s, row, s->mkey(why)); }
    void exhaust(pe_stack* s, uint32_t row, uint32_t dim) {
        const uint32_t nc = mclass(s, row);
        if (nc != PE_NONE) ce.add(nc);
        if (dim != PE_NONE) de.add(dim);
    }
    void exhaust(pe_stack* s, uint32_t row, const std::string& dim) { exhaust(s, row, s->mkey(dim)); }
    void exhaust(pe_stack* s, uint32_t row, const char* dim) { exhaust(s, row, s->mkey_p(dim)); }
};

// FeasibilityWrapper half of one Select's maps: the window's rows in visit
// order against the reference memo shadow (feasible.go:1061-1153); rows that
// pass go to `rows` for k_trace. `log` (or null) receives the memo changes.
static void metrics_walk(pe_stack* s, TgPlan& g, const std::vector<uint32_t>& order, uint32_t start,
                         uint32_t evaluated, MetricAcc& acc, std::vector<uint32_t>& rows,
                         std::vector<MemoDelta>* log = nullptr, std::vector<uint8_t>* pass = nullptr) {
    const size_t m = order.size();
    if (s->ref_job_memo.size() != s->ncls) s->ref_job_memo.assign(s->ncls, -1);
    auto& rt = s->ref_tg_memo[g.name];
    if (rt.size() != s->ncls) rt.assign(s->ncls, -1);
    pe::ConstraintEvaluator ev;
    static const char* kIneligible = "computed class ineligible";
    const uint32_t ineligible = s->mkey_p(kIneligible);
    auto set_job = [&](uint32_t c, int8_t v) {
        if (log) log->push_back({false, c, v});
        s->ref_job_memo[c] = v;
    };
    auto set_tg = [&](uint32_t c, int8_t v) {
        if (log) log->push_back({true, c, v});
        rt[c] = v;
    };
    jf_ready(s);
    // the loop's tables in locals (the row pushes would make the compiler
    // reload every member); the vectors are not resized inside it
    const uint32_t* cls_of = s->jf_cls.data();
    const char** jfp = s->jf.data();
    int8_t* jm = s->ref_job_memo.data();
    int8_t* tm = rt.data();
    const bool job_esc = s->job_escaped, job_cons = !s->job_constraints.empty(), tg_esc = g.escaped;
    auto job_why = [&](uint32_t row) -> const char* {   // job_fail_cached, its hit inlined
        const char* w = jfp[row];
        if (!w) return job_fail_cached(s, ev, row);   // fills jfp[row]
        return w == kJfPass ? nullptr : w;
    };
    uint32_t p = m ? start % (uint32_t)m : 0;
    for (uint32_t k = 0; k < evaluated && m; k++, p = p + 1 == m ? 0 : p + 1) {
        const uint32_t row = order[p];
        const uint32_t c = cls_of[row];
        const char* why = nullptr;
        // the node's attribute views only when a checker runs (a known class
        // decides the common case from the memo alone)
        if (job_esc) {
            why = job_why(row);
        } else if (jm[c] == 0) {
            why = kIneligible;
        } else if (jm[c] == -1 || job_cons) {
            why = job_why(row);
            if (why) set_job(c, 0);
            else if (jm[c] == -1) set_job(c, 1);
        }
        if (!why) {
            if (tg_esc) {
                why = tg_fail(s, ev, g, s->view(row));
            } else if (tm[c] == 0) {
                why = kIneligible;
            } else if (tm[c] == -1) {
                why = tg_fail(s, ev, g, s->view(row));
                set_tg(c, why ? 0 : 1);
            }
        }
        if (why) {
            acc.filter(s, row, why == kIneligible ? ineligible : s->mkey_p(why));
        } else {
            rows.push_back(row);
            if (pass) (*pass)[p] = 1;
        }
    }
}

// One k_trace outcome of a plain Select (o: its 6 score values).
static int metrics_outcome(pe_stack* s, TgPlan& g, const pe::Ask& a, uint32_t row, uint32_t code, const double* o,
                           MetricAcc& acc, std::map<int, std::vector<uint32_t>>& counts) {
    const bool has_aff = !g.affinities.empty();
    const bool generic = s->cfg.stack_kind == PE_STACK_GENERIC;
    switch (code & 255u) {
        case pe::kTrOption: {   // ScoreNode calls in chain order, then the NormScore push
            if (!acc.heap.enters(o[5])) break;
            ScoreMeta sm;
            sm.row = row;
            sm.scores.emplace_back(PE_SCORER_BINPACK, o[0]);
            if (a.dev_tw != 0.0) sm.scores.emplace_back(PE_SCORER_DEVICES, o[1]);
            if (generic) {   // the SystemStack ranks with BinPack alone (stack.go:277-281)
                if (a.anti_aff) sm.scores.emplace_back(PE_SCORER_JOB_ANTI_AFFINITY, o[2]);
                sm.scores.emplace_back(PE_SCORER_RESCHEDULE_PENALTY, (code & pe::kTrPenalty) ? -1.0 : 0.0);
                if (!has_aff) sm.scores.emplace_back(PE_SCORER_NODE_AFFINITY, 0.0);
                else if (o[3] != 0.0) sm.scores.emplace_back(PE_SCORER_NODE_AFFINITY, o[3]);
                if (o[4] != 0.0) sm.scores.emplace_back(PE_SCORER_ALLOCATION_SPREAD, o[4]);
            }
            sm.norm = o[5];
            acc.heap.push(sm);
            break;
        }
        case pe::kTrDistinctHosts: acc.filter(s, row, s->mkey_p("distinct_hosts")); break;
        case pe::kTrDistinctProp: {   // propertyset.go:213-244
            const int p = (int)(code >> 8);
            PsetDev& ps = *g.psets[p];
            uint32_t vid;
            Target tv = resolve(s, ps.target, s->view(row), &vid);
            if (!tv.found || tv.nil) {
                acc.filter(s, row, "missing property \"" + ps.target_text + "\"");
                break;
            }
            if (vid == PE_NONE) vid = s->lookup(tv.value);
            auto it = ps.value_index.find(vid);
            uint64_t used = 0;
            if (it != ps.value_index.end()) {
                auto& cnt = counts[p];
                if (cnt.empty()) {
                    cnt.resize(std::max<size_t>(ps.value_str.size(), 1));
                    HIP_TRY(s, hipMemcpyAsync(cnt.data(), ps.counts.p, cnt.size() * 4, hipMemcpyDeviceToHost,
                                              s->stream));
                    HIP_TRY(s, hipStreamSynchronize(s->stream));
                }
                used = cnt[it->second];
            }
            acc.filter(s, row, "distinct_property: " + ps.target_text + "=" + tv.value + " used by " +
                                   std::to_string(used) + " allocs");
            break;
        }
        case pe::kTrNoAddr: acc.exhaust(s, row, "network: no addresses available"); break;
        case pe::kTrStaticPort: {
            std::string why;
            if (!static_port_reason(s, g, row, &why)) why = static_port_collision(s, g);
            acc.exhaust(s, row, "network: " + why);
            break;
        }
        case pe::kTrTaskStatic: {
            std::string why;
            const uint32_t q = (code >> 8) & 255u;
            if ((code & pe::kMdCoded) && q < g.trports.size()) {   // a multi-device node: the host's record
                const auto& rp = g.trports[q];
                why = (code & pe::kMdInvalidPort)
                          ? "invalid port " + std::to_string(rp.first) + " (out of range)"
                          : "reserved port collision " + (rp.second == PE_NONE ? std::string() : s->S(rp.second)) +
                                "=" + std::to_string(rp.first);
            } else if (!task_port_reason(s, g, row, &why)) {
                why = static_port_collision(s, g);
            }
            acc.exhaust(s, row, "network: " + why);
            break;
        }
        case pe::kTrDynPorts: acc.exhaust(s, row, "network: dynamic port selection failed"); break;
        case pe::kTrNoNetworks: acc.exhaust(s, row, "network: no networks available"); break;
        case pe::kTrBandwidth: acc.exhaust(s, row, "network: bandwidth exceeded"); break;
        case pe::kTrTaskDyn: acc.exhaust(s, row, "network: dynamic port selection failed"); break;
        case pe::kTrDevNone: acc.exhaust(s, row, "devices: no devices available"); break;
        case pe::kTrDevZero: acc.exhaust(s, row, "devices: invalid request of zero devices"); break;
        case pe::kTrDevNoMatch: acc.exhaust(s, row, "devices: no devices match request"); break;
        case pe::kTrCpu: acc.exhaust(s, row, "cpu"); break;
        case pe::kTrCores: acc.exhaust(s, row, "cores"); break;
        case pe::kTrMemory: acc.exhaust(s, row, "memory"); break;
        case pe::kTrDisk: acc.exhaust(s, row, "disk"); break;
        case pe::kTrMismatch: return s->fail(PE_EHIP, "k_trace: device verdict differs from the host walk");
        default: return s->fail(PE_EHIP, "k_trace: unknown outcome code");
    }
    return PE_OK;
}

// One Select's maps in binary form (pe_last_metrics_bin), appended.
static void metrics_bin_into(MetricAcc& acc, std::vector<pe_metric_count>& counts,
                             std::vector<pe_metric_score>& scores) {
    acc.cf.append(PE_METRIC_CLASS_FILTERED, counts);
    acc.kf.append(PE_METRIC_CONSTRAINT_FILTERED, counts);
    acc.ce.append(PE_METRIC_CLASS_EXHAUSTED, counts);
    acc.de.append(PE_METRIC_DIMENSION_EXHAUSTED, counts);
    ScoreMeta items[ScoreHeap::cap];
    const uint32_t ni = acc.heap.reverse_items(items);
    for (uint32_t q = 0; q < ni; q++) {   // PopulateScoreMetaData: GetItemsReverse
        const ScoreMeta& it = items[q];
        pe_metric_score m;
        std::memset(&m, 0, sizeof(m));
        m.row = (int32_t)it.row;
        m.n_scores = it.scores.n;
        m.norm = it.norm;
        for (uint32_t k = 0; k < it.scores.n && k < PE_MAX_SCORES; k++) {
            m.scorer[k] = it.scores.name[k];
            m.score[k] = it.scores.val[k];
        }
        scores.push_back(m);
    }
}

static const std::string& metric_string(const pe_stack* s, uint32_t key) {
    static const std::string none;
    if (key & PE_METRIC_ENGINE_KEY) {
        const uint32_t i = key & ~PE_METRIC_ENGINE_KEY;
        return i < s->mstrs.size() ? s->mstrs[i] : none;
    }
    return s->S(key);
}

// The map key a row's k_trace outcome records in a single-node Select:
// *kind 0 an option (no key), PE_METRIC_CONSTRAINT_FILTERED (distinct_hosts)
// or PE_METRIC_DIMENSION_EXHAUSTED; false for outcomes whose reason needs the
// host's port mirrors or property counts (not on the system cache path).
static bool trace_key(pe_stack* s, uint32_t code, uint32_t* kind, uint32_t* key) {
    *kind = PE_METRIC_DIMENSION_EXHAUSTED;
    const char* t = nullptr;
    switch (code & 255u) {
        case pe::kTrOption: *kind = 0; *key = PE_NONE; return true;
        case pe::kTrDistinctHosts: *kind = PE_METRIC_CONSTRAINT_FILTERED; t = "distinct_hosts"; break;
        case pe::kTrNoAddr: t = "network: no addresses available"; break;
        case pe::kTrDynPorts: case pe::kTrTaskDyn: t = "network: dynamic port selection failed"; break;
        case pe::kTrNoNetworks: t = "network: no networks available"; break;
        case pe::kTrBandwidth: t = "network: bandwidth exceeded"; break;
        case pe::kTrDevNone: t = "devices: no devices available"; break;
        case pe::kTrDevZero: t = "devices: invalid request of zero devices"; break;
        case pe::kTrDevNoMatch: t = "devices: no devices match request"; break;
        case pe::kTrCpu: t = "cpu"; break;
        case pe::kTrCores: t = "cores"; break;
        case pe::kTrMemory: t = "memory"; break;
        case pe::kTrDisk: t = "disk"; break;
        default: return false;
    }
    *key = s->mkey_p(t);
    return true;
}

// pe_last_metrics' text of binary maps: "KIND\tKEY\tCOUNT" lines per map,
// keys sorted (Go's map keys in order), then ScoreMetaData lines
// "SM\trank\tnode id\tnorm\tname=value,..." with the names sorted and the
// values in the shortest round-trip decimal (the same doubles when parsed).
static void metrics_text_into(const pe_stack* s, const pe_metric_count* c, size_t nc, const pe_metric_score* sc,
                              size_t ns, std::string& out) {
    char num[64];
    static const char* kinds[5] = {"", "CF", "KF", "CE", "DE"};
    for (uint32_t kind = PE_METRIC_CLASS_FILTERED; kind <= PE_METRIC_DIMENSION_EXHAUSTED; kind++) {
        std::vector<std::pair<const std::string*, uint32_t>> kv;
        for (size_t i = 0; i < nc; i++)
            if (c[i].kind == kind) kv.emplace_back(&metric_string(s, c[i].key), c[i].count);
        std::sort(kv.begin(), kv.end(), [](const auto& x, const auto& y) { return *x.first < *y.first; });
        for (auto& e : kv) {
            out += kinds[kind];
            out += '\t';
            out += *e.first;
            out += '\t';
            const auto r = std::to_chars(num, num + sizeof num, e.second);
            out.append(num, r.ptr);
            out += '\n';
        }
    }
    auto put_num = [&](double x) {
        const auto r = std::to_chars(num, num + sizeof num, x);
        out.append(num, r.ptr);
    };
    for (size_t i = 0; i < ns; i++) {
        const pe_metric_score& it = sc[i];
        uint32_t order[PE_MAX_SCORES];
        const uint32_t n = std::min<uint32_t>(it.n_scores, PE_MAX_SCORES);
        for (uint32_t k = 0; k < n; k++) order[k] = k;
        std::sort(order, order + n, [&](uint32_t x, uint32_t y) {   // NodeScoreMeta.Scores is a map
            return std::strcmp(kScorerNames[it.scorer[x]], kScorerNames[it.scorer[y]]) < 0;
        });
        out += "SM\t";
        out += (char)('0' + i);
        out += '\t';
        out += s->S(s->nodes[(uint32_t)it.row].id);
        out += '\t';
        put_num(it.norm);
        out += '\t';
        for (uint32_t k = 0; k < n; k++) {
            if (k) out += ',';
            out += kScorerNames[it.scorer[order[k]]];
            out += '=';
            put_num(it.score[order[k]]);
        }
        out += '\n';
    }
}

// The last Select's maps (pe_last_metrics_bin) from an accumulator.
static void metrics_set_last(pe_stack* s, MetricAcc& acc) {
    s->m_counts.clear();
    s->m_scores.clear();
    metrics_bin_into(acc, s->m_counts, s->m_scores);
    s->metrics_text_ok = false;
    s->metrics_valid = true;
}

// The maps of a single-node system Select on `row` served from the view
// (code: the cache's outcome, 0 option / 1 filtered / 2 exhausted;
// failed_before: the row's memo class had already failed).
static void metrics_set_last_sys(pe_stack* s, uint32_t row, uint32_t code, bool failed_before) {
    const pe_stack::SysSpec& y = s->sys;
    s->m_counts.clear();
    s->m_scores.clear();
    const uint32_t nc = y.mnode_class[row];
    if (code == 0) {
        pe_metric_score m;
        std::memset(&m, 0, sizeof(m));
        m.row = (int32_t)row;
        m.n_scores = 1;
        m.norm = y.tscore[6 * (size_t)row + 5];
        m.scorer[0] = PE_SCORER_BINPACK;
        m.score[0] = y.mscore[row];
        s->m_scores.push_back(m);
    } else if (code == 1) {
        if (nc != PE_NONE) s->m_counts.push_back(pe_metric_count{PE_METRIC_CLASS_FILTERED, nc, 1});
        const uint32_t key = failed_before ? s->sysview.mkey_ineligible : y.mkey[row];
        s->m_counts.push_back(pe_metric_count{PE_METRIC_CONSTRAINT_FILTERED, key, 1});
    } else {
        if (nc != PE_NONE) s->m_counts.push_back(pe_metric_count{PE_METRIC_CLASS_EXHAUSTED, nc, 1});
        s->m_counts.push_back(pe_metric_count{PE_METRIC_DIMENSION_EXHAUSTED, y.mkey[row], 1});
    }
    s->metrics_text_ok = false;
    s->metrics_valid = true;
}

// Whole-list windows of one replay (spec_metrics_replay): once a walk over
// the whole list changes no memo entry, every node's verdict no longer depends
// on the visit order, so later whole-list walks take its filter counts and its
// passing positions (rotated to their start) instead of walking again.
struct WalkCache {
    bool valid = false;
    MetricCounts cf, kf;
    std::vector<uint8_t> pass;   // per visit position
    // the passing rows in position order and their positions, built at the
    // first reuse, and whether d_wc_list holds them
    std::vector<uint32_t> list, lpos;
    bool built = false, on_dev = false;
};

// PE_METRICS_PROF: compute_metrics' phases (walk, trace launches + syncs,
// eviction trace, outcomes) summed over a replay
static double g_cm_prof[4];

static int compute_metrics(pe_stack* s, TgPlan& g, const std::vector<uint32_t>& order, uint32_t start,
                           uint32_t evaluated, const pe_select_options* opts, bool evict = false,
                           std::vector<MemoDelta>* log = nullptr, WalkCache* wc = nullptr) {
    static const bool prof = std::getenv("PE_METRICS_PROF") != nullptr;
    double tp = prof ? now_us() : 0.0;
    auto lap = [&](int k) {
        if (!prof) return;
        const double t = now_us();
        g_cm_prof[k] += t - tp;
        tp = t;
    };
    s->metrics_valid = false;
    MetricAcc acc;
    std::vector<uint32_t> rows;
    const size_t m = order.size();
    const bool whole = wc && m && evaluated == m;
    bool rows_on_dev = false;
    if (whole && wc->valid) {
        acc.cf = wc->cf;
        acc.kf = wc->kf;
        if (!wc->built) {
            wc->list.clear();
            wc->lpos.clear();
            for (uint32_t p = 0; p < m; p++)
                if (wc->pass[p]) {
                    wc->list.push_back(order[p]);
                    wc->lpos.push_back(p);
                }
            wc->built = true;
            wc->on_dev = false;
        }
        // the window's passing rows: the list rotated to its start, on the
        // host and (two device copies of the list uploaded once) on the device
        const size_t P = wc->list.size();
        size_t s0 = (size_t)(std::lower_bound(wc->lpos.begin(), wc->lpos.end(), (uint32_t)(start % m)) -
                             wc->lpos.begin());
        if (s0 == P) s0 = 0;
        rows.reserve(P);
        rows.insert(rows.end(), wc->list.begin() + s0, wc->list.end());
        rows.insert(rows.end(), wc->list.begin(), wc->list.begin() + s0);
        if (P) {
            if (!wc->on_dev) {
                HIP_TRY(s, upload_s(s, s->d_wc_list, wc->list));
                wc->on_dev = true;
            }
            HIP_TRY(s, s->d_trace_rows.ensure(P * sizeof(uint32_t)));
            const uint32_t* l = s->d_wc_list.as<uint32_t>();
            uint32_t* r = s->d_trace_rows.as<uint32_t>();
            HIP_TRY(s, hipMemcpyAsync(r, l + s0, (P - s0) * sizeof(uint32_t), hipMemcpyDeviceToDevice, s->stream));
            if (s0)
                HIP_TRY(s, hipMemcpyAsync(r + (P - s0), l, s0 * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                                          s->stream));
            rows_on_dev = true;
        }
    } else {
        const size_t l0 = log ? log->size() : 0;
        if (whole) wc->pass.assign(m, 0);
        metrics_walk(s, g, order, start, evaluated, acc, rows, log, whole ? &wc->pass : nullptr);
        const bool changed = log && log->size() != l0;
        if (wc && (changed || !whole)) wc->valid = wc->valid && !changed;
        if (whole && !changed && log) {
            wc->valid = true;
            wc->built = false;
            wc->cf = acc.cf;
            wc->kf = acc.kf;
        }
    }
    lap(0);
    const pe_metric_score* dtop = nullptr;   // plain Selects: k_trace_top's items
    pe_metric_score dtop_items[5];
    uint32_t dtop_n = 0;
    if (!rows.empty()) {
        if (!rows_on_dev) HIP_TRY(s, upload_s(s, s->d_trace_rows, rows));
        // the codes, then (plain Selects) k_trace_top's items and count
        HIP_TRY(s, s->d_trace_out.ensure(((rows.size() * 4 + 15) & ~size_t(15)) + 5 * sizeof(pe_metric_score) + 8));
        HIP_TRY(s, s->d_trace_scores.ensure(rows.size() * 6 * sizeof(double)));
        pe::NodeSoA soa = soa_of(s);
        pe::TgTables t = tables_of(g);
        pe::Ask a = ask_for(s, g);
        const uint32_t* pbits = nullptr;
        if (opts && opts->penalty_count > 0) {
            std::vector<uint32_t> bits((s->nodes.size() + 31) / 32, 0);
            for (uint32_t i = 0; i < opts->penalty_count; i++) {
                const uint32_t r = opts->penalty_rows[i];
                if (r < s->nodes.size()) bits[r >> 5] |= 1u << (r & 31);
            }
            HIP_TRY(s, upload_s(s, s->d_penalty, bits));
            pbits = s->d_penalty.as<uint32_t>();
        }
        const double* stab = nullptr;
        if (t.n_spread > 0) {
            HIP_TRY(s, s->d_spread_tab.ensure(spread_tab_bytes(g)));
            HIP_TRY(s, pe_launch_spread_table(&t, s->d_spread_tab.as<double>(), s->stream));
            stab = s->d_spread_tab.as<double>();
        }
        HIP_TRY_STATE(s, pe_launch_trace(&soa, &t, &a, s->d_trace_rows.as<uint32_t>(), (uint32_t)rows.size(),
                                   s->d_trace_out.as<uint32_t>(), pbits, s->log10, stab,
                                   s->d_trace_scores.as<double>(), s->stream));
        // the outcome codes and (plain Selects) the top-5 ScoreMetaData from
        // k_trace_top come back; the score values stay on the device. (Host
        // vectors: the staged copy leaves them in the CPU's caches, and the
        // outcome loop read a pinned buffer the DMA wrote about twice as
        // slowly, same-box A/B.)
        const size_t n = rows.size();
        const size_t top_bytes = 5 * sizeof(pe_metric_score);
        static thread_local std::vector<uint32_t> codes_v, ecodes_v;
        static thread_local std::vector<double> named_v;
        // plain Selects: the codes, then the top-5 and its count, in one buffer
        // and one download
        const size_t top_at = (n * 4 + 15) & ~size_t(15);
        codes_v.resize(evict ? n : (top_at + top_bytes + 8) / 4);
        if (!evict) {
            const std::vector<uint32_t> ends{(uint32_t)n, 0u};
            const uint32_t* d_ends = reinterpret_cast<const uint32_t*>(stage_only(s, ends));
            if (!d_ends) {
                HIP_TRY(s, upload_s(s, s->d_cm_ends, ends));
                d_ends = s->d_cm_ends.as<uint32_t>();
            }
            pe::TraceSrc src{};
            src.rows = s->d_trace_rows.as<uint32_t>();
            src.rec_end = d_ends;
            src.rsrc = d_ends + 1;
            src.n_rec = 1;
            uint8_t* d_top = s->d_trace_out.as<uint8_t>() + top_at;
            const uint32_t flags = (a.dev_tw != 0.0 ? 1u : 0u) | (a.anti_aff ? 2u : 0u) |
                                   (!g.affinities.empty() ? 4u : 0u) |
                                   (s->cfg.stack_kind == PE_STACK_GENERIC ? 8u : 0u);
            HIP_TRY_STATE(s, pe_launch_trace_top(s->d_trace_out.as<uint32_t>(), s->d_trace_scores.as<double>(), &src,
                                                 flags, reinterpret_cast<pe_metric_score*>(d_top),
                                                 d_top + top_bytes, s->stream, (uint32_t)n));
            HIP_TRY(s, hipMemcpyAsync(codes_v.data(), s->d_trace_out.p, top_at + top_bytes + 1,
                                      hipMemcpyDeviceToHost, s->stream));
        } else {
            HIP_TRY(s, hipMemcpyAsync(codes_v.data(), s->d_trace_out.p, n * 4, hipMemcpyDeviceToHost, s->stream));
        }
        const uint8_t* top_buf = reinterpret_cast<const uint8_t*>(codes_v.data()) + top_at;
        // Select with Preempt: BinPack with evict per row (rank.go:480-503) and
        // the ScoreNode values of the options, preemption score included
        if (evict) {
            ecodes_v.resize(n);
            named_v.resize(n * 7);
        }
        uint32_t* ecodes = ecodes_v.data();
        double* named = named_v.data();
        if (evict) {
            if (prof) {
                HIP_TRY(s, hipStreamSynchronize(s->stream));
                lap(1);
            }
            pe::PreemptArgs P = preempt_args(s, g);
            P.penalty_bits = pbits;
            P.spread_tab = stab;
            if (!stab && !g.psets.empty()) {
                HIP_TRY(s, s->d_spread_tab.ensure(spread_tab_bytes(g)));
                HIP_TRY(s, pe_launch_spread_table(&P.tg, s->d_spread_tab.as<double>(), s->stream));
                P.spread_tab = s->d_spread_tab.as<double>();
            }
            HIP_TRY(s, s->d_ev_tcodes.ensure(rows.size() * sizeof(uint32_t)));
            HIP_TRY(s, s->d_ev_named.ensure(rows.size() * 7 * sizeof(double)));
            for (;;) {   // a row wider than the launch: the trace again, wider
                HIP_TRY_STATE(s, pe_launch_evict_trace(&P, s->d_trace_rows.as<uint32_t>(), (uint32_t)rows.size(),
                                                       s->d_ev_tcodes.as<uint32_t>(), s->d_ev_named.as<double>(),
                                                       s->stream));
                HIP_TRY(s, hipMemcpyAsync(ecodes, s->d_ev_tcodes.p, n * 4, hipMemcpyDeviceToHost,
                                          s->stream));
                HIP_TRY(s, hipMemcpyAsync(named, s->d_ev_named.p, n * 7 * sizeof(double), hipMemcpyDeviceToHost,
                                          s->stream));
                HIP_TRY(s, hipStreamSynchronize(s->stream));
                bool wider = false;
                for (size_t i = 0; i < n; i++) wider = wider || (((ecodes[i] >> 24) & pe::kEvictWider) != 0u);
                if (!wider) break;
                P.mask_words = wider_words(P.mask_words);
                if (!P.mask_words)
                    return s->fail(PE_EUNSUPPORTED, "preemption: a node's proposed allocs exceed the widest eviction "
                                                    "width");
            }
        }
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        lap(evict ? 2 : 1);
        const uint32_t* codes = codes_v.data();
        if (!evict) {
            std::memcpy(dtop_items, top_buf, top_bytes);
            dtop = dtop_items;
            dtop_n = std::min<uint32_t>(top_buf[top_bytes], 5u);
        }
        const bool has_aff = !g.affinities.empty();
        const bool generic = s->cfg.stack_kind == PE_STACK_GENERIC;
        std::map<int, std::vector<uint32_t>> counts;   // distinct_property use counts, read on demand
        for (size_t i = 0; i < rows.size(); i++) {
            const uint32_t row = rows[i], code = codes[i];
            const uint32_t base = code & 255u;
            if (evict && base != pe::kTrDistinctHosts && base != pe::kTrDistinctProp) {
                const uint32_t ec = ecodes[i], st = ec & 255u;
                if (ec >> 24) return s->fail(PE_EUNSUPPORTED, "preemption: a node outside the device path (several "
                                                              "network devices, reserved cores)");
                if (st == 0) {   // option (kOption), preempting or not
                    const double* o = &named[i * 7];
                    if (!acc.heap.enters(o[6])) continue;
                    const uint32_t fl = (ec >> 16) & 255u;
                    ScoreMeta sm;
                    sm.row = row;
                    sm.scores.emplace_back(PE_SCORER_BINPACK, o[0]);
                    if (a.dev_tw != 0.0) sm.scores.emplace_back(PE_SCORER_DEVICES, o[1]);
                    if (generic) {
                        if (a.anti_aff) sm.scores.emplace_back(PE_SCORER_JOB_ANTI_AFFINITY, o[2]);
                        sm.scores.emplace_back(PE_SCORER_RESCHEDULE_PENALTY, (fl & 1u) ? -1.0 : 0.0);
                        if (!has_aff) sm.scores.emplace_back(PE_SCORER_NODE_AFFINITY, 0.0);
                        else if (o[3] != 0.0) sm.scores.emplace_back(PE_SCORER_NODE_AFFINITY, o[3]);
                        if (o[4] != 0.0) sm.scores.emplace_back(PE_SCORER_ALLOCATION_SPREAD, o[4]);
                        if (fl & 2u) sm.scores.emplace_back(PE_SCORER_PREEMPTION, o[5]);
                    }
                    sm.norm = o[6];
                    acc.heap.push(sm);
                } else if (st == 2) {   // kExhausted: no preemption frees enough (ExhaustedNode(dim))
                    const uint32_t d = (ec >> 8) & 255u;
                    acc.exhaust(s, row, d == pe::kTrCpu ? "cpu" : (d == pe::kTrMemory ? "memory" : "disk"));   // literals
                } else if (st != 3) {   // kSkipped (device preemption failed) records nothing
                    return s->fail(PE_EHIP, "k_evict_trace: outcome differs from the host walk");
                }
                continue;
            }
            if (base == pe::kTrOption) continue;   // the options' ScoreMetaData came from k_trace_top
            const int rc = metrics_outcome(s, g, a, row, code, nullptr, acc, counts);
            if (rc) return rc;
        }
    }
    metrics_set_last(s, acc);
    if (dtop) s->m_scores.assign(dtop, dtop + dtop_n);
    lap(3);
    return PE_OK;
}

static void spec_metrics_reset(pe_stack::Spec& sp) {
    sp.mcounts.clear();
    sp.mscores.clear();
    sp.mcounts_off.assign(1, 0u);
    sp.mscores_off.assign(1, 0u);
}

static void spec_metrics_push(pe_stack::Spec& sp, MetricAcc& acc) {
    metrics_bin_into(acc, sp.mcounts, sp.mscores);
    sp.mcounts_off.push_back((uint32_t)sp.mcounts.size());
    sp.mscores_off.push_back((uint32_t)sp.mscores.size());
}

// AllocMetric maps of every record of a speculative run (§25): record k's
// Select saw the run's starting state plus the placements of records < k, so
// its window is walked on the host in record order (the FeasibilityWrapper
// half, with the reference memo), and every row that passes is traced in one
// k_trace launch against the checkpoint of the starting state, with dk = the
// earlier records' placements on the row and each record's spread boosts from
// its own use counts (k_spread_tables). Whole-list windows (full passes) whose
// walk no longer changes the memo are one cached list, rotated per record on
// the device (TraceSrc). Runs without evictions and distinct_property sets only
// (their state differs by placements alone; spec_metrics_batched).
static int spec_metrics(pe_stack* s, TgPlan& g, uint32_t off0) {
    static const bool prof = std::getenv("PE_METRICS_PROF") != nullptr;
    const double t0 = prof ? now_us() : 0.0;
    pe_stack::Spec& sp = s->spec;
    const auto& order = s->visit;
    auto& rt = s->ref_tg_memo[g.name];
    if (s->ref_job_memo.size() != s->ncls) s->ref_job_memo.assign(s->ncls, -1);
    if (rt.size() != s->ncls) rt.assign(s->ncls, -1);
    sp.memo_job0 = s->ref_job_memo;
    sp.memo_tg0 = rt;
    sp.memo_log.clear();
    sp.memo_off.assign(1, 0u);
    // one accumulator per record, kept across runs (no page faults per run)
    static thread_local std::vector<MetricAcc> acc;
    if (acc.size() < sp.n_rec) acc.resize(sp.n_rec);
    for (uint32_t k = 0; k < sp.n_rec; k++) acc[k].reset();
    // record k's rows: walked on the host into xrows (rsrc[k] = their offset),
    // or, once a whole-list walk no longer changes the memo, the cached walk's
    // passing rows `list` rotated to the record's start (kTraceRot | index)
    std::vector<uint32_t> xrows, rec_end(sp.n_rec), rsrc(sp.n_rec), list, lpos;
    xrows.reserve(16 * (size_t)sp.n_rec);
    bool list_live = false, list_done = false;   // one cached list per batch
    uint32_t off = off0, n_entries = 0;
    uint64_t walked = 0;
    const size_t m = order.size();
    WalkCache wc;
    for (uint32_t k = 0; k < sp.n_rec; k++) {
        const uint32_t ev = sp.compact ? sp.crecs[k].nodes_evaluated : sp.recs[k].nodes_evaluated;
        walked += ev;
        const bool whole = m && ev == m;
        if (whole && wc.valid && list_live) {
            acc[k].cf = wc.cf;
            acc[k].kf = wc.kf;
            const uint32_t st = (uint32_t)(off % m);
            size_t s0 = (size_t)(std::lower_bound(lpos.begin(), lpos.end(), st) - lpos.begin());
            if (s0 == lpos.size()) s0 = 0;
            rsrc[k] = pe::kTraceRot | (uint32_t)s0;
            n_entries += (uint32_t)list.size();
        } else {
            const size_t x0 = xrows.size(), l0 = sp.memo_log.size();
            if (whole) wc.pass.assign(m, 0);
            metrics_walk(s, g, order, off, ev, acc[k], xrows, &sp.memo_log, whole ? &wc.pass : nullptr);
            wc.valid = whole && sp.memo_log.size() == l0;
            list_live = false;
            if (wc.valid && !list_done) {
                wc.cf = acc[k].cf;
                wc.kf = acc[k].kf;
                for (uint32_t p = 0; p < m; p++)
                    if (wc.pass[p]) {
                        list.push_back(order[p]);
                        lpos.push_back(p);
                    }
                list_done = list_live = true;
            }
            rsrc[k] = (uint32_t)x0;
            n_entries += (uint32_t)(xrows.size() - x0);
        }
        if (xrows.size() >= (size_t)pe::kTraceRot) return s->fail(PE_EINTERNAL, "spec_metrics: trace rows overflow");
        sp.memo_off.push_back((uint32_t)sp.memo_log.size());
        rec_end[k] = n_entries;
        off = sp.compact ? sp.crecs[k].new_offset : sp.recs[k].new_offset;
    }
    auto row_of = [&](uint32_t k, uint32_t j) -> uint32_t {   // trace_row on the host
        const uint32_t src = rsrc[k];
        if (!(src & pe::kTraceRot)) return xrows[src + j];
        size_t p = (size_t)(src - pe::kTraceRot) + j;
        if (p >= list.size()) p -= list.size();
        return list[p];
    };
    const double t1 = prof ? now_us() : 0.0;
    // one upload (walked rows, records' ends and sources, the cached list, the
    // placements) and one download (every record's ScoreMetaData from
    // k_trace_top, its count, the outcome codes) through buffers kept across
    // runs; the score values stay on the device
    const size_t n_rows = n_entries;
    const size_t top_bytes = 5 * sizeof(pe_metric_score) * (size_t)sp.n_rec;
    // per record: its entries that are not options, and the first kOther of
    // them (entry, code) as k_trace_top lists them
    constexpr uint32_t kOther = 128;   // = kTopOther (kernels.hip)
    const size_t other_at = (top_bytes + sp.n_rec + 15) & ~size_t(15);
    const size_t olist_at = (other_at + 4 * (size_t)sp.n_rec + 15) & ~size_t(15);
    const size_t codes_at = (olist_at + 8 * (size_t)kOther * sp.n_rec + 15) & ~size_t(15);
    // the lists pay off when the codes are many times their size (full passes)
    const bool use_list = 4 * (size_t)n_rows > 4 * 8 * (size_t)kOther * sp.n_rec;
    bool all_codes = !use_list;
    HIP_TRY(s, s->h_trace_top.ensure(codes_at + std::max<size_t>(n_rows, 1) * sizeof(uint32_t)));
    const uint32_t* olist = reinterpret_cast<const uint32_t*>(s->h_trace_top.as<uint8_t>() + olist_at);
    const uint32_t* n_other = reinterpret_cast<const uint32_t*>(s->h_trace_top.as<uint8_t>() + other_at);
    const pe_metric_score* top = s->h_trace_top.as<pe_metric_score>();
    const uint8_t* n_top = s->h_trace_top.as<uint8_t>() + top_bytes;
    const uint32_t* codes = reinterpret_cast<const uint32_t*>(s->h_trace_top.as<uint8_t>() + codes_at);
    pe::Ask a = ask_for(s, g);
    if (n_rows) {
        std::vector<uint64_t> pl;   // (row, record) of the run's placements
        for (uint32_t k = 0; k < sp.n_rec; k++) {
            const int32_t row = spec_rec_row(sp, k);
            if (row >= 0) pl.push_back((uint64_t)(uint32_t)row << 32 | k);
        }
        std::sort(pl.begin(), pl.end());
        std::vector<uint32_t> in;
        in.reserve(xrows.size() + 2 * (size_t)sp.n_rec + list.size() + 2 * pl.size() + 1);
        in.insert(in.end(), xrows.begin(), xrows.end());
        const size_t at_end = in.size();
        in.insert(in.end(), rec_end.begin(), rec_end.end());
        const size_t at_src = in.size();
        in.insert(in.end(), rsrc.begin(), rsrc.end());
        const size_t at_list = in.size();
        in.insert(in.end(), list.begin(), list.end());
        if (in.size() & 1) in.push_back(0u);
        const size_t at_pl = in.size();
        in.resize(at_pl + 2 * pl.size());
        if (!pl.empty()) std::memcpy(in.data() + at_pl, pl.data(), pl.size() * sizeof(uint64_t));
        HIP_TRY(s, upload_s(s, s->d_trace_rows, in));
        const uint32_t* d_in = s->d_trace_rows.as<uint32_t>();
        pe::TraceSrc src{};
        src.rows = d_in;
        src.rec_end = d_in + at_end;
        src.rsrc = d_in + at_src;
        src.list = d_in + at_list;
        src.pl = reinterpret_cast<const uint64_t*>(d_in + at_pl);
        src.n_rec = sp.n_rec;
        src.n_list = (uint32_t)list.size();
        src.n_pl = (uint32_t)pl.size();
        HIP_TRY(s, s->d_trace_scores.ensure(n_rows * 6 * sizeof(double)));
        HIP_TRY(s, s->d_trace_top.ensure(codes_at + n_rows * sizeof(uint32_t)));
        uint32_t* d_codes = reinterpret_cast<uint32_t*>(s->d_trace_top.as<uint8_t>() + codes_at);
        pe::NodeSoA soa = soa_of(s);   // the run's starting state: the checkpoint
        pe::TgTables t = tables_of(g);
        soa.rec = s->ck_rec.as<pe::NodeRec>();
        soa.coll_job = s->ck_coll_job.as<uint32_t>();
        t.coll_tg = s->ck_coll_tg.as<uint32_t>();
        if (t.dev_free) t.dev_free = s->ck_dev_free.as<uint32_t>();
        const double* stab = nullptr;
        if (t.n_spread > 0) {   // every record's boosts from its own use counts (k_spread_tables)
            for (int p = 0; p < t.n_psets; p++) t.pset_counts[p] = s->ck_pset[p].as<uint32_t>();
            const size_t nc = t.pset_cnt_total;
            std::vector<uint32_t> delta((size_t)sp.n_rec * nc, 0u), cur(nc, 0u);
            for (uint32_t k = 0; k < sp.n_rec; k++) {
                std::copy(cur.begin(), cur.end(), delta.begin() + (size_t)k * nc);
                const int32_t row = spec_rec_row(sp, k);
                if (row < 0) continue;
                for (int p = 0; p < t.n_psets; p++) {
                    const PsetDev& ps = *g.psets[p];
                    const uint32_t c = s->nodes[(uint32_t)row].cls;
                    if (ps.per_node ? ps.h_val_node.size() <= (size_t)row : ps.h_val_class.size() <= c)
                        return s->fail(PE_EINTERNAL, "spec_metrics: a spread set's host values are missing");
                    const uint32_t v = ps.per_node ? ps.h_val_node[(uint32_t)row] : ps.h_val_class[c];
                    if (v != pe::kMissing) cur[t.pset_cnt_off[p] + v]++;
                }
            }
            HIP_TRY(s, upload_s(s, s->d_trace_delta, delta));
            HIP_TRY(s, s->d_trace_tabs.ensure(sizeof(double) * (size_t)sp.n_rec * t.pset_tab_total));
            HIP_TRY_STATE(s, pe_launch_spread_tables(&t, sp.n_rec, s->d_trace_delta.as<uint32_t>(),
                                                     s->d_trace_tabs.as<double>(), s->stream));
            stab = s->d_trace_tabs.as<double>();
        }
        HIP_TRY_STATE(s, pe_launch_trace_batch(&soa, &t, &a, &src, (uint32_t)n_rows, d_codes, s->log10, stab,
                                               s->d_trace_scores.as<double>(), s->stream));
        const uint32_t flags = (a.dev_tw != 0.0 ? 1u : 0u) | (a.anti_aff ? 2u : 0u) |
                               (!g.affinities.empty() ? 4u : 0u) |
                               (s->cfg.stack_kind == PE_STACK_GENERIC ? 8u : 0u);
        HIP_TRY_STATE(s, pe_launch_trace_top(d_codes, s->d_trace_scores.as<double>(), &src, flags,
                                             s->d_trace_top.as<pe_metric_score>(),
                                             s->d_trace_top.as<uint8_t>() + top_bytes, s->stream, (uint32_t)n_rows,
                                             reinterpret_cast<uint32_t*>(s->d_trace_top.as<uint8_t>() + other_at),
                                             use_list ? reinterpret_cast<uint2*>(s->d_trace_top.as<uint8_t>() +
                                                                                 olist_at)
                                                      : nullptr));
        if (use_list) {
            // the ScoreMetaData, the per-record counts and lists first; every
            // code only when a record has more than its list holds
            HIP_TRY(s, hipMemcpyAsync(s->h_trace_top.p, s->d_trace_top.p, codes_at, hipMemcpyDeviceToHost,
                                      s->stream));
            HIP_TRY(s, hipStreamSynchronize(s->stream));
            for (uint32_t k = 0; k < sp.n_rec && !all_codes; k++) all_codes = n_other[k] > kOther;
            if (all_codes) {
                HIP_TRY(s, hipMemcpyAsync(s->h_trace_top.as<uint8_t>() + codes_at, d_codes,
                                          n_rows * sizeof(uint32_t), hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(s, hipStreamSynchronize(s->stream));
            }
        } else {   // short runs: everything in one copy
            HIP_TRY(s, hipMemcpyAsync(s->h_trace_top.p, s->d_trace_top.p, codes_at + n_rows * sizeof(uint32_t),
                                      hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(s, hipStreamSynchronize(s->stream));
        }
    } else {
        std::memset(s->h_trace_top.as<uint8_t>() + top_bytes, 0, codes_at - top_bytes);
    }
    const double t2 = prof ? now_us() : 0.0;
    spec_metrics_reset(sp);
    std::map<int, std::vector<uint32_t>> counts;
    size_t i = 0;
    for (uint32_t k = 0; k < sp.n_rec; k++) {
        const size_t b = i;
        if (!n_other[k]) {
            i = rec_end[k];   // options only
        } else if (use_list && n_other[k] <= kOther) {   // the listed entries (maps are counts: order is free)
            for (uint32_t q = 0; q < n_other[k]; q++) {
                const uint32_t j = olist[2 * ((size_t)k * kOther + q)], code = olist[2 * ((size_t)k * kOther + q) + 1];
                const int rc = metrics_outcome(s, g, a, row_of(k, j), code, nullptr, acc[k], counts);
                if (rc) return rc;
            }
            i = rec_end[k];
        }
        for (; i < rec_end[k]; i++) {   // the options' ScoreMetaData came from k_trace_top
            if ((codes[i] & 255u) == pe::kTrOption) continue;
            const int rc = metrics_outcome(s, g, a, row_of(k, (uint32_t)(i - b)), codes[i], nullptr, acc[k], counts);
            if (rc) return rc;
        }
        acc[k].cf.append(PE_METRIC_CLASS_FILTERED, sp.mcounts);
        acc[k].kf.append(PE_METRIC_CONSTRAINT_FILTERED, sp.mcounts);
        acc[k].ce.append(PE_METRIC_CLASS_EXHAUSTED, sp.mcounts);
        acc[k].de.append(PE_METRIC_DIMENSION_EXHAUSTED, sp.mcounts);
        sp.mscores.insert(sp.mscores.end(), top + 5 * (size_t)k, top + 5 * (size_t)k + n_top[k]);
        sp.mcounts_off.push_back((uint32_t)sp.mcounts.size());
        sp.mscores_off.push_back((uint32_t)sp.mscores.size());
    }
    sp.metrics = true;
    if (prof)
        std::fprintf(stderr, "spec_metrics: %u records, %llu walked, %zu traced rows: walk %.1f us, trace %.1f us, "
                             "maps %.1f us (%zu counts, %zu scores)\n", sp.n_rec,
                     (unsigned long long)walked, n_rows, t1 - t0, t2 - t1, now_us() - t2, sp.mcounts.size(), sp.mscores.size());
    return PE_OK;
}

static int spec_copy(pe_stack* s, TgPlan& g, bool to_ckpt);

// AllocMetric maps of the runs the batched trace cannot rebuild — evicting
// runs (a record's state depends on earlier evictions and on the plan's
// preemption counts), full passes and property sets (spread boosts and
// distinct_property counts move with every commit): the records' Selects are
// re-traced one by one (compute_metrics: the FeasibilityWrapper walk with the
// reference memo, k_trace / k_evict_trace) against the state each saw — the
// run's checkpoint plus the earlier records' evictions and commits, replayed
// in order. The device ends where the run left it (checkpoint + every record).
// Whole-list windows (full passes, the nil Selects of a saturated cluster)
// reuse one walk once the memo has settled (WalkCache).
static int spec_metrics_replay(pe_stack* s, TgPlan& g, uint32_t off0) {
    static const bool prof = std::getenv("PE_METRICS_PROF") != nullptr;
    const double t0 = prof ? now_us() : 0.0;
    pe_stack::Spec& sp = s->spec;
    auto& rt = s->ref_tg_memo[g.name];
    if (s->ref_job_memo.size() != s->ncls) s->ref_job_memo.assign(s->ncls, -1);
    if (rt.size() != s->ncls) rt.assign(s->ncls, -1);
    sp.memo_job0 = s->ref_job_memo;
    sp.memo_tg0 = rt;
    sp.memo_log.clear();
    sp.memo_off.assign(1, 0u);
    spec_metrics_reset(sp);
    int rc = spec_copy(s, g, false);   // the run's starting state (host core mirror included)
    if (rc) return rc;
    const pe::Ask a = ask_for(s, g);
    const pe::NodeSoA soa = soa_of(s);
    const pe::TgTables t = tables_of(g);
    pe_select_options pre;
    std::memset(&pre, 0, sizeof(pre));
    pre.preempt = 1;
    WalkCache wc;
    const uint32_t words = s->evict_words;
    std::vector<uint32_t> mask;
    uint32_t off = off0;
    for (uint32_t k = 0; k < sp.n_rec; k++) {
        pe_ranked_node r;
        if (sp.compact) widen_rec(sp.crecs[k], &r);
        else r = sp.recs[k];
        const bool preempt = sp.evict && (sp.rflags[k] & PE_SPEC_PREEMPT) != 0;
        rc = compute_metrics(s, g, s->visit, off, r.nodes_evaluated, preempt ? &pre : nullptr, preempt, &sp.memo_log,
                             &wc);
        if (rc) return rc;
        sp.memo_off.push_back((uint32_t)sp.memo_log.size());
        sp.mcounts.insert(sp.mcounts.end(), s->m_counts.begin(), s->m_counts.end());
        sp.mscores.insert(sp.mscores.end(), s->m_scores.begin(), s->m_scores.end());
        sp.mcounts_off.push_back((uint32_t)sp.mcounts.size());
        sp.mscores_off.push_back((uint32_t)sp.mscores.size());
        off = r.new_offset;
        const bool placement = sp.evict ? sp.rec_place[k] != PE_NONE : k < sp.placed;
        if (!placement || r.row < 0) continue;
        const uint32_t row = (uint32_t)r.row;
        if (const uint32_t np = spec_rec_npre(sp, k)) {   // Plan.AppendPreemptedAlloc, then the placement
            const uint32_t b = s->h_node_alloc_off[row];
            mask.assign(words, 0u);
            for (uint32_t j = 0; j < np; j++) {
                const uint32_t ai = spec_rec_pre(sp, k)[j];
                core_hold(s, ai, false);
                const uint32_t q = s->alloc_slot[ai] - b;
                if (q >= 32u * words) return s->fail(PE_EINTERNAL, "replayed preemption past the eviction width");
                mask[q >> 5] |= 1u << (q & 31u);
            }
            pe::PreemptArgs P = preempt_args(s, g);
            HIP_TRY(s, upload_s(s, s->d_pre_mask, mask));
            HIP_TRY_STATE(s, pe_launch_commit_preempt(&P, row, s->d_pre_mask.as<uint32_t>(),
                                                      s->d_preempted.as<uint8_t>(), s->d_pcount.as<uint32_t>(),
                                                      s->d_dev_free.as<uint32_t>(), s->stream));
        }
        HIP_TRY_STATE(s, pe_launch_commit(&soa, &t, &a, row, pack_offers(&r), s->stream));
    }
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    s->metrics_valid = false;
    sp.metrics = true;
    if (prof) {
        std::fprintf(stderr, "spec_metrics_replay: %u records: %.1f us (%zu counts, %zu scores); walk %.1f, trace "
                             "%.1f, evict trace %.1f, outcomes %.1f us\n", sp.n_rec, now_us() - t0, sp.mcounts.size(),
                     sp.mscores.size(), g_cm_prof[0], g_cm_prof[1], g_cm_prof[2], g_cm_prof[3]);
        for (double& x : g_cm_prof) x = 0.0;
    }
    return PE_OK;
}

// The reference memo after the run's first `served` records: the run's
// starting memo plus those records' walks.
static void spec_memo_rewind(pe_stack* s, uint32_t served) {
    pe_stack::Spec& sp = s->spec;
    if (!sp.metrics || sp.tgi >= s->tgs.size()) return;
    auto& rt = s->ref_tg_memo[s->tgs[sp.tgi]->name];
    s->ref_job_memo = sp.memo_job0;
    rt = sp.memo_tg0;
    const uint32_t end = sp.memo_off[std::min<uint32_t>(served, (uint32_t)sp.memo_off.size() - 1)];
    for (uint32_t j = 0; j < end; j++) {
        const MemoDelta& d = sp.memo_log[j];
        if (d.tg) rt[d.cls] = d.v;
        else s->ref_job_memo[d.cls] = d.v;
    }
}

// ---- SystemScheduler per-node Selects from a per-row cache ------------------

constexpr uint64_t kSysNaN = 0x7FF8000000000000ull;
constexpr uint64_t kSysDirty = kSysNaN | 3u;   // a row changed since the cache pass

static void sys_touch(pe_stack* s, uint32_t row) {
    if (s->sys.active && row < s->nodes.size()) s->h_sys_cache.as<uint64_t>()[row] = kSysDirty;
}

// The queued Plan.AppendAllocs of served system Selects, into HBM at once.
static int sys_flush(pe_stack* s) {
    ApiScope prof_(s, "sys_flush");
    pe_stack::SysSpec& y = s->sys;
    if (y.pending.empty()) return PE_OK;
    if (y.tgi >= s->tgs.size()) { y.pending.clear(); return s->fail(PE_ESTATE, "queued system commits lost their task group"); }
    HIP_TRY(s, hipSetDevice(s->device));
    TgPlan& g = *s->tgs[y.tgi];
    HIP_TRY(s, upload_s(s, s->d_commit_rows, y.pending));
    pe::NodeSoA soa = soa_of(s);
    pe::TgTables t = tables_of(g);
    pe::Ask a = ask_for(s, g);
    HIP_TRY_STATE(s, pe_launch_commit_rows(&soa, &t, &a, s->d_commit_rows.as<uint32_t>(), (uint32_t)y.pending.size(),
                                     s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    y.pending.clear();
    return PE_OK;
}

// Whether one k_system pass can stand in for this group's single-node Selects:
// outcomes must be per row (no distinct_property value counts), the memo
// verdict of every class independent of the visit order (uniform classes or
// an escaped group), and the result record the cache holds complete (no
// device offers, reserved cores or static ports to return).
static bool sys_cacheable(pe_stack* s, TgPlan& g) {
    return g.unsupported.empty() && g.psets.empty() && g.dev_reqs.empty() && g.ask.cores == 0 && !has_static(g) &&
           (g.escaped || g.nonuniform.empty()) && s->visit_unique;
}

// The served system-Select view's per-row AllocMetric entries (nomad_pe.h,
// pe_system_view.mkey ...) from the cache pass's k_trace outcomes: the
// FeasibilityWrapper reason of each row as if its class were unknown to the
// memo (the job checkers per row, cached; the task-group checkers per node
// signature, or per row when the group escapes), the memo class that turns
// later nodes of a failing class into "computed class ineligible", and the
// BinPack outcome. The caller's memo starts from the reference memo.
static void sys_metrics_build(pe_stack* s, TgPlan& g) {
    pe_stack::SysSpec& y = s->sys;
    const uint32_t n = (uint32_t)s->nodes.size(), ncls = s->ncls;
    y.mready = false;
    if (y.tcode.size() != n) return;
    jf_ready(s);
    y.mkey.assign(n, PE_NONE);
    y.mclass.assign(n, PE_NONE);
    y.mscore.assign(n, 0.0);
    y.mnode_class.resize(n);
    for (uint32_t r = 0; r < n; r++) {
        const uint32_t nc = s->nodes[r].node_class;
        y.mnode_class[r] = (nc != PE_NONE && !s->S(nc).empty()) ? nc : PE_NONE;
    }
    if (s->ref_job_memo.size() != ncls) s->ref_job_memo.assign(ncls, -1);
    auto& rt = s->ref_tg_memo[g.name];
    if (rt.size() != ncls) rt.assign(ncls, -1);
    y.mfailed.assign(2 * (size_t)ncls, 0);
    for (uint32_t c = 0; c < ncls; c++) {
        y.mfailed[c] = s->ref_job_memo[c] == 0;
        y.mfailed[ncls + c] = rt[c] == 0;
    }
    y.mfailed_eng = y.mfailed;
    pe::ConstraintEvaluator ev;
    std::vector<const char*> by_sig(s->sig_rep.size(), nullptr);
    std::vector<uint8_t> sig_done(s->sig_rep.size(), 0);
    for (uint32_t r = 0; r < n; r++) {
        const uint32_t c = s->jf_cls[r];
        const char* why = job_fail_cached(s, ev, r);
        uint32_t mc = PE_NONE;
        if (why) {
            if (!s->job_escaped) mc = c;
        } else if (g.escaped) {
            why = tg_fail(s, ev, g, s->view(r));
        } else {
            const uint32_t sg = s->nodes[r].sig;
            if (sg < sig_done.size()) {
                if (!sig_done[sg]) { by_sig[sg] = tg_fail(s, ev, g, s->view(r)); sig_done[sg] = 1; }
                why = by_sig[sg];
            } else {
                why = tg_fail(s, ev, g, s->view(r));
            }
            if (why) mc = ncls + c;
        }
        if (why) {
            y.mkey[r] = s->mkey_p(why);
            y.mclass[r] = mc;
            continue;
        }
        uint32_t kind, key;
        if (!trace_key(s, y.tcode[r], &kind, &key)) return;   // the view carries no maps: Selects cross
        y.mkey[r] = key;
        if (kind == 0) y.mscore[r] = y.tscore[6 * (size_t)r];   // binpack
    }
    y.mready = true;
}

static int sys_start(pe_stack* s, uint32_t tgi) {
    ApiScope prof_(s, "sys_start");
    pe_stack::SysSpec& y = s->sys;
    int rc = spec_flush(s);
    if (rc) return rc;
    HIP_TRY(s, hipSetDevice(s->device));
    rc = prepare_tg(s, tgi, s->visit, 0);
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (!sys_cacheable(s, g)) return PE_EUNSUPPORTED;   // the single Select path answers
    const uint32_t n = (uint32_t)s->nodes.size();
    if (s->identity_n != n) {
        std::vector<uint32_t> id(n);
        for (uint32_t i = 0; i < n; i++) id[i] = i;
        HIP_TRY(s, s->d_identity.ensure(sizeof(uint32_t) * (size_t)std::max<uint32_t>(n, 1)));
        HIP_TRY(s, hipMemcpyAsync(s->d_identity.p, id.data(), sizeof(uint32_t) * n, hipMemcpyHostToDevice, s->stream));
        s->identity_n = n;
    }
    HIP_TRY(s, s->d_sys_res.ensure(sizeof(uint64_t) * (size_t)std::max<uint32_t>(n, 1)));
    HIP_TRY(s, s->h_sys_cache.ensure(sizeof(uint64_t) * (size_t)std::max<uint32_t>(n, 1)));
    pe::SystemArgs A;
    std::memset(&A, 0, sizeof(A));
    A.soa = soa_of(s);
    A.tg = tables_of(g);
    A.ask = ask_for(s, g);
    A.log10 = s->log10;
    A.commit = 0;
    A.rank_of = s->d_identity.as<uint32_t>();   // every row, at its own position
    A.res = s->d_sys_res.as<uint64_t>();
    A.n_rows = n;
    A.n_list = 0;                                // outcomes stay in res, by row
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    HIP_TRY_STATE(s, pe_launch_system(&A, s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    HIP_TRY(s, hipMemcpyAsync(s->h_sys_cache.p, s->d_sys_res.p, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, s->stream));
    y.tcode.clear();
    y.tscore.clear();
    if (s->metrics_on) {
        // the AllocMetric outcome of every row in the same state (k_trace over
        // all rows; the FeasibilityWrapper half is walked per Select, since its
        // reasons depend on the order the caller visits the classes in)
        HIP_TRY(s, s->d_trace_out.ensure(sizeof(uint32_t) * (size_t)std::max<uint32_t>(n, 1)));
        HIP_TRY(s, s->d_trace_scores.ensure(6 * sizeof(double) * (size_t)std::max<uint32_t>(n, 1)));
        y.tcode.resize(n);
        y.tscore.resize(6 * (size_t)n);
        HIP_TRY_STATE(s, pe_launch_trace(&A.soa, &A.tg, &A.ask, s->d_identity.as<uint32_t>(), n,
                                         s->d_trace_out.as<uint32_t>(), nullptr, s->log10, nullptr,
                                         s->d_trace_scores.as<double>(), s->stream));
        HIP_TRY(s, hipMemcpyAsync(y.tcode.data(), s->d_trace_out.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                                  s->stream));
        HIP_TRY(s, hipMemcpyAsync(y.tscore.data(), s->d_trace_scores.p, 6 * sizeof(double) * n,
                                  hipMemcpyDeviceToHost, s->stream));
    }
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    y.mready = false;
    if (s->metrics_on) sys_metrics_build(s, g);
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    y.active = true;
    y.tgi = tgi;
    y.served_row = -1;
    y.passes++;
    sys_view_publish(s);
    return PE_OK;
}

// A plain single-node SystemStack.Select (stack.go:301-333) answered from the
// per-row cache. Returns false when the caller must take the single Select path.
static bool sys_serve(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out, int* rc) {
    pe_stack::SysSpec& y = s->sys;
    if (s->visit.size() != 1 || !s->have_job || tgi >= s->tgs.size()) return false;
    if (opts && (opts->penalty_count || opts->preferred_count || opts->preempt)) return false;
    if (!y.active || y.tgi != tgi) {
        // start at the group's first single-node Select: one pass over the
        // snapshot (~90 us at 100k rows) costs less than one single Select
        // after SetJob (~130 us with its launch and synchronisation)
        if (y.singles_tgi != tgi) { y.singles_tgi = tgi; y.singles = 0; }
        if (y.singles == PE_NONE) return false;   // not cacheable: the single Select path, until SetJob
        y.singles++;
        const int r = sys_start(s, tgi);
        if (r == PE_EUNSUPPORTED) { y.singles = PE_NONE; s->err.clear(); return false; }
        if (r) { *rc = r; return true; }
    }
    const uint32_t row = s->visit[0];
    const uint64_t v = s->h_sys_cache.as<uint64_t>()[row];
    if (v == kSysDirty) return false;
    const bool nan = (v & kSysNaN) == kSysNaN;
    const uint8_t st = nan ? (uint8_t)(v & 3u) : 0;
    if (st == 2 && s->cfg.preempt) return false;   // BinPack with evict: the single Select path
    double sc;
    std::memcpy(&sc, &v, sizeof(sc));
    out->row = st == 0 ? (int32_t)row : -1;
    out->n_scores = st == 0 ? 1u : 0u;
    out->final_score = st == 0 ? sc : 0.0;
    out->scores[0] = out->final_score;
    out->nodes_evaluated = 1;
    out->nodes_filtered = st == 1;
    out->nodes_exhausted = st == 2;
    out->new_offset = 0;
    out->n_preempted = 0;
    out->n_device_offers = 0;
    out->reserved_cores[0] = out->reserved_cores[1] = out->reserved_cores[2] = out->reserved_cores[3] = 0;
    y.served_row = out->row;
    y.served++;
    s->offer_row = out->row;
    s->offers = 0xFFFFFFFFu;
    s->metrics_valid = false;
    elig_log_span(s, tgi, 0, 1);
    *rc = PE_OK;
    if (s->metrics_on && row < y.tcode.size()) {   // the one node's maps (compute_metrics' steps)
        TgPlan& g = *s->tgs[tgi];
        MetricAcc acc;
        std::vector<uint32_t> rows;
        std::vector<MemoDelta> d;
        metrics_walk(s, g, s->visit, 0, 1, acc, rows, &d);   // advances the reference memo
        for (const MemoDelta& m : d)   // ... and the view's memo of failed classes
            if (m.v == 0 && y.mready && m.cls < s->ncls) {
                const size_t i = (m.tg ? s->ncls : 0u) + m.cls;
                if (i < y.mfailed.size()) y.mfailed[i] = y.mfailed_eng[i] = 1;
            }
        if (!rows.empty()) {
            std::map<int, std::vector<uint32_t>> counts;
            *rc = metrics_outcome(s, g, ask_for(s, g), row, y.tcode[row], &y.tscore[6 * (size_t)row], acc, counts);
        }
        if (*rc == PE_OK) metrics_set_last(s, acc);
    }
    return true;
}

int pe_select(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out) {
    PE_FLUSH_RESET(s);
    if (!s || !out) return PE_EINVAL;
    s->pre_overflow.clear();
    int rc = PE_OK;
    if (s->cfg.stack_kind == PE_STACK_SYSTEM && !s->test_fallback_every && sys_serve(s, tgi, opts, out, &rc))
        return rc;
    if (s->test_fallback_every && ++s->test_select_calls % s->test_fallback_every == 0) {
        // test hook: this Select is answered by the caller's Go chain (the
        // shim's PE_EUNSUPPORTED path); the engine state is the committed prefix
        rc = spec_flush(s);
        if (rc) return rc;
        return s->fail(PE_EUNSUPPORTED, "PE_TEST_FALLBACK_EVERY");
    }
    if (!spec_serve(s, tgi, opts, out)) {
        rc = spec_flush(s);
        if (rc) return rc;
        rc = spec_eligible(s, tgi, opts) ? spec_start(s, tgi, out) : select_impl(s, tgi, opts, out);
    }
    if (rc == PE_OK) {
        s->offer_row = out->row;
        s->offers = pack_offers(out);
        if (tgi < s->tgs.size()) core_record(s, *s->tgs[tgi], out->row, false, out->reserved_cores);
    }
    return rc;
}

// `rec`: the record's index in the call's output (PreemptedAllocs overflow).
static int select_impl(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out, uint32_t rec) {
    if (!s || !out) return PE_EINVAL;
    s->gen++;
    s->metrics_valid = false;
    HIP_TRY(s, hipSetDevice(s->device));
    if (s->cfg.stack_kind != PE_STACK_GENERIC) {
        // SystemStack.Select: single pass over the (single-node) list, no limit;
        // BinPack evicts when the scheduler configuration enables preemption
        // (multi-device verdicts are built for the state the Select sees)
        if (s->cfg.preempt && tgi < s->tgs.size() && tg_md(s, *s->tgs[tgi])) s->tgs[tgi]->tables_valid = false;
        int rc = prepare_tg(s, tgi, s->visit, 0);
        if (rc) return rc;
        uint32_t placed, no;
        const uint32_t saved = s->limit;
        s->limit = 1;
        if (s->cfg.preempt) rc = run_evict_select(s, *s->tgs[tgi], s->visit, 0, nullptr, out, &no, rec);
        else rc = run_place(s, tgi, 1, 0, s->visit, 0, nullptr, out, &placed, &no);
        s->limit = saved;
        if (rc == PE_OK) elig_log_span(s, tgi, 0, out->nodes_evaluated);
        if (rc == PE_OK && s->metrics_on)
            rc = compute_metrics(s, *s->tgs[tgi], s->visit, 0, out->nodes_evaluated, nullptr, s->cfg.preempt != 0);
        return rc;
    }
    if (opts && opts->preferred_count > 0) {
        // stack.go:121-132: select from the preferred nodes first, then the full
        // list; SetNodes resets the cursor to 0 either way.
        std::vector<uint32_t> pref(opts->preferred_rows, opts->preferred_rows + opts->preferred_count);
        std::vector<uint32_t> scan = pref;
        scan.insert(scan.end(), s->visit.begin(), s->visit.end());
        invalidate_tables(s);
        int rc = prepare_tg(s, tgi, scan, 0);
        if (rc) return rc;
        TgPlan& g = *s->tgs[tgi];
        if (tg_full_scan(s, g)) s->limit = 0x7FFFFFFF;
        pe_select_options o2 = *opts;
        o2.preferred_count = 0;
        uint32_t placed, no;
        if (opts->preempt) rc = run_evict_select(s, g, pref, 0, &o2, out, &no, rec);
        else rc = run_place(s, tgi, 1, 0, pref, 0, &o2, out, &placed, &no);
        if (rc) return rc;
        elig_visit_list(s, tgi, pref, out->nodes_evaluated);
        // the inner Select over the preferred list has its own AllocMetric
        // (ctx.Reset per Select); its walk also advances the memo shadow
        if (s->metrics_on) {
            rc = compute_metrics(s, g, pref, 0, out->nodes_evaluated, &o2, opts->preempt != 0);
            if (rc) return rc;
        }
        s->offset = 0;
        invalidate_tables(s);
        if (out->row >= 0) return PE_OK;
        return select_impl(s, tgi, &o2, out, rec);
    }
    if (opts && opts->preempt && tgi < s->tgs.size() && tg_md(s, *s->tgs[tgi]))
        s->tgs[tgi]->tables_valid = false;   // the multi-device verdicts for the state this Select sees
    int rc = prepare_tg(s, tgi, s->visit, s->offset);
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (tg_full_scan(s, g)) s->limit = 0x7FFFFFFF;   // never reset until SetNodes (stack.go:165-167)
    if (opts && opts->preempt) {
        uint32_t no;
        const uint32_t start0 = s->offset;
        rc = run_evict_select(s, g, s->visit, s->offset, opts, out, &no, rec);
        if (rc) return rc;
        s->offset = no;
        elig_log_span(s, tgi, start0, out->nodes_evaluated);
        if (s->metrics_on) rc = compute_metrics(s, g, s->visit, start0, out->nodes_evaluated, opts, true);
        return rc;
    }
    const uint32_t start = s->offset;
    if (s->limit >= s->visit.size() && s->visit.size() >= s->sweep_min && g.n_spread == (int)g.psets.size() &&
        s->visit_unique) {
        // a whole pass over a large list: multi-CU sweep instead of one workgroup
        rc = run_sweep_select(s, g, opts, out);
        if (rc == PE_OK) elig_log_span(s, tgi, start, out->nodes_evaluated);
        if (rc == PE_OK && s->metrics_on) rc = compute_metrics(s, g, s->visit, start, out->nodes_evaluated, opts);
        return rc;
    }
    uint32_t placed, no;
    rc = run_place(s, tgi, 1, 0, s->visit, s->offset, opts, out, &placed, &no);
    if (rc) return rc;
    s->offset = no;
    elig_log_span(s, tgi, start, out->nodes_evaluated);
    if (s->metrics_on) rc = compute_metrics(s, g, s->visit, start, out->nodes_evaluated, opts);
    return rc;
}

static int commit_impl(pe_stack* s, uint32_t tgi, int32_t row) {
    if (!s) return PE_EINVAL;
    if (!s->have_job || tgi >= s->tgs.size() || row < 0 || (size_t)row >= s->nodes.size())
        return s->fail(PE_EINVAL, "bad commit");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    TgPlan& g = *s->tgs[tgi];
    if (!g.psets_built) {
        int rc = build_psets(s, g);
        if (rc) return rc;
    }
    pe::NodeSoA soa = soa_of(s);
    pe::TgTables t = tables_of(g);
    pe::Ask a = ask_for(s, g);
    // the Select's own device offers when it chose this node (rank.go:404-405)
    const uint32_t offers = row == s->offer_row ? s->offers : 0xFFFFFFFFu;
    s->offer_row = -1;
    HIP_TRY_STATE(s, pe_launch_commit(&soa, &t, &a, (uint32_t)row, offers, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    plan_of(s).emplace_back(g.name, (uint32_t)row);
    invalidate_job_distinct(s, tgi);
    if (g.psets_dynamic) g.psets_built = false;   // cleared values: GetCombinedUseMap is not additive
    // the coll_tg of other task groups with the same name also see this alloc
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi && s->tgs[k]->name == g.name) {
            int rc = build_collisions(s);
            if (rc) return rc;
            break;
        }
    return PE_OK;
}

// Common checks of the sharded full-pass Select (pe_select_shard / pe_select_merge).
static int shard_prepare(pe_stack* s, uint32_t tgi, TgPlan** gp) {
    if (s->cfg.stack_kind != PE_STACK_GENERIC) return s->fail(PE_ESTATE, "sharded Select needs a generic stack");
    int rc = prepare_tg(s, tgi, s->visit, s->offset);
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (tg_full_scan(s, g)) s->limit = 0x7FFFFFFF;
    if (s->limit < s->visit.size())
        return s->fail(PE_EUNSUPPORTED, "sharded Select needs a full pass (affinities or spreads: limit MaxInt32)");
    if (!s->visit_unique) return s->fail(PE_EUNSUPPORTED, "sharded Select needs a visit list without repeated rows");
    if (g.n_spread != (int)g.psets.size()) return s->fail(PE_EUNSUPPORTED, "sharded Select with distinct_property");
    *gp = &g;
    return PE_OK;
}

int pe_select_shard(pe_stack* s, uint32_t tgi, uint32_t row_begin, uint32_t row_end, pe_shard_rec* out) {
    PE_FLUSH_RESET(s);
    if (!s || !out) return PE_EINVAL;
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    if (row_begin > row_end || row_end > s->nodes.size()) return s->fail(PE_EINVAL, "bad shard row range");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    TgPlan* g = nullptr;
    int rc = shard_prepare(s, tgi, &g);
    if (rc) return rc;
    pe::SweepArgs A;
    pe::SweepRec rec;
    rc = sweep_partial(s, *g, nullptr, row_begin, row_end, &A, &rec);
    if (rc) return rc;
    std::memset(out, 0, sizeof(*out));
    std::memcpy(out->bytes, &rec, sizeof(rec));
    return PE_OK;
}

int pe_select_merge(pe_stack* s, uint32_t tgi, const pe_shard_rec* recs, uint32_t n_recs, pe_ranked_node* out) {
    PE_FLUSH_RESET(s);
    if (!s || !out || (!recs && n_recs)) return PE_EINVAL;
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    TgPlan* g = nullptr;
    int rc = shard_prepare(s, tgi, &g);
    if (rc) return rc;
    pe::SweepRec all;
    pe_rec_init(&all);
    for (uint32_t i = 0; i < n_recs; i++) {
        pe::SweepRec r;
        std::memcpy(&r, recs[i].bytes, sizeof(r));
        pe_rec_merge(&all, &r);
    }
    pe::SweepArgs A;
    pe::SweepRec none;
    rc = sweep_partial(s, *g, nullptr, 0, 0, &A, &none);   // tables for the winner's record
    if (rc) return rc;
    rc = sweep_finish(s, A, all, out);
    if (rc) return rc;
    s->offer_row = out->row;
    s->offers = pack_offers(out);
    elig_log_span(s, tgi, s->offset, (uint32_t)s->visit.size());   // a full pass
    return PE_OK;
}

static int commit_preempt_impl(pe_stack* s, uint32_t tgi, int32_t row, const uint32_t* preempted,
                               uint32_t n_preempted) {
    if (!s) return PE_EINVAL;
    if (n_preempted == 0) return commit_impl(s, tgi, row);
    if (!preempted || !s->have_job || tgi >= s->tgs.size() || row < 0 || (size_t)row >= s->nodes.size())
        return s->fail(PE_EINVAL, "bad commit");
    if (!s->preempt_unsupported.empty()) return s->fail(PE_EUNSUPPORTED, "preemption: " + s->preempt_unsupported);
    // Plan.AppendPreemptedAlloc (structs.go:10664-10680) of allocs on the chosen node
    const uint32_t words = s->evict_words;
    std::vector<uint32_t> mask(words, 0u);
    const uint32_t b = s->h_node_alloc_off[(uint32_t)row];
    for (uint32_t i = 0; i < n_preempted; i++) {
        const uint32_t a = preempted[i];
        if (a >= s->allocs.size() || s->alloc_slot[a] == PE_NONE || s->allocs[a].row != (uint32_t)row)
            return s->fail(PE_EINVAL, "preempted alloc is not a live alloc of the node");
        const uint32_t k = s->alloc_slot[a] - b;
        if (k >= 32u * words) return s->fail(PE_EINTERNAL, "preempted alloc past the eviction width");
        mask[k >> 5] |= 1u << (k & 31u);
    }
    HIP_TRY(s, hipSetDevice(s->device));
    TgPlan& g = *s->tgs[tgi];
    pe::PreemptArgs P = preempt_args(s, g);
    HIP_TRY(s, upload_s(s, s->d_pre_mask, mask));
    HIP_TRY_STATE(s, pe_launch_commit_preempt(&P, (uint32_t)row, s->d_pre_mask.as<uint32_t>(),
                                              s->d_preempted.as<uint8_t>(), s->d_pcount.as<uint32_t>(),
                                              s->d_dev_free.as<uint32_t>(), s->stream));
    for (uint32_t i = 0; i < n_preempted; i++) {
        s->h_preempted[s->alloc_slot[preempted[i]]] = 1;
        invalidate_static(s);
        core_hold(s, preempted[i], false);
    }
    return commit_impl(s, tgi, row);
}


// Device-resident count loop over sparse options (k_ploop): the parallel
// Select loop of place_impl (plain Select, Preempt retry on nil, commit) as
// one single-workgroup launch. Valid while a commit changes the outcome of
// its own row only: no property sets (spread / distinct_property), a visit
// list without repeated rows, no max_parallel penalty (the plan's preemption
// counts would reach other nodes' eviction choices). *handled = false leaves
// the loop to the host-driven path (nothing committed).
// `rec0`: index of out[0] in the call's records; `words`: eviction width
// (0: the snapshot's). A launch that meets a node wider than its width stops
// there (the placements before it are committed) and the rest reruns wider.
static int ploop_count_loop(pe_stack* s, TgPlan& g, uint32_t tgi, uint32_t count, bool retry,
                            pe_ranked_node* out, uint32_t* placed, bool* handled, uint32_t rec0 = 0,
                            uint32_t words = 0) {
    *handled = false;
    *placed = 0;
    const uint32_t n = (uint32_t)s->visit.size();
    if (!count || (std::getenv("PE_PLOOP") && std::getenv("PE_PLOOP")[0] == '0')) return PE_OK;
    if (!g.psets.empty() || g.psets_dynamic || !s->visit_unique || n == 0) return PE_OK;
    if (g.ask.cores > 0) return PE_OK;   // k_ploop is compiled without reserved cores
    if (has_static(g)) return PE_OK;  // the static port gate is rebuilt on the host after evictions
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi && s->tgs[k]->name == g.name) return PE_OK;
    if (retry && !s->preempt_unsupported.empty()) return PE_OK;
    pe::BatchArgs A = batch_args(s, g);
    HIP_TRY(s, upload_visit(s, s->visit));
    A.perms = s->d_visit.as<uint32_t>();
    A.n_visit = n;
    HIP_TRY(s, s->d_ev_status_p.ensure(n));
    HIP_TRY(s, s->d_ev_score_p.ensure(sizeof(double) * n));
    HIP_TRY(s, s->d_ev_status.ensure(n));
    HIP_TRY(s, s->d_ev_score.ensure(sizeof(double) * n));
    HIP_TRY(s, s->d_ev_out.ensure(16));
    HIP_TRY(s, s->d_ev_flags.ensure(16));
    if (!words) words = s->evict_words;
    if (words > pe::kPLoopMaxWords) return PE_OK;   // nodes past k_ploop's width: the per-Select path (W = 32)
    if (n > pe_ploop_max_n(words)) return PE_OK;   // the outcome codes outgrow the workgroup's LDS
    HIP_TRY(s, s->d_loop_out.ensure(sizeof(pe_ranked_node) * (size_t)count));
    HIP_TRY(s, s->d_ploop_mask.ensure(sizeof(uint32_t) * words * (size_t)count));
    HIP_TRY(s, s->d_loop_state.ensure(8 * sizeof(uint32_t)));
    HIP_TRY(s, hipMemsetAsync(s->d_ev_out.p, 0, 16, s->stream));
    HIP_TRY(s, hipMemsetAsync(s->d_ev_flags.p, 0, 16, s->stream));
    HIP_TRY(s, hipMemsetAsync(s->d_loop_state.p, 0, 8 * sizeof(uint32_t), s->stream));
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    HIP_TRY(s, s->d_ploop_pparts.ensure(sizeof(double) * PE_MAX_SCORES * (size_t)n));
    HIP_TRY(s, s->d_ploop_pnparts.ensure(n));
    HIP_TRY_STATE(s, pe_launch_census(&A, s->d_ev_out.as<uint32_t>(), s->d_ev_status_p.as<uint8_t>(),
                                      s->d_ev_score_p.as<double>(), s->stream, s->d_ploop_pparts.as<double>(),
                                      s->d_ploop_pnparts.as<uint8_t>()));
    pe::PLoopArgs L;
    std::memset(&L, 0, sizeof(L));
    L.P = preempt_args(s, g);
    L.P.mask_words = words;
    L.P.visit = s->d_visit.as<uint32_t>();
    L.P.n_visit = n;
    L.P.status = s->d_ev_status.as<uint8_t>();
    L.P.score = s->d_ev_score.as<double>();
    L.P.flags = s->d_ev_flags.as<uint32_t>();
    if (retry) {
        HIP_TRY(s, s->d_ev_dep.ensure(n));
        L.P.dep_out = s->d_ev_dep.as<uint8_t>();
        L.dep_init = L.P.dep_out;
        // the Preempt record of every position is kept (and refreshed with its
        // outcome): a Preempt winner's record is then read, not re-evaluated
        HIP_TRY(s, s->d_ev_masks.ensure(sizeof(uint32_t) * words * (size_t)n));
        HIP_TRY(s, s->d_ev_offers.ensure(sizeof(uint32_t) * (size_t)n));
        HIP_TRY(s, s->d_ploop_parts.ensure(sizeof(double) * PE_MAX_SCORES * (size_t)n));
        HIP_TRY(s, s->d_ploop_nparts.ensure(n));
        L.P.mask_out = s->d_ev_masks.as<uint32_t>();
        L.P.offers_out = s->d_ev_offers.as<uint32_t>();
        L.P.parts_out = s->d_ploop_parts.as<double>();
        L.P.nparts_out = s->d_ploop_nparts.as<uint8_t>();
        HIP_TRY_STATE(s, pe_launch_evict_only(&L.P, s->stream));
        L.P.dep_out = nullptr;
        uint32_t flags = 0;
        HIP_TRY(s, hipMemcpyAsync(&flags, L.P.flags, sizeof(flags), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        if (flags & pe::kEvictUnsup) return PE_OK;   // outside the device path: the host loop reports it when reached
        if (flags & pe::kEvictWider) {   // nothing committed yet: the whole loop wider
            const uint32_t w = wider_words(words);
            if (!w) return PE_OK;
            return ploop_count_loop(s, g, tgi, count, retry, out, placed, handled, rec0, w);
        }
    } else {
        HIP_TRY(s, hipMemsetAsync(L.P.status, 3, n, s->stream));
    }
    L.st_plain = s->d_ev_status_p.as<uint8_t>();
    L.sc_plain = s->d_ev_score_p.as<double>();
    L.parts_plain = s->d_ploop_pparts.as<double>();
    L.nparts_plain = s->d_ploop_pnparts.as<uint8_t>();
    L.preempted = s->d_preempted.as<uint8_t>();
    L.pcount = s->d_pcount.as<uint32_t>();
    L.dev_free = s->d_dev_free.as<uint32_t>();
    L.offset = s->offset % n;
    L.limit = s->limit;
    L.count = count;
    L.retry = retry ? 1 : 0;
    {
        const char* cd = std::getenv("PE_PLOOP_CHECK_DEAD");
        L.check_dead = (cd && cd[0] && cd[0] != '0') ? 1 : 0;
    }
    L.out = s->d_loop_out.as<pe_ranked_node>();
    L.out_mask = s->d_ploop_mask.as<uint32_t>();
    L.state = s->d_loop_state.as<uint32_t>();
    if (retry && s->nil_sink) {   // the plain nils the Preempt retries follow (speculative run records)
        HIP_TRY(s, s->d_ploop_nil.ensure(sizeof(uint32_t) * 4 * (size_t)count));
        HIP_TRY(s, hipMemsetAsync(s->d_ploop_nil.p, 0xFF, sizeof(uint32_t) * 4 * (size_t)count, s->stream));
        L.nil_out = s->d_ploop_nil.as<uint32_t>();
    }
    const bool prof = std::getenv("PE_PLACE_PROF") != nullptr;
    if (prof) {
        HIP_TRY(s, s->d_prof.ensure(24 * sizeof(unsigned long long)));
        HIP_TRY(s, hipMemsetAsync(s->d_prof.p, 0, 24 * sizeof(unsigned long long), s->stream));
        L.prof = s->d_prof.as<unsigned long long>();
    }
    HIP_TRY_STATE(s, pe_launch_ploop(&L, s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    uint32_t st[4];
    HIP_TRY(s, hipMemcpyAsync(st, L.state, sizeof(st), hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    const uint32_t recs = std::min(st[3], count);
    std::vector<uint32_t> masks((size_t)recs * words);
    std::vector<std::array<uint32_t, 4>> nils(L.nil_out ? recs : 0u);
    if (recs) {
        HIP_TRY(s, hipMemcpyAsync(out, L.out, sizeof(pe_ranked_node) * recs, hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipMemcpyAsync(masks.data(), L.out_mask, sizeof(uint32_t) * words * recs, hipMemcpyDeviceToHost,
                                  s->stream));
        if (L.nil_out)
            HIP_TRY(s, hipMemcpyAsync(nils.data(), L.nil_out, sizeof(uint32_t) * 4 * recs, hipMemcpyDeviceToHost,
                                      s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        for (uint32_t k = 0; k < (uint32_t)nils.size(); k++)
            if (nils[k][0] != PE_NONE && rec0 + k < s->nil_sink->size()) (*s->nil_sink)[rec0 + k] = nils[k];
    }
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    if (prof) {
        unsigned long long h[24];
        HIP_TRY(s, hipMemcpy(h, L.prof, sizeof(h), hipMemcpyDeviceToHost));
        std::fprintf(stderr, "k_ploop: %u placements, %.3f ms total; us: plain resolve %.1f, refresh %.1f, preempt "
                             "resolve %.1f, winner %.1f (its evict_eval %.1f, commit %.1f); refreshed %llu dirty + %llu pcount "
                             "readers; winner evict_eval again, cache-warm %.1f (%llu calls); the next row's after it, data cold "
                             "%.1f (%llu calls)\n",
                     st[0], ms, h[0] / 100.0, h[1] / 100.0, h[2] / 100.0, h[3] / 100.0, h[6] / 100.0, h[7] / 100.0, h[4],
                     h[5], h[8] / 100.0, h[9], h[10] / 100.0, h[11]);
        std::fprintf(stderr, "k_ploop resolves: %llu steps in %llu calls; committed rows' plain re-evaluation %.1f us "
                             "(%llu calls)\n", h[12], h[13], h[14] / 100.0, h[15]);
        std::fprintf(stderr, "k_ploop winner detail us: record staging %.1f, plain eval + bookkeeping %.1f, end "
                             "barrier %.1f, plain winner records %.1f (%llu)\n",
                     h[17] / 100.0, h[18] / 100.0, h[19] / 100.0, h[20] / 100.0, h[21]);
    }
    *handled = true;
    const uint32_t p = std::min(st[0], count);
    for (uint32_t k = 0; k < recs; k++) std::memset(out[k].preempted, 0, sizeof(out[k].preempted));
    for (uint32_t k = 0; k < p; k++) {
        const uint32_t row = (uint32_t)out[k].row;
        plan_of(s).emplace_back(g.name, row);
        set_preempted(s, out[k], rec0 + k, row, masks.data() + (size_t)k * words, words, true);
    }
    *placed = p;
    s->offset = st[1];
    if (st[2] == 4) {   // a node wider than this launch: the remaining placements wider
        const uint32_t w = wider_words(words);
        if (!w) return s->fail(PE_EUNSUPPORTED, "preemption: a node's proposed allocs exceed the widest eviction width");
        uint32_t p2 = 0;
        bool h2 = false;
        const int rc = ploop_count_loop(s, g, tgi, count - p, retry, out + p, &p2, &h2, rec0 + p, w);
        *placed = p + p2;
        if (rc) return rc;
        *handled = h2;   // not handled: the host loop continues from *placed
        return PE_OK;
    }
    if (st[2] == 1)
        return s->fail(PE_EUNSUPPORTED, "preemption: a node outside the device path (several network devices, "
                                        "reserved cores)");
    if (st[2] == 2) return s->fail(PE_EINTERNAL, "k_ploop: the resolved winner is not an option");
    if (st[2] == 3)
        return s->fail(PE_EINTERNAL, "k_ploop: a plain Select skipped as provably failing found a winner");
    return PE_OK;
}

// Device-resident full-pass count loop (see pe_place). Same results as
// `count` x (run_sweep_select + pe_commit).
static int sweep_count_loop(pe_stack* s, TgPlan& g, uint32_t tgi, uint32_t count, pe_ranked_node* out,
                            uint32_t* placed) {
    ApiScope prof_(s, "sweep_count_loop");
    const uint32_t n = (uint32_t)s->visit.size();
    pe::SweepArgs A;
    uint32_t blocks = 0;
    int rc = sweep_setup(s, g, nullptr, 0, (uint32_t)s->nodes.size(), &A, &blocks);
    if (rc) return rc;
    // one placement is latency-bound: spread the rows over more workgroups
    // (256 rows each) than a single bandwidth-bound sweep would use
    blocks = std::max<uint32_t>(blocks, std::min<uint32_t>(((uint32_t)s->nodes.size() + 255) / 256,
                                                           (uint32_t)s->n_cu * (uint32_t)s->sweep_per_cu_aux));
    if (const char* e = std::getenv("PE_LOOP_BLOCKS")) blocks = (uint32_t)std::max(1, std::atoi(e));
    HIP_TRY(s, s->d_sweep_recs.ensure(sizeof(pe::SweepRec) * blocks));
    A.recs = s->d_sweep_recs.as<pe::SweepRec>();
    HIP_TRY(s, upload_visit(s, s->visit));
    HIP_TRY(s, s->d_loop_out.ensure(sizeof(pe_ranked_node) * (size_t)(count + 1)));
    HIP_TRY(s, s->d_loop_state.ensure(8 * sizeof(uint32_t)));
    HIP_TRY(s, hipMemsetAsync(s->d_loop_state.p, 0, 8 * sizeof(uint32_t), s->stream));
    uint32_t* state = s->d_loop_state.as<uint32_t>();
    uint32_t h_state[6] = {0, 0, 0, 0, 0, 0};
    const uint32_t chunk = 64;
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    // the first placement's spread table; each step rebuilds it for the next
    if (A.spread_tab) HIP_TRY(s, pe_launch_spread_table(&A.tg, s->d_spread_tab.as<double>(), s->stream));
    // lists whose options fit one workgroup's LDS: the whole loop in one
    // launch (k_fullpass_lds: 16 B of LDS per option, only the committed
    // node refreshed); more options than entries -> state[5], the loops below
    bool lds_loop = A.node_aux != nullptr && n <= kFullLdsMaxN && count > 0;
    if (const char* e = std::getenv("PE_FULL_LDS")) lds_loop = lds_loop && std::atoi(e) != 0;
    if (lds_loop) {
        const bool fprof = std::getenv("PE_FULL_PROF") != nullptr;   // per-phase clocks of the loop
        DevMem d_prof;
        if (fprof) HIP_TRY(s, d_prof.ensure(12 * sizeof(unsigned long long)));
        HIP_TRY(s, hipMemsetAsync(s->d_loop_out.p, 0, sizeof(pe_ranked_node) * (size_t)count, s->stream));
        s->h_full_args = A;
        HIP_TRY(s, s->d_full_args.ensure(sizeof(pe::SweepArgs)));
        HIP_TRY(s, hipMemcpyAsync(s->d_full_args.p, &s->h_full_args, sizeof(pe::SweepArgs), hipMemcpyHostToDevice,
                                  s->stream));
        const int np = A.spread_tab ? A.tg.n_psets : 0;
        // the service-wave loop (k_fullpass_svc, up to 3840 options): target
        // spreads and asks without devices or reserved cores (its commit is
        // the stores-only one), on runs long enough to repay building every
        // option's next entry too
        bool svc = !fprof && count >= 8 && A.ask.n_dev == 0 && A.ask.cores == 0 && np == A.tg.n_psets &&
                   A.tg.n_psets == A.tg.n_spread;
        for (int p = 0; p < g.n_spread && svc; p++) svc = !g.psets[p]->even;
        if (const char* e = std::getenv("PE_FULL_SVC")) svc = svc && std::atoi(e) != 0;
        if (svc) {
            ApiScope prof_k_(s, "sweep.svc_kernel+sync");
            // the lean service evaluation: asks whose dk-dependent checks are AllocsFit's alone
            bool lean = !A.ask.distinct_job && !A.ask.distinct_tg && A.ask.tg_dyn == 0 && !A.ask.has_task_net &&
                        !A.tg.static_gate && !A.tg.task_gate && !A.tg.md;
            if (const char* e = std::getenv("PE_SVC_LEAN")) lean = lean && std::atoi(e) != 0;
            HIP_TRY_STATE(s, pe_launch_fullpass_svc(s->d_full_args.as<pe::SweepArgs>(), np, lean,
                                              s->d_visit.as<uint32_t>(), n, count,
                                              s->d_loop_out.as<pe_ranked_node>(), state, s->stream));
            HIP_TRY(s, hipMemcpyAsync(h_state, state, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(s, hipStreamSynchronize(s->stream));
            svc = h_state[5] == 0;   // more options than its entries: nothing committed, the loop below
            if (!svc) HIP_TRY(s, hipMemsetAsync(state, 0, 8 * sizeof(uint32_t), s->stream));
        }
        if (!svc) {
            HIP_TRY_STATE(s, pe_launch_fullpass_lds(s->d_full_args.as<pe::SweepArgs>(), np,
                                              s->d_visit.as<uint32_t>(), n, count, s->d_loop_out.as<pe_ranked_node>(),
                                              state, fprof ? d_prof.as<unsigned long long>() : nullptr, s->stream));
            HIP_TRY(s, hipMemcpyAsync(h_state, state, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
            HIP_TRY(s, hipStreamSynchronize(s->stream));
        }
        if (fprof) {
            unsigned long long h[12];
            HIP_TRY(s, hipMemcpy(h, d_prof.p, sizeof(h), hipMemcpyDeviceToHost));
            const double p = std::max<uint32_t>(1, h_state[1]);
            std::fprintf(stderr, "k_fullpass_lds us/placement (wave 0): approx %.2f amax-reduce %.2f exact %.2f "
                         "best-reduce %.2f barrier %.2f resolve %.2f winner+commit %.2f table %.2f; winner lane: "
                         "load %.2f score %.2f record+commit %.2f\n",
                         h[4] / 100.0 / p, h[5] / 100.0 / p, h[6] / 100.0 / p, h[7] / 100.0 / p, h[0] / 100.0 / p,
                         h[1] / 100.0 / p, h[2] / 100.0 / p, h[3] / 100.0 / p, h[8] / 100.0 / p, h[9] / 100.0 / p,
                         h[10] / 100.0 / p);
        }
        if (h_state[5]) lds_loop = false;
    }
    const char* pe_env = std::getenv("PE_LOOP_PERSISTENT");
    // measured slower than back-to-back launches (10k nodes: 38.4 vs 34.6 us,
    // 100k: 145 vs 91 us per placement: the agent-scope barrier fences cost
    // more than the launch gaps they remove), so it is opt-in
    const bool persistent = pe_env ? std::atoi(pe_env) != 0 : false;
    if (persistent && count && !lds_loop) {
        // one launch for the whole loop: grid barriers between the sweep and
        // the step; at most one workgroup per CU so that all are resident
        const uint32_t pb = std::max<uint32_t>(1, std::min<uint32_t>(blocks, (uint32_t)s->n_cu));
        A.recs = s->d_sweep_recs.as<pe::SweepRec>();
        HIP_TRY_STATE(s, pe_launch_sweep_loop(&A, pb, count, s->d_visit.as<uint32_t>(), n, s->offset,
                                        s->d_loop_out.as<pe_ranked_node>(), state, s->stream));
        HIP_TRY(s, hipMemcpyAsync(h_state, state, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        if (h_state[4]) {
            s->have_state = false;   // partially committed: the caller must reload
            return s->fail(PE_EHIP, "persistent count loop: grid barrier timed out");
        }
    }
    for (uint32_t k = 0; !persistent && !lds_loop && k < count && !h_state[0]; k += chunk) {
        const uint32_t m = std::min(chunk, count - k);
        for (uint32_t j = 0; j < m; j++)
            HIP_TRY_STATE(s, pe_launch_sweep_step(&A, blocks, s->d_visit.as<uint32_t>(), n, s->offset,
                                            s->d_loop_out.as<pe_ranked_node>(), state, s->stream));
        HIP_TRY(s, hipMemcpyAsync(h_state, state, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
    }
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    const uint32_t p = h_state[1];
    const uint32_t nrec = std::min(count, p + (h_state[0] ? 1u : 0u));
    HIP_TRY(s, hipMemcpyAsync(out, s->d_loop_out.p, sizeof(pe_ranked_node) * nrec, hipMemcpyDeviceToHost, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    for (uint32_t i = 0; i < p; i++) plan_of(s).emplace_back(g.name, (uint32_t)out[i].row);   // Plan.AppendAlloc
    s->offer_row = -1;
    *placed = p;
    return PE_OK;
}

// The count loop of computePlacements on the device (pe_place). With
// `retry_preempt` a nil Select is retried with Preempt=true (selectNextOption,
// generic_sched.go:773-792) when the configuration enables preemption; without
// it the loop stops at the first nil Select (the speculative loop behind
// pe_select leaves the retry to the caller).
// The plain nil Select that placement k's Preempt retry follows, for the
// speculative run's records (nil_sink).
static inline void note_nil(pe_stack* s, uint32_t k, const pe_ranked_node& r) {
    if (s->nil_sink && k < s->nil_sink->size())
        (*s->nil_sink)[k] = {r.nodes_evaluated, r.nodes_filtered, r.nodes_exhausted, r.new_offset};
}

static int place_impl(pe_stack* s, uint32_t tgi, uint32_t count, pe_ranked_node* out, uint32_t* placed,
                      bool retry_preempt) {
    const bool prof = std::getenv("PE_PLACE_PROF") != nullptr;
    const double t_enter = prof ? now_us() : 0.0;
    if (!s || (!out && count)) return PE_EINVAL;
    // compact chain records for the speculation (spec_start), honoured by the
    // plain count loop below only
    std::vector<pe::EmitRec>* sink = s->emit_sink;
    s->emit_sink = nullptr;
    if (s->cfg.stack_kind != PE_STACK_GENERIC) return s->fail(PE_ESTATE, "pe_place needs a generic stack");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    // The table build's fold may ride in the windowed chain's first launch
    // (run_place); every other path below launches it first, and nothing
    // leaves this function with it pending.
    struct FoldGuard {
        pe_stack* s;
        ~FoldGuard() {
            s->fold_defer_ok = false;
            if (s->fold_pending) (void)flush_fold(s);
        }
    } fold_guard{s};
    s->fold_defer_ok = true;
    int rc = prepare_tg(s, tgi, s->visit, s->offset);
    s->fold_defer_ok = false;
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (tg_full_scan(s, g)) s->limit = 0x7FFFFFFF;
    const bool retry = retry_preempt && s->cfg.preempt;
    if (retry && g.md_on)   // the Preempt verdicts hold for one state: per Select (pe_select)
        return s->fail(PE_EUNSUPPORTED, "count loop with preemption on multi-device nodes");
    uint32_t p = 0, no = s->offset;
    if (g.psets_dynamic || retry || tg_full_scan(s, g)) {
        // no windowed chain launch first on these paths
        rc = flush_fold(s);
        if (rc) return rc;
    }
    if (g.psets_dynamic) {
        // plan stops clear property values: one Select at a time, the counts
        // rebuilt on the host after every commit
        while (p < count) {
            rc = select_impl(s, tgi, nullptr, &out[p], p);
            if (rc) return rc;
            if (out[p].row < 0) {
                if (!retry) break;
                note_nil(s, p, out[p]);
                pe_select_options o;   // selectNextOption: retry with Preempt=true
                std::memset(&o, 0, sizeof(o));
                o.preempt = 1;
                rc = select_impl(s, tgi, &o, &out[p], p);
                if (rc) return rc;
                if (out[p].row < 0) break;
                s->offer_row = out[p].row;
                s->offers = pack_offers(&out[p]);
                rc = commit_preempt_impl(s, tgi, out[p].row, preempted_list(s, p, out[p]), out[p].n_preempted);
                if (rc) return rc;
                p++;
                continue;
            }
            s->offer_row = out[p].row;
            s->offers = pack_offers(&out[p]);
            rc = commit_impl(s, tgi, out[p].row);
            if (rc) return rc;
            p++;
        }
        if (placed) *placed = p;
        return PE_OK;
    }
    // Sparse options (a saturated cluster): a windowed Select would walk
    // ~limit * n / options positions with one wave. Then every Select
    // evaluates the list in parallel and resolves the window on the device.
    bool parallel = false;
    const uint32_t nv = (uint32_t)s->visit.size();
    const double t_prep = prof ? now_us() : 0.0;
    const bool chain_ok = s->limit <= pe_chain_max_limit();
    if (count && g.psets.empty() && nv >= kParallelMinNodes && (s->cfg.preempt || !chain_ok)) {
        uint32_t cnt[3];
        rc = flush_fold(s);
        if (rc) return rc;
        rc = census(s, g, cnt);
        if (rc) return rc;
        parallel = cnt[0] == 0 || (uint64_t)std::min<uint32_t>(s->limit, nv) * nv / cnt[0] > kParallelWalk;
    }
    if (parallel) {
        bool handled = false;
        rc = ploop_count_loop(s, g, tgi, count, retry, out, &p, &handled);
        if (rc) return rc;
        while (!handled && p < count) {
            rc = run_parallel_select(s, g, &out[p], &no);
            if (rc) return rc;
            s->offset = no;
            if (out[p].row >= 0) {
                s->offer_row = out[p].row;
                s->offers = pack_offers(&out[p]);
                rc = commit_impl(s, tgi, out[p].row);
                if (rc) return rc;
                p++;
                continue;
            }
            if (!retry) break;
            note_nil(s, p, out[p]);
            pe_select_options o;   // selectNextOption: retry with Preempt=true
            std::memset(&o, 0, sizeof(o));
            o.preempt = 1;
            rc = run_evict_select(s, g, s->visit, s->offset, &o, &out[p], &no, p);
            if (rc) return rc;
            s->offset = no;
            if (out[p].row < 0) break;
            s->offer_row = out[p].row;
            s->offers = pack_offers(&out[p]);
            rc = commit_preempt_impl(s, tgi, out[p].row, preempted_list(s, p, out[p]), out[p].n_preempted);
            if (rc) return rc;
            if (has_static(g)) {   // the evictions freed ports: the gates and port records again
                rc = prepare_tg(s, tgi, s->visit, s->offset);
                if (rc) return rc;
            }
            p++;
        }
        count = 0;   // done: skip the fused loop below
        no = s->offset;
    }
    bool same_name = false;   // pe_commit would rebuild other task groups' collision counts
    for (size_t k = 0; k < s->tgs.size(); k++) same_name = same_name || (k != tgi && s->tgs[k]->name == g.name);
    if (count && !parallel && !retry && s->limit >= nv && nv >= s->loop_sweep_min && s->visit_unique &&
        g.n_spread == (int)g.psets.size() && !same_name) {
        // A whole pass per placement over a long list: k_place would sweep it
        // with one workgroup. Here every placement is a multi-CU sweep +
        // merge followed by k_sweep_step (winner record + commit on the
        // device), queued back to back with no host round trip; the host only
        // checks the stop flag between chunks. A full pass leaves the cursor.
        rc = flush_fold(s);
        if (rc) return rc;
        rc = sweep_count_loop(s, g, tgi, count, out, &p);
        if (rc) return rc;
        count = 0;
        no = s->offset;
    }
    if (count) {
        s->emit_sink = retry ? nullptr : sink;   // nothing below reads the records without a retry
        rc = run_place(s, tgi, count, 1, s->visit, s->offset, nullptr, out, &p, &no);
        s->emit_sink = nullptr;
        if (rc) return rc;
        s->offset = no;
        // selectNextOption (generic_sched.go:773-792): a nil Select is retried
        // with Preempt=true; the placement then evicts (handlePreemptions)
        while (retry && p < count) {
            note_nil(s, p, out[p]);   // out[p]: the plain Select's nil
            pe_select_options o;
            std::memset(&o, 0, sizeof(o));
            o.preempt = 1;
            rc = run_evict_select(s, g, s->visit, s->offset, &o, &out[p], &no, p);
            if (rc) return rc;
            s->offset = no;
            if (out[p].row < 0) break;
            s->offer_row = out[p].row;
            s->offers = pack_offers(&out[p]);
            rc = commit_preempt_impl(s, tgi, out[p].row, preempted_list(s, p, out[p]), out[p].n_preempted);
            if (rc) return rc;
            if (has_static(g)) {   // the evictions freed ports: the gates and port records again
                rc = prepare_tg(s, tgi, s->visit, s->offset);
                if (rc) return rc;
            }
            p++;
            if (p == count) break;
            if (!g.psets.empty()) {   // spread / distinct counts: the fused count loop
                uint32_t p2 = 0;
                rc = run_place(s, tgi, count - p, 1, s->visit, s->offset, nullptr, out + p, &p2, &no);
                if (rc) return rc;
                s->offset = no;
                p += p2;
                continue;
            }
            // Options are sparse once the cluster is saturated: plain Selects
            // evaluate the whole list in parallel and resolve the window on the
            // device instead of walking it with one wave, until one is nil.
            while (p < count) {
                rc = run_parallel_select(s, g, &out[p], &no);
                if (rc) return rc;
                s->offset = no;
                if (out[p].row < 0) break;
                s->offer_row = out[p].row;
                s->offers = pack_offers(&out[p]);
                rc = commit_impl(s, tgi, out[p].row);
                if (rc) return rc;
                p++;
            }
        }
        no = s->offset;
    }
    s->offset = no;
    if (placed) *placed = p;
    if (prof)
        std::fprintf(stderr, "pe_place: prepare %.1f us, loop %.1f us (kernels %.1f us)\n", t_prep - t_enter,
                     now_us() - t_prep, s->last_ms * 1e3);
    if (p) invalidate_job_distinct(s, tgi);
    // multi-tg jobs sharing a name see these allocs in their collision counts
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi && s->tgs[k]->name == g.name) { rc = build_collisions(s); if (rc) return rc; break; }
    return PE_OK;
}

// ---- speculative count loop behind pe_select / pe_commit --------------------
//
// GenericScheduler.computePlacements drives the stack one placement at a time:
// Select, build the alloc, Plan.AppendAlloc (generic_sched.go:552-627); the
// shim mirrors the append with pe_commit. Every fresh placement of a task
// group has the same empty SelectOptions, so the results of the next k
// Select/commit pairs are a pure function of the current state: exactly the
// device count loop (place_impl). The first plain Select therefore runs that
// loop for the group's remaining count and serves the first record; each
// later plain Select is served from the records as long as every commit named
// the predicted row. The loop commits into HBM after a checkpoint of the
// dynamic columns; when the caller deviates (another row, options, another
// task group, SetJob, SetNodes, ...) the columns are restored and the
// confirmed prefix is replayed (k_apply_commits), so the device state is
// always what the sequential calls would have produced.

static bool spec_serve(pe_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out) {
    view_take(s);
    pe_stack::Spec& sp = s->spec;
    if (!sp.active || sp.pending || tgi != sp.tgi || sp.served >= sp.n_rec || (s->metrics_on && !sp.metrics))
        return false;
    if (opts && (opts->penalty_count || opts->preferred_count)) return false;
    // a Preempt retry is answered by a Preempt record only, and vice versa
    const bool want_pre = opts && opts->preempt;
    if (want_pre != (sp.evict && (sp.rflags[sp.served] & PE_SPEC_PREEMPT) != 0)) return false;
    s->gen++;
    const uint32_t k = sp.served++;
    if (sp.compact) widen_rec(sp.crecs[k], out);
    else *out = sp.recs[k];
    if (spec_rec_npre(sp, k) > PE_MAX_PREEMPT)   // pe_preempted_of(s, 0, ...) of this Select
        s->pre_overflow.emplace_back(0u, std::vector<uint32_t>(spec_rec_pre(sp, k),
                                                                spec_rec_pre(sp, k) + spec_rec_npre(sp, k)));
    spec_settle(sp);
    elig_log_span(s, tgi, s->offset, out->nodes_evaluated);
    s->offset = out->new_offset;   // the StaticIterator cursor after this Select
    s->metrics_valid = false;
    spec_metrics_served(s, k);
    s->spec_stats[1]++;
    s->sview.served = sp.served;
    s->sview.confirmed = sp.confirmed;
    return true;
}

// Whether place_impl runs this group's loop as the phase-static chain.
static bool spec_chain_path(pe_stack* s, TgPlan& g) {
    const uint32_t nv = (uint32_t)s->visit.size();
    (void)nv;
    return !tg_full_scan(s, g) && !s->cfg.preempt && s->use_base && s->visit_unique &&
           s->limit <= pe_chain_max_limit() && g.ask.cores == 0;
}

static bool spec_eligible(pe_stack* s, uint32_t tgi, const pe_select_options* opts) {
    if (!s->spec_on || s->cfg.stack_kind != PE_STACK_GENERIC) return false;
    if (opts && (opts->penalty_count || opts->preferred_count || opts->preempt)) return false;
    if (!s->have_state || !s->have_job || tgi >= s->tgs.size()) return false;
    if (s->tgs[tgi]->ask.cores > 0) return false;   // the rollback kernel does not return reserved cores
    for (size_t k = 0; k < s->tgs.size(); k++)   // commits would rebuild a sibling's collision counts
        if (k != tgi && s->tgs[k]->name == s->tgs[tgi]->name) return false;
    // with AllocMetric on, the records' maps come from the batched trace
    // (spec_metrics) or the replay (spec_metrics_replay); static port asks
    // read host port mirrors that hold the run's end state: per Select
    if (s->metrics_on && has_static(*s->tgs[tgi])) return false;
    // multi-device nodes: the Preempt verdicts are built per Select (and
    // the maps' port texts from the host's records): no evicting or traced runs
    if ((s->cfg.preempt || s->metrics_on) && tg_md(s, *s->tgs[tgi])) return false;
    return true;
}

// Whether a run's maps come from one batched trace against the checkpoint
// (windowed, no evictions, no property sets: a record's state differs from
// the run's start by earlier placements alone), else from the replay.
// Whether spec_metrics traces the run's records in one batch: not for
// evicting runs nor distinct_property sets (their state moves with more than
// the placements), and within the batch's sizes (every record's passing rows
// of a full pass, every record's spread counts).
constexpr uint64_t kBatchedTraceRows = 12u << 20;
constexpr uint64_t kBatchedSpreadCounts = 4u << 20;
static bool spec_metrics_batched(pe_stack* s, TgPlan& g) {
    if (s->spec.evict || !g.distinct_props.empty() || g.psets.size() != (size_t)g.n_spread) return false;
    for (auto& c : s->job_constraints)
        if (c.op == "distinct_property") return false;
    const uint64_t n_rec = s->spec.n_rec;
    if (tg_full_scan(s, g) && n_rec * s->visit.size() > kBatchedTraceRows) return false;
    uint64_t nc = 0;
    for (auto& ps : g.psets) nc += ps->value_str.size();
    return n_rec * nc <= kBatchedSpreadCounts;
}

// Copies between the live dynamic columns and the checkpoint (to_ckpt: save).
static int spec_copy(pe_stack* s, TgPlan& g, bool to_ckpt) {
    {
        const int frc = flush_counts(s);   // the checkpoint copies the count arrays
        if (frc) return frc;
    }
    const size_t n = s->nodes.size();
    auto cp = [&](DevMem& live, DevMem& ck, size_t bytes) -> hipError_t {
        if (!bytes || !live.p) return hipSuccess;
        if (to_ckpt) {
            hipError_t e = ck.ensure(bytes);
            if (e != hipSuccess) return e;
            return hipMemcpyAsync(ck.p, live.p, bytes, hipMemcpyDeviceToDevice, s->stream);
        }
        return hipMemcpyAsync(live.p, ck.p, bytes, hipMemcpyDeviceToDevice, s->stream);
    };
    HIP_TRY(s, cp(s->d_rec, s->ck_rec, n * sizeof(pe::NodeRec)));
    HIP_TRY(s, cp(s->d_coll_job, s->ck_coll_job, n * sizeof(uint32_t)));
    HIP_TRY(s, cp(g.coll_tg, s->ck_coll_tg, n * sizeof(uint32_t)));
    HIP_TRY(s, cp(s->d_dev_free, s->ck_dev_free, n * sizeof(uint32_t)));
    for (size_t p = 0; p < g.psets.size() && p < (size_t)pe::kMaxPsets; p++)
        HIP_TRY(s, cp(g.psets[p]->counts, s->ck_pset[p], std::max<size_t>(g.psets[p]->value_str.size(), 1) * 4));
    if (s->spec.evict) {   // Plan.NodePreemptions: the preempted flags and the per-(job, tg) counts
        HIP_TRY(s, cp(s->d_preempted, s->ck_preempted, s->h_preempted.size()));
        HIP_TRY(s, cp(s->d_pcount, s->ck_pcount, sizeof(uint32_t) * std::max<uint32_t>(s->n_jtg_keys, 1)));
        // evictions free the evicted allocs' reserved cores (apply_preempt)
        if (s->has_cores) {
            HIP_TRY(s, cp(s->d_core_used, s->ck_core_used, sizeof(uint64_t) * 4 * n));
            if (to_ckpt) s->spec.core_used0 = s->h_core_used;
            else if (s->spec.core_used0.size() == s->h_core_used.size()) s->h_core_used = s->spec.core_used0;
        }
    }
    return PE_OK;
}

// An evicting run (§25) is undone from its checkpoint: the columns, the
// preempted flags and counts go back, the unconfirmed placements' preempted
// allocs rejoin the host mirror, and the confirmed prefix is replayed
// (its evictions, then its commits: both are sums, so their order is free).
static int spec_rollback_evict(pe_stack* s, uint32_t conf) {
    pe_stack::Spec& sp = s->spec;
    TgPlan& g = *s->tgs[sp.tgi];
    bool freed = false;
    for (uint32_t i = conf; i < sp.placed; i++) {
        const uint32_t k = sp.place_rec[i];
        for (uint32_t j = 0; j < spec_rec_npre(sp, k); j++) {
            const uint32_t slot = s->alloc_slot[spec_rec_pre(sp, k)[j]];
            if (slot != PE_NONE) s->h_preempted[slot] = 0;
            freed = true;
        }
    }
    if (freed) invalidate_static(s);
    int rc = spec_copy(s, g, false);
    if (rc) return rc;
    if (conf == 0) {
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        return PE_OK;
    }
    pe::Ask a = ask_for(s, g);
    pe::NodeSoA soa = soa_of(s);
    pe::TgTables t = tables_of(g);
    const uint32_t words = s->evict_words;
    std::vector<uint32_t> masks, mrows, rows(conf), offers(conf);
    for (uint32_t i = 0; i < conf; i++) {
        const uint32_t k = sp.place_rec[i];
        const uint32_t row = (uint32_t)spec_rec_row(sp, k);
        rows[i] = row;
        offers[i] = pack_offers(&sp.recs[k]);
        if (!spec_rec_npre(sp, k)) continue;
        const uint32_t b = s->h_node_alloc_off[row];
        const size_t at = masks.size();
        masks.resize(at + words, 0u);
        for (uint32_t j = 0; j < spec_rec_npre(sp, k); j++) {
            core_hold(s, spec_rec_pre(sp, k)[j], false);   // the confirmed eviction's cores stay free
            const uint32_t q = s->alloc_slot[spec_rec_pre(sp, k)[j]] - b;
            if (q >= 32u * words) return s->fail(PE_EINTERNAL, "replayed preemption past the eviction width");
            masks[at + (q >> 5)] |= 1u << (q & 31u);
        }
        mrows.push_back(row);
    }
    if (!mrows.empty()) {
        pe::PreemptArgs P = preempt_args(s, g);
        HIP_TRY(s, upload_s(s, s->d_pre_mask, masks));
        for (size_t j = 0; j < mrows.size(); j++)
            HIP_TRY_STATE(s, pe_launch_commit_preempt(&P, mrows[j], s->d_pre_mask.as<uint32_t>() + j * words,
                                                      s->d_preempted.as<uint8_t>(), s->d_pcount.as<uint32_t>(),
                                                      s->d_dev_free.as<uint32_t>(), s->stream));
    }
    HIP_TRY(s, upload_s(s, s->d_commit_rows, rows));
    HIP_TRY(s, upload_s(s, s->d_commit_offers, offers));
    HIP_TRY_STATE(s, pe_launch_apply_commits(&soa, &t, &a, s->d_commit_rows.as<uint32_t>(),
                                             s->d_commit_offers.as<uint32_t>(), conf, 1, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    return PE_OK;
}

static int spec_flush(pe_stack* s) {
    if (!s->sys.pending.empty()) {
        const int rc = sys_flush(s);
        if (rc) return rc;
    }
    view_take(s);
    pe_stack::Spec& sp = s->spec;
    if (!sp.active) return PE_OK;
    view_withdraw(s);
    sp.active = false;
    sp.pending = false;
    if (sp.metrics) {   // the reference memo as the served records' walks left it
        spec_memo_rewind(s, sp.served);
        sp.metrics = false;
    }
    const uint32_t conf = spec_conf_placed(sp);
    const bool used_up = sp.served == sp.n_rec && conf == sp.placed && sp.n_rec > 0 &&
                         spec_rec_row(sp, sp.n_rec - 1) >= 0;
    // run length of the next run on a costly path: x4 while runs get used up
    // (a run's fixed cost, ~0.1-0.4 ms, over fewer runs), back to one
    // placement after a deviation
    sp.grow = used_up ? std::min<uint32_t>(4 * sp.grow, 4096) : 1;
    if (conf == sp.placed) return PE_OK;   // HBM holds exactly the confirmed placements
    HIP_TRY(s, hipSetDevice(s->device));
    s->spec_stats[2]++;
    if (sp.evict) return spec_rollback_evict(s, conf);
    TgPlan& g = *s->tgs[sp.tgi];
    pe::Ask a = ask_for(s, g);
    pe::NodeSoA soa = soa_of(s);
    pe::TgTables t = tables_of(g);
    if (!sp.checkpoint) {
        // no device ask: every commit added the same ask to its row, so the
        // unconfirmed placements are taken back by subtracting them again
        std::vector<uint32_t> rows(sp.placed - conf), offers(rows.size(), 0xFFFFFFFFu);
        for (uint32_t i = conf; i < sp.placed; i++) rows[i - conf] = (uint32_t)spec_row(sp, i);
        HIP_TRY(s, upload_s(s, s->d_commit_rows, rows));
        HIP_TRY(s, upload_s(s, s->d_commit_offers, offers));
        HIP_TRY_STATE(s, pe_launch_apply_commits(&soa, &t, &a, s->d_commit_rows.as<uint32_t>(),
                                           s->d_commit_offers.as<uint32_t>(), (uint32_t)rows.size(), -1,
                                           s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        return PE_OK;
    }
    int rc = spec_copy(s, g, false);
    if (rc) return rc;
    if (conf == 0) return PE_OK;
    std::vector<uint32_t> rows(conf), offers(conf);
    bool ordered_only = false;   // a device ask without a recorded offer: replay one by one
    for (uint32_t i = 0; i < conf; i++) {
        rows[i] = (uint32_t)spec_row(sp, i);
        if (sp.compact) {
            pe_ranked_node r;
            widen_rec(sp.crecs[i], &r);
            offers[i] = pack_offers(&r);
        } else {
            offers[i] = pack_offers(&sp.recs[i]);
        }
        if (a.n_dev > 0 && offers[i] == 0xFFFFFFFFu) ordered_only = true;
    }
    if (ordered_only) {
        for (uint32_t i = 0; i < conf; i++)
            HIP_TRY_STATE(s, pe_launch_commit(&soa, &t, &a, rows[i], offers[i], s->stream));
    } else {
        HIP_TRY(s, upload_s(s, s->d_commit_rows, rows));
        HIP_TRY(s, upload_s(s, s->d_commit_offers, offers));
        HIP_TRY_STATE(s, pe_launch_apply_commits(&soa, &t, &a, s->d_commit_rows.as<uint32_t>(),
                                           s->d_commit_offers.as<uint32_t>(), conf, 1, s->stream));
    }
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    return PE_OK;
}

// Drop the speculation without touching the device (the state is being reset).
static void spec_drop(pe_stack* s) {
    view_withdraw(s);
    s->spec.metrics = false;
    s->spec.active = false;
    s->spec.pending = false;
    s->spec.grow = 1;
    sys_deactivate(s);   // a new evaluation context: queued commits are moot
    s->sys.pending.clear();
    s->sys.singles = 0;
    s->sys.singles_tgi = PE_NONE;
    s->sys.served_row = -1;
}

static int spec_start(pe_stack* s, uint32_t tgi, pe_ranked_node* out) {
    ApiScope prof_(s, "spec_start");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    // the table build's fold may ride in the run's first launch (place_impl,
    // run_place); nothing leaves spec_start with it pending
    struct FoldGuard {
        pe_stack* s;
        ~FoldGuard() {
            s->fold_defer_ok = false;
            if (s->fold_pending) (void)flush_fold(s);
        }
    } fold_guard{s};
    s->fold_defer_ok = true;
    int rc = prepare_tg(s, tgi, s->visit, s->offset);
    s->fold_defer_ok = false;
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (g.psets_dynamic) return select_impl(s, tgi, nullptr, out);   // counts rebuilt per commit: no run
    pe_stack::Spec& sp = s->spec;
    // placements of the group still to come in this evaluation (tg.Count minus
    // the plan's), at least the run length grown from earlier used-up runs
    uint32_t done = 0;
    for (auto& p : plan_of(s)) done += p.first == g.name;
    uint32_t count = g.count > 0 && (uint32_t)g.count > done ? (uint32_t)g.count - done : 0u;
    // The phase-static chain (k_base + k_chain) costs about the same for one
    // placement as for the whole count: run the group's remaining count. Every
    // other loop pays per placement: start with one and double while the runs
    // get used up (spec_flush).
    // A full-pass loop (k_fullpass_svc) pays ~50 us to build its entries
    // and ~0.1 ms of launch and host work per run whatever its length, and
    // ~3.5 us per placement: its runs start at 64.
    const uint32_t grow = tg_full_scan(s, g) && !s->cfg.preempt ? std::max<uint32_t>(sp.grow, 64u) : sp.grow;
    sp.grow = grow;   // (x4 from here while the runs get used up)
    count = spec_chain_path(s, g) ? std::max<uint32_t>(count, 1u) : std::max<uint32_t>(std::min(count, grow), 1u);
    // (with AllocMetric on, spec_metrics counts a row's earlier placements in 16 bits)
    count = std::min<uint32_t>(count, s->metrics_on ? 0xFFFFu : 1u << 16);
    // With preemption enabled the run is selectNextOption's loop (generic_sched.go:
    // 773-792): a nil plain Select retried with Preempt=true, whose placement
    // evicts (§25). Evictions are not undone by subtraction: checkpoint.
    sp.evict = s->cfg.preempt != 0;
    sp.metrics = false;
    // device offers are not undone by subtraction; the AllocMetric trace reads
    // the starting state from the checkpoint
    sp.checkpoint = sp.evict || ask_for(s, g).n_dev > 0 || s->metrics_on;
    if (sp.checkpoint) {
        rc = spec_copy(s, g, true);
        if (rc) return rc;
    }
    const size_t plan0 = plan_of(s).size();
    if (sp.recs.size() < count) sp.recs.resize(count);
    uint32_t placed = 0;
    s->emit_sink = sp.evict ? nullptr : &sp.crecs;
    s->emit_sunk = false;
    const uint32_t off0 = s->offset;
    std::vector<std::array<uint32_t, 4>> nils;
    if (sp.evict) {
        nils.assign(count + 1, std::array<uint32_t, 4>{PE_NONE, 0u, 0u, 0u});
        s->nil_sink = &nils;
        s->pre_overflow.clear();
    }
    s->elig_mute = true;   // records are logged when served
    rc = place_impl(s, tgi, count, sp.recs.data(), &placed, sp.evict);
    s->elig_mute = false;
    s->emit_sink = nullptr;
    s->nil_sink = nullptr;
    sp.compact = !sp.evict && s->emit_sunk;
    plan_of(s).resize(plan0);   // the plan holds confirmed placements only
    // A failed run leaves the device as the caller last saw it (and the host
    // mirror of the preempted allocs: the run's placements are dropped).
    auto undo_run = [&](int err) {
        if (sp.checkpoint) {
            if (sp.evict)
                for (uint32_t k = 0; k < placed && k < count; k++) {
                    const uint32_t* l = preempted_list(s, k, sp.recs[k]);
                    for (uint32_t j = 0; l && j < sp.recs[k].n_preempted; j++) {
                        const uint32_t slot = s->alloc_slot[l[j]];
                        if (slot != PE_NONE) s->h_preempted[slot] = 0;
                    }
                }
            const int rc2 = spec_copy(s, g, false);
            (void)rc2;
            if (sp.evict) invalidate_static(s);
        }
        (void)hipStreamSynchronize(s->stream);
        sp.evict = false;
        return err;
    };
    if (rc) return undo_run(rc);
    sp.active = true;
    sp.pending = false;
    sp.tgi = tgi;
    sp.placed = placed;
    sp.n_rec = placed < count ? placed + 1 : placed;
    if (sp.evict) {
        // the Select answers in order: an evicting placement is the plain
        // Select's nil, then the Preempt retry's option
        std::vector<pe_ranked_node> seq;
        seq.reserve(2 * (size_t)sp.n_rec);
        sp.rec_place.clear();
        sp.place_rec.clear();
        sp.rflags.clear();
        sp.pre_off.assign(1, 0u);
        sp.pre_list.clear();
        for (uint32_t k = 0; k < sp.n_rec; k++) {
            const pe_ranked_node& r = sp.recs[k];
            if (nils[k][0] != PE_NONE) {
                pe_ranked_node z;
                std::memset(&z, 0, sizeof(z));
                z.row = -1;
                z.nodes_evaluated = nils[k][0];
                z.nodes_filtered = nils[k][1];
                z.nodes_exhausted = nils[k][2];
                z.new_offset = nils[k][3];
                seq.push_back(z);
                sp.rec_place.push_back(PE_NONE);
                sp.rflags.push_back(0u);
                sp.pre_off.push_back((uint32_t)sp.pre_list.size());
            }
            const uint32_t np = r.row >= 0 ? r.n_preempted : 0u;
            const uint32_t* l = np ? preempted_list(s, k, r) : nullptr;
            if (np && !l) return undo_run(s->fail(PE_EINTERNAL, "speculative loop: a record's PreemptedAllocs are missing"));
            if (k < placed) sp.place_rec.push_back((uint32_t)seq.size());
            seq.push_back(r);
            sp.rec_place.push_back(k < placed ? k : PE_NONE);
            sp.rflags.push_back(nils[k][0] != PE_NONE ? PE_SPEC_PREEMPT : 0u);
            sp.pre_list.insert(sp.pre_list.end(), l, l + np);
            sp.pre_off.push_back((uint32_t)sp.pre_list.size());
        }
        sp.recs.swap(seq);
        sp.n_rec = (uint32_t)sp.recs.size();
        s->pre_overflow.clear();
    }
    if (s->metrics_on) {
        const int mrc = spec_metrics_batched(s, g) ? spec_metrics(s, g, off0) : spec_metrics_replay(s, g, off0);
        if (mrc) {   // nothing served yet: the device and the memo go back to the run's start
            sp.active = true;
            sp.served = sp.confirmed = 0;
            sp.metrics = true;   // spec_metrics set memo_job0 / memo_tg0 / memo_off first: rewind to them
            spec_memo_rewind(s, 0);
            sp.metrics = false;
            (void)spec_flush(s);
            return mrc;
        }
    }
    sp.served = 0;
    sp.confirmed = 0;
    s->spec_stats[0]++;
    s->spec_stats[3] += sp.n_rec;
    s->offer_row = -1;
    s->offset = off0;   // the run left the cursor at its end: serving advances it record by record
    if (!spec_serve(s, tgi, nullptr, out)) return s->fail(PE_ESTATE, "speculative loop produced no record");
    s->spec_stats[1]--;   // the first record is the Select that started the run
    view_publish(s);
    return PE_OK;
}

static int place_one(pe_stack* s, uint32_t tgi, uint32_t count, pe_ranked_node* out, uint32_t* placed) {
    if (!s) return PE_EINVAL;
    int rc = spec_flush(s);
    if (rc) return rc;
    uint32_t p = 0;
    const uint32_t start = s->offset;
    s->elig_mute = true;   // the windows are logged from the records below
    rc = place_impl(s, tgi, count, out, &p, true);
    s->elig_mute = false;
    if (placed) *placed = p;
    if (rc == PE_OK && count) {
        // Consecutive windows continue the cursor. A nil Select (the last
        // record when p < count, or the plain Select before a Preempt retry,
        // whose placement then evicts) pulled the whole list.
        uint64_t pulled = 0;
        bool whole = p < count;
        for (uint32_t k = 0; k < std::min(p + 1, count); k++) {
            pulled += out[k].nodes_evaluated;
            whole = whole || (k < p && out[k].n_preempted > 0);
        }
        elig_log_span(s, tgi, start, whole ? (uint32_t)s->visit.size()
                                           : (uint32_t)std::min<uint64_t>(pulled, s->visit.size()));
    }
    if (tgi < s->tgs.size() && s->tgs[tgi]->ask.cores > 0)   // the placements' reserved cores, in order
        for (uint32_t k = 0; k < p && k < count; k++) core_record(s, *s->tgs[tgi], out[k].row, true, out[k].reserved_cores);
    return rc;
}

static int commit_one(pe_stack* s, uint32_t tgi, int32_t row) {
    if (!s) return PE_EINVAL;
    if (s->sys.active && tgi == s->sys.tgi && row >= 0 && row == s->sys.served_row) {
        // the served single-node Select's Plan.AppendAlloc: queued for HBM
        s->sys.served_row = -1;
        s->sys.pending.push_back((uint32_t)row);
        s->h_sys_cache.as<uint64_t>()[(uint32_t)row] = kSysDirty;
        plan_of(s).emplace_back(s->tgs[tgi]->name, (uint32_t)row);
        s->offer_row = -1;
        return PE_OK;
    }
    if (s->sys.active && row >= 0) sys_touch(s, (uint32_t)row);
    view_take(s);
    pe_stack::Spec& sp = s->spec;
    if (sp.active && sp.pending && tgi == sp.tgi && row == spec_rec_row(sp, sp.served - 1) &&
        spec_rec_npre(sp, sp.served - 1) == 0) {
        // the predicted Plan.AppendAlloc: already in HBM
        sp.pending = false;
        sp.confirmed = sp.served;
        s->sview.confirmed = sp.confirmed;
        spec_confirm_rec(s, sp.served - 1, false);   // pe_commit logs it for the replicas
        s->offer_row = -1;
        return PE_OK;
    }
    int rc = spec_flush(s);
    if (rc) return rc;
    rc = commit_impl(s, tgi, row);
    uint64_t cores[4];
    if (rc == PE_OK) core_record(s, *s->tgs[tgi], row, true, cores);
    return rc;
}

static int commit_preempt_one(pe_stack* s, uint32_t tgi, int32_t row, const uint32_t* preempted, uint32_t n_preempted) {
    if (!s) return PE_EINVAL;
    if (n_preempted == 0) return commit_one(s, tgi, row);
    view_take(s);
    pe_stack::Spec& sp = s->spec;
    if (preempted && sp.active && sp.pending && tgi == sp.tgi && row == spec_rec_row(sp, sp.served - 1) &&
        n_preempted == spec_rec_npre(sp, sp.served - 1) &&
        std::equal(preempted, preempted + n_preempted, spec_rec_pre(sp, sp.served - 1))) {
        // the predicted Plan.AppendAlloc + AppendPreemptedAlloc: already in HBM
        sp.pending = false;
        sp.confirmed = sp.served;
        s->sview.confirmed = sp.confirmed;
        spec_confirm_rec(s, sp.served - 1, false);   // pe_commit_preempt logs it for the replicas
        s->offer_row = -1;
        return PE_OK;
    }
    int rc = spec_flush(s);
    if (rc) return rc;
    if (s->sys.active && row >= 0) sys_touch(s, (uint32_t)row);
    rc = commit_preempt_impl(s, tgi, row, preempted, n_preempted);
    uint64_t cores[4];
    if (rc == PE_OK) core_record(s, *s->tgs[tgi], row, true, cores);
    return rc;
}

// Plan.NodeUpdate bookkeeping shared by pe_plan_stop / pe_plan_pop_update:
// allocs whose entry count crossed 0 <-> 1 leave / rejoin the proposed state.
static int apply_stop_delta(pe_stack* s, const std::vector<uint32_t>& allocs, int sign) {
    std::vector<uint32_t> slots, rows;
    for (uint32_t ai : allocs) {
        const HostAlloc& a = s->allocs[ai];
        const uint32_t slot = s->alloc_slot[ai];
        if (a.terminal || slot == PE_NONE) continue;   // not in AllocsByNodeTerminal(false)
        uint8_t& f = s->h_preempted[slot];
        if (sign > 0 ? f != 0 : f != 2) continue;        // already out via a plan preemption
        f = sign > 0 ? 2 : 0;
        slots.push_back(slot);
        rows.push_back(a.row);
        if (s->sys.active) sys_touch(s, a.row);   // its node's cached outcome is stale
        core_hold(s, ai, sign < 0);   // its reserved cores leave (rejoin) the node's used set
        invalidate_static(s);         // and its ports
    }
    if (!slots.empty()) {
        HIP_TRY(s, upload_s(s, s->d_stop_slots, slots));
        HIP_TRY(s, upload_s(s, s->d_stop_rows, rows));
        HIP_TRY(s, pe_launch_plan_stop(s->d_rec.as<pe::NodeRec>(), s->dev_packable ? s->d_dev_free.as<uint32_t>() : nullptr,
                                       s->d_palloc.as<pe::PreemptAlloc>(), s->d_preempted.as<uint8_t>(),
                                       s->d_stop_slots.as<uint32_t>(), s->d_stop_rows.as<uint32_t>(),
                                       (uint32_t)slots.size(), sign, s->has_cores ? s->d_core_used.as<uint64_t>() : nullptr,
                                       s->has_cores ? s->d_palloc_cores.as<uint64_t>() : nullptr, s->stream));
    }
    // the job's own allocs feed the collision counts and the property sets
    for (auto& g : s->tgs) g->psets_built = false;
    if (s->have_job) return build_job_counts(s);
    return PE_OK;
}

static int plan_stop_one(pe_stack* s, const uint32_t* allocs, uint32_t n) {
    if (!s || (!allocs && n)) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    for (uint32_t i = 0; i < n; i++)
        if (allocs[i] >= s->allocs.size()) return s->fail(PE_EINVAL, "alloc index out of range");
    int rc = spec_flush(s);
    if (rc) return rc;
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    if (s->stop_count.size() != s->allocs.size()) s->stop_count.assign(s->allocs.size(), 0);
    std::vector<uint32_t> fresh;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t ai = allocs[i];
        s->node_update[s->allocs[ai].row].push_back(ai);   // AppendStoppedAlloc: NodeUpdate[node] += alloc
        if (s->stop_count[ai]++ == 0) fresh.push_back(ai);
    }
    return apply_stop_delta(s, fresh, +1);
}

static int plan_pop_update_one(pe_stack* s, uint32_t alloc) {
    if (!s) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    if (alloc >= s->allocs.size()) return s->fail(PE_EINVAL, "alloc index out of range");
    int rc = spec_flush(s);
    if (rc) return rc;
    auto it = s->node_update.find(s->allocs[alloc].row);
    // PopUpdate (structs.go:10691-10702): only the node's last entry, by ID
    if (it == s->node_update.end() || it->second.empty() || it->second.back() != alloc) return PE_OK;
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    it->second.pop_back();
    if (it->second.empty()) s->node_update.erase(it);
    std::vector<uint32_t> gone;
    if (--s->stop_count[alloc] == 0) gone.push_back(alloc);
    return apply_stop_delta(s, gone, -1);
}

// ---- multi-GPU ------------------------------------------------

int pe_comm_unique_id(uint8_t* out, size_t cap) {
    if (!out || cap < NCCL_UNIQUE_ID_BYTES) return PE_EINVAL;
    ncclUniqueId id;
    if (rc_GetUniqueId(&id) != ncclSuccess) return PE_EHIP;
    std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return PE_OK;
}

int pe_comm_init(pe_stack* s, int nranks, int rank, const uint8_t* id) {
    PE_FLUSH_RESET(s);
    if (!s || !id || nranks < 1 || rank < 0 || rank >= nranks) return PE_EINVAL;
    HIP_TRY(s, hipSetDevice(s->device));
    if (s->comm) {
        (void)rc_CommDestroy(s->comm);
        s->comm = nullptr;
    }
    s->xfn = nullptr;
    s->xctx = nullptr;
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    const ncclResult_t r = rc_CommInitRank(&s->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        s->comm = nullptr;
        return s->fail(PE_EHIP, std::string("ncclCommInitRank: ") + rc_GetErrorString(r));
    }
    s->nranks = nranks;
    s->rank = rank;
    if (!s->ev_x0) HIP_TRY(s, hipEventCreate(&s->ev_x0));
    if (!s->ev_x1) HIP_TRY(s, hipEventCreate(&s->ev_x1));
    return PE_OK;
}

int pe_comm_init_host(pe_stack* s, int nranks, int rank, pe_exchange_fn exchange, void* ctx) {
    PE_FLUSH_RESET(s);
    if (!s || !exchange || nranks < 1 || rank < 0 || rank >= nranks) return PE_EINVAL;
    HIP_TRY(s, hipSetDevice(s->device));
    if (s->comm) {
        (void)rc_CommDestroy(s->comm);
        s->comm = nullptr;
    }
    if (s->h_xbuf) {
        (void)hipHostFree(s->h_xbuf);
        s->h_xbuf = nullptr;
    }
    HIP_TRY(s, hipHostMalloc(&s->h_xbuf, sizeof(pe::SweepRec) * ((size_t)nranks + 1), hipHostMallocDefault));
    s->xfn = exchange;
    s->xctx = ctx;
    s->nranks = nranks;
    s->rank = rank;
    return PE_OK;
}

// The full-pass count loop (limit >= list, affinity / spread task groups)
// sharded over the communicator's ranks: every rank holds the whole snapshot
// and sweeps rows [row_begin, row_end); per placement k_sweep's last
// workgroup merges the rank's workgroup records into its one 80-byte record
// (at its rank's slot of the gather buffer), one in-place ncclAllGather of the
// nranks records runs over xGMI on the engine stream (an identity at one rank,
// skipped), and k_sweep_step merges them, resolves the winner (SURVEY.md
// Appendix A1), writes its record and commits it on every rank. Nothing
// returns to the host between placements; the stop flag is read every 64
// placements. With a host transport (pe_comm_init_host) the record goes
// through the caller's all-gather instead, once per placement.
static int place_sharded_impl(pe_stack* s, uint32_t tgi, uint32_t count, uint32_t row_begin, uint32_t row_end,
                     pe_ranked_node* out, uint32_t* placed) {
    if (!s || (!out && count)) return PE_EINVAL;
    if (!s->comm && !s->xfn) return s->fail(PE_ESTATE, "pe_comm_init not called");
    if (s->cfg.stack_kind != PE_STACK_GENERIC) return s->fail(PE_ESTATE, "sharded placement needs a generic stack");
    int rc = spec_flush(s);
    if (rc) return rc;
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    if (row_begin > row_end || row_end > s->nodes.size()) return s->fail(PE_EINVAL, "bad shard row range");
    rc = prepare_tg(s, tgi, s->visit, s->offset);
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    if (!tg_full_scan(s, g)) return s->fail(PE_EUNSUPPORTED, "sharded placement: a windowed task group (replicas only)");
    if (g.ask.cores > 0 || has_static(g))
        return s->fail(PE_EUNSUPPORTED, "sharded placement with reserved cores or static ports");
    if (!s->visit_unique) return s->fail(PE_EUNSUPPORTED, "sharded placement needs a list without repeated rows");
    if (g.n_spread != (int)g.psets.size() || g.psets_dynamic)
        return s->fail(PE_EUNSUPPORTED, "sharded placement with distinct_property or cleared property values");
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi && s->tgs[k]->name == g.name)
            return s->fail(PE_EUNSUPPORTED, "sharded placement: task groups sharing a name");
    s->limit = 0x7FFFFFFF;
    const uint32_t n = (uint32_t)s->visit.size();
    pe::SweepArgs A;
    uint32_t blocks = 0;
    rc = sweep_setup(s, g, nullptr, row_begin, row_end, &A, &blocks);
    if (rc) return rc;
    // per placement: the rank's sweep merged to one record at its slot of the
    // gather buffer, nranks x 80 B exchanged, the step merges the nranks records
    const uint32_t rows_max = (uint32_t)((s->nodes.size() + (size_t)s->nranks - 1) / (size_t)s->nranks);
    blocks = std::max<uint32_t>(1, std::min<uint32_t>((rows_max + 255) / 256,
                                                      (uint32_t)s->n_cu * (uint32_t)s->sweep_per_cu_aux));
    const size_t rec_bytes = sizeof(pe::SweepRec);
    HIP_TRY(s, s->d_sweep_recs.ensure(rec_bytes * blocks));
    HIP_TRY(s, s->d_gather.ensure(rec_bytes * (size_t)s->nranks));
    HIP_TRY(s, s->d_sweep_done.ensure(sizeof(uint32_t)));
    HIP_TRY(s, hipMemsetAsync(s->d_sweep_done.p, 0, sizeof(uint32_t), s->stream));
    A.recs = s->d_sweep_recs.as<pe::SweepRec>();
    A.merged = s->d_gather.as<pe::SweepRec>() + s->rank;
    A.done = s->d_sweep_done.as<uint32_t>();
    pe::SweepArgs A2 = A;   // the step merges the gathered records
    A2.recs = s->d_gather.as<pe::SweepRec>();
    uint32_t nrecs = (uint32_t)s->nranks;
    // one rank exchanges nothing: its step merges the workgroup records itself
    // (PE_SHARD_MERGE_ONE=1 runs the per-rank merge anyway, for measurement)
    static const bool merge_one = std::getenv("PE_SHARD_MERGE_ONE") != nullptr;
    const bool local_merge = s->nranks > 1 || merge_one;
    if (!local_merge) {
        A2.recs = A.recs;
        nrecs = blocks;
    }
    HIP_TRY(s, upload_visit(s, s->visit));
    HIP_TRY(s, s->d_loop_out.ensure(sizeof(pe_ranked_node) * (size_t)(count + 1)));
    HIP_TRY(s, s->d_loop_state.ensure(8 * sizeof(uint32_t)));
    HIP_TRY(s, hipMemsetAsync(s->d_loop_state.p, 0, 8 * sizeof(uint32_t), s->stream));
    uint32_t* state = s->d_loop_state.as<uint32_t>();
    uint32_t h_state[5] = {0, 0, 0, 0, 0};
    const uint32_t chunk = 64;
    double x_us = 0, x_min = 1e300, x_max = 0;
    uint32_t x_n = 0;
    auto x_add = [&](double us) {
        x_us += us;
        x_min = std::min(x_min, us);
        x_max = std::max(x_max, us);
        x_n++;
    };
    const bool host_x = s->xfn != nullptr && s->nranks > 1;
    if (s->nranks > 1 && !host_x && s->ev_xs.empty()) {   // an event pair around every placement's all-gather
        s->ev_xs.resize(2 * chunk, nullptr);
        for (auto& e : s->ev_xs) HIP_TRY(s, hipEventCreate(&e));
    }
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    if (A.spread_tab) HIP_TRY(s, pe_launch_spread_table(&A.tg, s->d_spread_tab.as<double>(), s->stream));
    for (uint32_t k = 0; k < count && !h_state[0]; k += chunk) {
        const uint32_t m = std::min(chunk, count - k);
        for (uint32_t j = 0; j < m; j++) {
            if (local_merge) HIP_TRY_STATE(s, pe_launch_sweep_local(&A, blocks, s->stream));
            else HIP_TRY_STATE(s, pe_launch_sweep_only(&A, blocks, s->stream));
            if (host_x) {   // the caller's transport: record to host, all-gather, records back
                char* hb = static_cast<char*>(s->h_xbuf);
                HIP_TRY(s, hipMemcpyAsync(hb, A.merged, rec_bytes, hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(s, hipStreamSynchronize(s->stream));
                const double t0 = now_us();
                const int xr = s->xfn(s->xctx, hb, hb + rec_bytes, rec_bytes);
                x_add(now_us() - t0);
                if (xr != 0) return s->fail(PE_EHIP, "pe_comm_init_host exchange failed: " + std::to_string(xr));
                HIP_TRY(s, hipMemcpyAsync(A2.recs, hb + rec_bytes, rec_bytes * (size_t)s->nranks,
                                          hipMemcpyHostToDevice, s->stream));
            } else if (s->nranks > 1) {   // in place: this rank's record already sits at its offset
                HIP_TRY(s, hipEventRecord(s->ev_xs[2 * j], s->stream));
                const ncclResult_t r = rc_AllGather(A.merged, s->d_gather.p, rec_bytes, ncclUint8, s->comm, s->stream);
                if (r != ncclSuccess) return s->fail(PE_EHIP, std::string("ncclAllGather: ") + rc_GetErrorString(r));
                HIP_TRY(s, hipEventRecord(s->ev_xs[2 * j + 1], s->stream));
            }
            HIP_TRY_STATE(s, pe_launch_step_only(&A2, nrecs, s->d_visit.as<uint32_t>(), n, s->offset,
                                           s->d_loop_out.as<pe_ranked_node>(), state, s->stream));
        }
        HIP_TRY(s, hipMemcpyAsync(h_state, state, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        for (uint32_t j = 0; s->nranks > 1 && !host_x && j < m; j++) {   // every placement's all-gather
            float xms = 0;
            if (hipEventElapsedTime(&xms, s->ev_xs[2 * j], s->ev_xs[2 * j + 1]) != hipSuccess) continue;
            x_add(xms * 1e3);
        }
    }
    s->last_exchange_us = x_n ? x_us / x_n : 0.0;
    s->last_exchange_stats[0] = s->last_exchange_us;
    s->last_exchange_stats[1] = x_n ? x_min : 0.0;
    s->last_exchange_stats[2] = x_max;
    s->last_exchange_stats[3] = x_n;
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    const uint32_t p = h_state[1];
    const uint32_t nrec = std::min(count, p + (h_state[0] ? 1u : 0u));
    if (nrec)
        HIP_TRY(s, hipMemcpyAsync(out, s->d_loop_out.p, sizeof(pe_ranked_node) * nrec, hipMemcpyDeviceToHost,
                                  s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    for (uint32_t i = 0; i < p; i++) plan_of(s).emplace_back(g.name, (uint32_t)out[i].row);   // Plan.AppendAlloc
    invalidate_job_distinct(s, tgi);
    s->offer_row = -1;
    if (placed) *placed = p;
    return PE_OK;
}

double pe_last_exchange_us(const pe_stack* s) { return s ? s->last_exchange_us : 0.0; }

int pe_last_exchange_stats(const pe_stack* s, double* out4) {
    if (!s || !out4) return PE_EINVAL;
    for (int i = 0; i < 4; i++) out4[i] = s->last_exchange_stats[i];
    return PE_OK;
}

int pe_speculation_stats(const pe_stack* s, uint64_t* out4) {
    if (!s || !out4) return PE_EINVAL;
    view_take(const_cast<pe_stack*>(s));
    for (int i = 0; i < 4; i++) out4[i] = s->spec_stats[i];
    return PE_OK;
}

int pe_stage_orders(pe_stack* s, const uint32_t* orders, uint32_t n_evals, uint32_t n) {
    PE_FLUSH_RESET(s);
    if (!s || (!orders && n_evals && n)) return PE_EINVAL;
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    const size_t total = (size_t)n_evals * n;
    for (size_t i = 0; i < total; i++)
        if (orders[i] >= s->nodes.size()) return s->fail(PE_EINVAL, "row out of range in staged order");
    s->h_orders.assign(orders, orders + total);
    HIP_TRY(s, upload_s(s, s->d_orders, s->h_orders));
    {
        // generation-stamped duplicate check over every staged order
        std::vector<uint32_t> stamp(s->nodes.size(), 0);
        s->orders_unique = true;
        for (uint32_t e = 0; e < n_evals && s->orders_unique; e++) {
            const uint32_t* o = orders + (size_t)e * n;
            for (uint32_t i = 0; i < n; i++) {
                if (stamp[o[i]] == e + 1) { s->orders_unique = false; break; }
                stamp[o[i]] = e + 1;
            }
        }
    }
    s->staged_evals = n_evals;
    s->staged_n = n;
    return PE_OK;
}

namespace {

// Host preparation of a batch launch: fresh-memo feasibility tables, limit and
// overlay size, exactly as SetNodes(order) + Select would set them up.
int prepare_batch(pe_stack* s, uint32_t tgi, uint32_t count) {
    const uint32_t E = s->staged_evals, n = s->staged_n;
    TgPlan& g = *s->tgs[tgi];
    if (!g.unsupported.empty()) return s->fail(PE_EUNSUPPORTED, g.unsupported);
    if (!g.psets_built) {
        int rc = build_psets(s, g);
        if (rc) return rc;
        if (!g.unsupported.empty()) return s->fail(PE_EUNSUPPORTED, g.unsupported);
    }
    // Each eval is a fresh EvalContext: build the tables with an empty memo.
    const std::vector<uint32_t> order0(s->h_orders.begin(), s->h_orders.begin() + n);
    auto saved_memo = s->tg_memo;
    s->tg_memo.erase(g.name);
    g.tables_valid = false;
    int rc = build_tables(s, g, order0, 0);
    s->tg_memo = saved_memo;
    g.tables_valid = false;
    if (rc) return rc;
    // limit as SetNodes(order) + Select would set it (stack.go:83-90, 165-167)
    uint32_t lim = 2;
    if (!s->cfg.batch) lim = std::max<uint32_t>(2, (uint32_t)std::ceil(std::log2((double)n)));
    if (!g.affinities.empty() || !g.spreads.empty() || !s->job_spreads.empty()) lim = 0x7FFFFFFF;
    const uint32_t saved_limit = s->limit;
    s->limit = lim;
    pe::BatchArgs A = batch_args(s, g);
    s->limit = saved_limit;
    const bool full = !g.psets.empty() || lim >= n;
    if (full) {
        const int prc = place_pset_tables(s, A, E, s->d_pset_gb);   // kept with batch_A
        if (prc) return prc;
    }
    A.hash_bits = hash_bits_for(count, full, A.pset_lds);
    A.packed_overlay = packed_kbits(s, count, full);
    if ((1u << A.hash_bits) < 2u * count)
        return s->fail(PE_EUNSUPPORTED, "count too large for the per-eval LDS overlay in batch mode");
    if (!g.nonuniform.empty() && !g.node_ok_used) {
        // order-dependent memo outcomes: one class table per eval
        std::vector<uint8_t> tabs((size_t)E * s->ncls);
        pe::ConstraintEvaluator ev;
        for (uint32_t e = 0; e < E; e++) {
            std::vector<int8_t> memo(s->ncls, -1);
            decide_classes(s, g, ev, memo, s->h_orders.data() + (size_t)e * n, n, 0);
            auto ok = class_verdicts(s, g, memo);
            std::copy(ok.begin(), ok.end(), tabs.begin() + (size_t)e * s->ncls);
        }
        HIP_TRY(s, upload_s(s, g.class_ok_batch, tabs));
        A.tg.class_ok = g.class_ok_batch.as<uint8_t>();
        A.tg.node_feas = nullptr;
        A.class_ok_stride = s->ncls;
    }
    A.perms = s->d_orders.as<uint32_t>();
    A.perm_stride = n;
    A.n_visit = n;
    A.count = count;
    A.offset0 = 0;
    A.commit = 1;
    A.writeback = 0;
    s->batch_chain = false;
    if (!full && s->use_base && A.class_ok_stride == 0 && s->orders_unique && n <= pe_chain_max_n() && g.ask.cores == 0 &&
        A.limit <= pe_chain_max_limit()) {
        // one base pass shared by every evaluation, then k_chain (persistent grid)
        HIP_TRY(s, s->d_base.ensure(sizeof(double) * std::max<size_t>(s->nodes.size(), 1)));
        A.base = s->d_base.as<double>();
        HIP_TRY(s, s->d_base1.ensure(sizeof(double) * std::max<size_t>(s->nodes.size(), 1)));
        A.base1 = s->d_base1.as<double>();
        s->batch_chain = true;
        const size_t lds = pe_chain_lds_bytes(A.hash_bits, A.packed_overlay != 0, n);
        s->chain_grid = (uint32_t)(pe_chain_blocks_per_cu(lds) * s->n_cu);
        HIP_TRY(s, s->d_chain_vs.ensure(sizeof(double) * (size_t)pe_chain_max_n() * s->chain_grid));
        A.chain_vs = s->d_chain_vs.as<double>();
    }
    HIP_TRY(s, s->d_batch_out.ensure(sizeof(pe_placement) * (size_t)E * std::max<uint32_t>(count, 1)));
    HIP_TRY(s, s->d_batch_status.ensure(sizeof(uint32_t) * 2 * (size_t)E));
    HIP_TRY(s, s->h_batch_out.ensure(sizeof(pe_placement) * (size_t)E * std::max<uint32_t>(count, 1)));
    HIP_TRY(s, s->h_batch_status.ensure(sizeof(uint32_t) * 2 * (size_t)E));
    A.out = s->d_batch_out.as<pe_placement>();
    A.eval_status = s->d_batch_status.as<uint32_t>();
    s->batch_direct = false;
    if (!full && !s->results_via_copy) {
        // the windowed kernel streams its records into the mapped host buffer
        pe_placement* o = s->h_batch_out.dev<pe_placement>();
        uint32_t* st = s->h_batch_status.dev<uint32_t>();
        if (o && st) {
            A.out = o;
            A.eval_status = st;
            s->batch_direct = true;
        }
    }
    s->batch_A = A;
    s->batch_full = full;
    s->batch_tgi = tgi;
    s->batch_count = count;
    s->batch_gen = s->gen;
    return PE_OK;
}

}  // namespace

int pe_place_batch(pe_stack* s, uint32_t tgi, uint32_t count, pe_placement* out, uint32_t* placed) {
    PE_FLUSH_RESET(s);
    if (!s) return PE_EINVAL;
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    if (s->cfg.stack_kind != PE_STACK_GENERIC) return s->fail(PE_ESTATE, "pe_place_batch needs a generic stack");
    if (!plan_of(s).empty()) return s->fail(PE_ESTATE, "batch evaluations start from a fresh plan (pe_reset_plan)");
    if (!s->have_job || tgi >= s->tgs.size()) return s->fail(PE_ESTATE, "pe_set_job not called / bad task group");
    const auto t0 = std::chrono::steady_clock::now();
    HIP_TRY(s, hipSetDevice(s->device));
    const uint32_t E = s->staged_evals, n = s->staged_n;
    if (E == 0 || n == 0 || count == 0) {
        HIP_TRY(s, s->h_batch_out.ensure(sizeof(pe_placement) * std::max<size_t>((size_t)E * count, 1)));
        HIP_TRY(s, s->h_batch_status.ensure(sizeof(uint32_t) * 2 * std::max<uint32_t>(E, 1)));
        pe_placement* res = s->h_batch_out.as<pe_placement>();
        for (uint32_t e = 0; e < E; e++) {
            s->h_batch_status.as<uint32_t>()[2 * e] = 0;
            if (placed) placed[e] = 0;
            if (count) {
                res[(size_t)e * count].row = -1;
                res[(size_t)e * count].nodes_evaluated = 0;
                res[(size_t)e * count].final_score = 0.0;
            }
        }
        if (out && count) std::memcpy(out, res, sizeof(pe_placement) * (size_t)E * count);
        s->batch_count = count;
        s->batch_gen = 0;
        return PE_OK;
    }
    if (s->batch_gen != s->gen || s->batch_tgi != tgi || s->batch_count != count) {
        int rc = prepare_batch(s, tgi, count);
        if (rc) return rc;
    }
    const pe::BatchArgs& A = s->batch_A;
    const auto t1 = std::chrono::steady_clock::now();
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    if (s->batch_chain) HIP_TRY_STATE(s, pe_launch_chain(&A, E, s->chain_grid, s->stream));
    else HIP_TRY_STATE(s, pe_launch_place(&A, E, s->batch_full, s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    if (!s->batch_direct) {
        HIP_TRY(s, hipMemcpyAsync(s->h_batch_status.p, A.eval_status, sizeof(uint32_t) * 2 * (size_t)E,
                                  hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipMemcpyAsync(s->h_batch_out.p, A.out, sizeof(pe_placement) * (size_t)E * count,
                                  hipMemcpyDeviceToHost, s->stream));
    }
    HIP_TRY(s, hipEventRecord(s->ev2, s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0, copy_ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    HIP_TRY(s, hipEventElapsedTime(&copy_ms, s->ev1, s->ev2));
    s->last_ms = ms;
    s->last_ms_pending = false;
    const uint32_t* st = s->h_batch_status.as<uint32_t>();
    if (s->batch_chain)
        for (uint32_t e = 0; e < E; e++)
            if (st[2 * e + 1] & kChainErrFlag)
                return s->fail(PE_EINTERNAL, "k_chain: a bounds guard tripped (batch evaluation stopped)");
    if (placed)
        for (uint32_t e = 0; e < E; e++) placed[e] = st[2 * e];
    if (out) std::memcpy(out, s->h_batch_out.p, sizeof(pe_placement) * (size_t)E * count);
    const auto t2 = std::chrono::steady_clock::now();
    s->phase_ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    s->phase_ms[1] = ms;
    s->phase_ms[2] = copy_ms;
    s->phase_ms[3] = std::chrono::duration<double, std::milli>(t2 - t0).count();
    return PE_OK;
}

int pe_batch_results(const pe_stack* s, const pe_placement** out, const uint32_t** status, uint32_t* n_evals,
                     uint32_t* count) {
    if (!s) return PE_EINVAL;
    if (out) *out = s->h_batch_out.as<const pe_placement>();
    if (status) *status = s->h_batch_status.as<const uint32_t>();
    if (n_evals) *n_evals = s->staged_evals;
    if (count) *count = s->batch_count;
    return PE_OK;
}

void pe_last_phase_ms(const pe_stack* s, double* out4) {
    if (!s || !out4) return;
    for (int i = 0; i < 4; i++) out4[i] = s->phase_ms[i];
}

// SystemScheduler placements of a task group with distinct_property sets
// (scheduler_system.go:283-425; stack.go:252 DistinctPropertyIterator): the
// nodes in list order, each passing when every set's combined use of its value
// is below the allowed count, then the plain fit (decided by k_system) or, when
// it is exhausted, BinPack with evict; every placement grows the counts.
static int system_place_distinct(pe_stack* s, uint32_t tgi, TgPlan& g, double* out_score, uint8_t* out_status,
                                 uint32_t* placed) {
    std::vector<PsetDev*> ds;
    std::vector<std::vector<uint32_t>> cnt;
    for (size_t q = (size_t)g.n_spread; q < g.psets.size(); q++) {
        ds.push_back(g.psets[q].get());
        cnt.push_back(g.psets[q]->h_counts);
    }
    auto value = [&](const PsetDev* ps, uint32_t row) {
        return ps->per_node ? ps->h_val_node[row] : ps->h_val_class[s->nodes[row].cls];
    };
    std::vector<uint32_t> accepted;
    uint32_t p = 0;
    const uint32_t saved = s->limit;
    s->limit = 1;
    int rc = PE_OK;
    for (uint32_t i = 0; i < (uint32_t)s->visit.size() && rc == PE_OK; i++) {
        const uint32_t row = s->visit[i];
        if (out_status[i] == 1) continue;
        bool ok = true;
        for (size_t k = 0; k < ds.size() && ok; k++) {
            const uint32_t v = value(ds[k], row);
            ok = v != pe::kMissing && cnt[k][v] < ds[k]->allowed;
        }
        if (!ok) {
            out_status[i] = 1;
            out_score[i] = std::nan("");
            continue;
        }
        if (out_status[i] != 0) {   // exhausted: BinPack with evict on this node alone
            if (!s->cfg.preempt) continue;
            pe_ranked_node r;
            uint32_t no;
            rc = run_evict_select(s, g, std::vector<uint32_t>{row}, 0, nullptr, &r, &no);
            if (rc || r.row < 0) continue;
            s->offer_row = r.row;
            s->offers = pack_offers(&r);
            rc = commit_preempt_impl(s, tgi, r.row, preempted_list(s, 0, r), r.n_preempted);
            if (rc) continue;
            out_status[i] = 0;
            out_score[i] = r.final_score;
        } else {
            accepted.push_back(row);
        }
        for (size_t k = 0; k < ds.size(); k++) cnt[k][value(ds[k], row)]++;
        p++;
    }
    s->limit = saved;
    if (rc) return rc;
    if (!accepted.empty()) {
        HIP_TRY(s, upload_s(s, s->d_commit_rows, accepted));
        pe::NodeSoA soa = soa_of(s);
        pe::TgTables t = tables_of(g);
        pe::Ask a = ask_for(s, g);
        HIP_TRY_STATE(s, pe_launch_commit_rows(&soa, &t, &a, s->d_commit_rows.as<uint32_t>(), (uint32_t)accepted.size(),
                                         s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        for (uint32_t r : accepted) plan_of(s).emplace_back(g.name, r);
    }
    for (auto& q : g.psets) q->h_counts.clear();   // stale: the next Select rebuilds the sets
    g.psets_built = false;
    invalidate_job_distinct(s, tgi);
    *placed = p;
    return PE_OK;
}

static int system_place_impl(pe_stack* s, uint32_t tgi, double* out_score, uint8_t* out_status, uint32_t* placed) {
    // out_score and out_status both null: the results stay in the engine's
    // page-locked staging (pe_system_results), no copy into the caller's arrays
    if (!s || (!out_score) != (!out_status)) return PE_EINVAL;
    plan_settle(s);   // the staging below is overwritten
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    if (s->cfg.stack_kind != PE_STACK_SYSTEM) return s->fail(PE_ESTATE, "pe_system_place needs a system stack");
    s->gen++;
    HIP_TRY(s, hipSetDevice(s->device));
    // every node appears once (checked by SetNodes): the single-node Selects are independent
    if (!s->visit_unique) return s->fail(PE_EUNSUPPORTED, "duplicate rows in the system placement list");
    int rc;
    {
        ApiScope prof_(s, "system.prepare_tg");
        rc = prepare_tg(s, tgi, s->visit, 0);
    }
    if (rc) return rc;
    TgPlan& g = *s->tgs[tgi];
    const uint32_t n = (uint32_t)s->visit.size();
    ApiScope prof_run_(s, "system.upload+kernel+results");
    HIP_TRY(s, upload_visit(s, s->visit));
    // results: device buffers, one DMA each into page-locked staging (a kernel
    // storing into mapped host memory runs 50x slower), then copied out
    // one device block [scores | outcomes | placed], one DMA into page-locked staging
    const size_t st_off = sizeof(double) * (size_t)n;
    const size_t placed_off = st_off + (((size_t)n + 3) & ~(size_t)3);
    const size_t placed_bytes = sizeof(uint32_t) * pe::kPlacedSlots;
    HIP_TRY(s, s->d_sys_out.ensure(placed_off + placed_bytes));
    HIP_TRY(s, s->h_sys_out.ensure(placed_off + placed_bytes));
    uint8_t* dsys = s->d_sys_out.as<uint8_t>();
    HIP_TRY(s, hipMemsetAsync(dsys + placed_off, 0, placed_bytes, s->stream));
    pe::SystemArgs A;
    std::memset(&A, 0, sizeof(A));
    A.soa = soa_of(s);
    A.tg = tables_of(g);
    A.ask = ask_for(s, g);
    A.list = s->d_visit.as<uint32_t>();
    A.n_list = n;
    A.log10 = s->log10;
    A.out_score = reinterpret_cast<double*>(dsys);
    A.out_status = dsys + st_off;
    A.placed = reinterpret_cast<uint32_t*>(dsys + placed_off);
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));   // the timed device work: rank_of + k_system
    if ((uint64_t)n * 4 >= s->nodes.size()) {
        // a list covering much of the snapshot: row-order evaluation (coalesced)
        const uint32_t nn = (uint32_t)s->nodes.size();
        HIP_TRY(s, s->d_rank_of.ensure(sizeof(uint32_t) * (size_t)std::max<uint32_t>(nn, 1)));
        HIP_TRY(s, s->d_sys_res.ensure(sizeof(uint64_t) * (size_t)std::max<uint32_t>(nn, 1)));
        if (!s->rank_of_valid)   // (kept while the list is unchanged)
            HIP_TRY(s, pe_launch_rank_of(s->d_visit.as<uint32_t>(), n, s->d_rank_of.as<uint32_t>(), nn, s->stream));
        s->rank_of_valid = true;   // the same table ensure_rank_of would build
        A.rank_of = s->d_rank_of.as<uint32_t>();
        A.res = s->d_sys_res.as<uint64_t>();
        A.n_rows = nn;
    }
    // distinct_property couples the nodes through the value counts: the kernel
    // evaluates every node without it and without committing, the host then
    // walks the list in order (DistinctPropertyIterator before BinPack)
    const bool distinct = g.psets.size() > (size_t)g.n_spread;
    A.commit = distinct ? 0 : 1;
    if (distinct) A.tg.n_psets = A.tg.n_spread;
    HIP_TRY_STATE(s, pe_launch_system(&A, s->stream));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    {
        // the kernels' wait, then the DMA: measured faster than queueing the
        // DMA behind the kernels and waiting once (median 107 vs 110-150 us
        // for SetNodes + SystemPlaceView on one box, 400 calls x 3 runs each)
        ApiScope prof_k_(s, "system.kernel_sync");
        HIP_TRY(s, hipStreamSynchronize(s->stream));
    }
    {
        ApiScope prof_d_(s, "system.d2h");
        HIP_TRY(s, hipMemcpyAsync(s->h_sys_out.p, dsys, placed_off + placed_bytes, hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
    }
    uint32_t p;
    {
        ApiScope prof_c_(s, "system.copy_out");
        const uint8_t* h = s->h_sys_out.as<uint8_t>();
        p = 0;
        for (uint32_t k = 0; k < pe::kPlacedSlots; k++) {
            uint32_t v;
            std::memcpy(&v, h + placed_off + 4 * k, 4);
            p += v;
        }
        if (out_score) {
            std::memcpy(out_score, h, sizeof(double) * n);
            std::memcpy(out_status, h + st_off, n);
        } else {   // the staging arrays are the results (and the inputs of the steps below)
            out_score = reinterpret_cast<double*>(s->h_sys_out.as<uint8_t>());
            out_status = s->h_sys_out.as<uint8_t>() + st_off;
        }
        s->sys_res_n = n;
    }
    ApiScope prof_p_(s, "system.plan");
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    if (distinct) {
        rc = system_place_distinct(s, tgi, g, out_score, out_status, &p);
        if (rc) return rc;
        if (placed) *placed = p;
        uint64_t cores[4];
        if (g.ask.cores > 0)   // the host mirror of the placements' reserved cores
            for (uint32_t i = 0; i < n; i++) if (out_status[i] == 0) core_record(s, g, (int32_t)s->visit[i], true, cores);
        return PE_OK;
    }
    {
        // Plan.AppendAlloc of every placed node: written when the plan is next
        // read (plan_settle; ResetPlan drops it), from the staged outcomes when
        // the caller reads them there, else from its copy
        s->plan_defer.active = true;
        s->plan_defer.name = g.name;
        s->plan_defer.n = n;
        s->plan_defer.status = s->h_sys_out.as<uint8_t>() + st_off;
        if (s->cfg.preempt || g.ask.cores > 0) plan_settle(s);   // the steps below append / read it
        uint64_t cores[4];
        if (g.ask.cores > 0)   // the host mirror of the placements' reserved cores
            for (uint32_t i = 0; i < n; i++) if (out_status[i] == 0) core_record(s, g, (int32_t)s->visit[i], true, cores);
    }

    if (s->cfg.preempt) {
        // BinPack with evict (stack.go:267-278) on the nodes the plain fit exhausted
        std::vector<uint32_t> pos, rows;
        for (uint32_t i = 0; i < n; i++)
            if (out_status[i] == 2) { pos.push_back(i); rows.push_back(s->visit[i]); }
        if (!rows.empty()) {
            if (!s->preempt_unsupported.empty()) return s->fail(PE_EUNSUPPORTED, "preemption: " + s->preempt_unsupported);
            if (g.ask.cores > 0) return s->fail(PE_EUNSUPPORTED, "reserved cores with preemption");
            if (g.md_on)
                for (uint32_t r : rows)
                    if (md_node(s, r)) return s->fail(PE_EUNSUPPORTED, "system preemption on multi-device nodes");
            // the max_parallel penalty reads the plan's preemption counts, which
            // earlier nodes grow: then the nodes go one at a time in list order
            bool serial = false;
            for (uint32_t r : rows) {
                for (uint32_t k = s->h_node_alloc_off[r]; k < s->h_node_alloc_off[r + 1] && !serial; k++)
                    serial = s->allocs[s->h_palloc_index[k]].max_parallel > 0;
                if (serial) break;
            }
            if (serial) {
                const uint32_t saved = s->limit;
                s->limit = 1;
                for (size_t k = 0; k < rows.size(); k++) {
                    pe_ranked_node r;
                    uint32_t no;
                    rc = run_evict_select(s, g, std::vector<uint32_t>{rows[k]}, 0, nullptr, &r, &no);
                    if (rc) { s->limit = saved; return rc; }
                    if (r.row < 0) continue;
                    s->offer_row = r.row;
                    s->offers = pack_offers(&r);
                    rc = commit_preempt_impl(s, tgi, r.row, preempted_list(s, 0, r), r.n_preempted);
                    if (rc) { s->limit = saved; return rc; }
                    out_status[pos[k]] = 0;
                    out_score[pos[k]] = r.final_score;
                    p++;
                }
                s->limit = saved;
            } else {
                const uint32_t E = (uint32_t)rows.size();
                pe::PreemptArgs P = preempt_args(s, g);
                HIP_TRY(s, upload_s(s, s->d_ev_rows, rows));
                HIP_TRY(s, s->d_ev_status.ensure(E));
                HIP_TRY(s, s->d_ev_score.ensure(sizeof(double) * E));
                HIP_TRY(s, s->d_ev_masks.ensure(sizeof(uint32_t) * pe::kEvictMaxWords * E));
                HIP_TRY(s, s->d_ev_offers.ensure(sizeof(uint32_t) * E));
                HIP_TRY(s, s->d_ev_flags.ensure(16));
                HIP_TRY(s, hipMemsetAsync(s->d_ev_flags.p, 0, 16, s->stream));
                HIP_TRY(s, s->d_status.ensure(16));
                HIP_TRY(s, hipMemsetAsync(s->d_status.p, 0, 16, s->stream));
                P.visit = s->d_ev_rows.as<uint32_t>();
                P.n_visit = E;
                P.status = s->d_ev_status.as<uint8_t>();
                P.score = s->d_ev_score.as<double>();
                P.mask_out = s->d_ev_masks.as<uint32_t>();
                P.offers_out = s->d_ev_offers.as<uint32_t>();
                P.flags = s->d_ev_flags.as<uint32_t>();
                HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
                uint32_t flags = 0;
                for (;;) {   // nothing is committed before the launch that covers every node
                    HIP_TRY_STATE(s, pe_launch_evict_only(&P, s->stream));
                    HIP_TRY(s, hipMemcpyAsync(&flags, P.flags, sizeof(flags), hipMemcpyDeviceToHost, s->stream));
                    HIP_TRY(s, hipStreamSynchronize(s->stream));
                    if ((flags & pe::kEvictUnsup) || !(flags & pe::kEvictWider)) break;
                    P.mask_words = wider_words(P.mask_words);
                    if (!P.mask_words) break;
                    HIP_TRY(s, hipMemsetAsync(s->d_ev_flags.p, 0, 16, s->stream));
                }
                if (flags & pe::kEvictUnsup)
                    return s->fail(PE_EUNSUPPORTED, "preemption: a node outside the device path (several network "
                                                    "devices, reserved cores)");
                if (!P.mask_words)
                    return s->fail(PE_EUNSUPPORTED, "preemption: a node's proposed allocs exceed the widest eviction "
                                                    "width");
                HIP_TRY_STATE(s, pe_launch_commit_evicted(&P, s->d_preempted.as<uint8_t>(), s->d_pcount.as<uint32_t>(),
                                                    s->d_dev_free.as<uint32_t>(), s->d_status.as<uint32_t>(),
                                                    s->stream));
                HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
                std::vector<uint8_t> st(E);
                std::vector<double> sc(E);
                const uint32_t W = P.mask_words;
                std::vector<uint32_t> masks((size_t)W * E);
                HIP_TRY(s, hipMemcpyAsync(st.data(), P.status, E, hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(s, hipMemcpyAsync(sc.data(), P.score, sizeof(double) * E, hipMemcpyDeviceToHost, s->stream));
                HIP_TRY(s, hipMemcpyAsync(masks.data(), P.mask_out, sizeof(uint32_t) * W * E, hipMemcpyDeviceToHost,
                                          s->stream));
                HIP_TRY(s, hipStreamSynchronize(s->stream));
                float ms2 = 0;
                HIP_TRY(s, hipEventElapsedTime(&ms2, s->ev0, s->ev1));
                s->last_ms += ms2;
                s->last_ms_pending = false;
                for (uint32_t k = 0; k < E; k++) {
                    if (st[k] != 0) continue;   // exhausted / skipped nodes stay exhausted
                    out_status[pos[k]] = 0;
                    out_score[pos[k]] = sc[k];
                    plan_of(s).emplace_back(g.name, rows[k]);
                    pe_ranked_node r;   // the host mirrors of the evictions k_commit_evicted applied
                    set_preempted(s, r, k, rows[k], masks.data() + (size_t)k * W, W, true);
                    p++;
                }
            }
        }
    }
    if (placed) *placed = p;
    return PE_OK;
}

}  // extern "C"

extern "C" int pe_set_metrics(pe_stack* s, int on) {
    if (!s) return PE_EINVAL;
    view_take(s);
    {
        const int frc = spec_flush(s);
        if (frc) return frc;
    }
    if ((on != 0) != s->metrics_on) sys_deactivate(s);   // the next cache pass traces rows (or stops)
    s->metrics_on = on != 0;
    if (s->metrics_on) sys_view_withdraw(s);   // the view's outcomes carry no maps
    s->metrics_valid = false;
    return PE_OK;
}

extern "C" int64_t pe_last_metrics(const pe_stack* s, char* buf, size_t cap) {
    if (!s) return PE_EINVAL;
    pe_stack* m = const_cast<pe_stack*>(s);
    view_take(m);   // Selects the caller served from the view: the last one's maps
    if (!s->metrics_valid) return PE_ESTATE;
    if (!s->metrics_text_ok) {
        m->metrics_text.clear();
        metrics_text_into(s, s->m_counts.data(), s->m_counts.size(), s->m_scores.data(), s->m_scores.size(),
                          m->metrics_text);
        m->metrics_text_ok = true;
    }
    if (buf && cap) {
        const size_t k = std::min(cap - 1, s->metrics_text.size());
        std::memcpy(buf, s->metrics_text.data(), k);
        buf[k] = 0;
    }
    return (int64_t)s->metrics_text.size() + 1;
}

extern "C" int pe_last_metrics_bin(const pe_stack* s, const pe_metric_count** counts, uint32_t* n_counts,
                                   const pe_metric_score** scores, uint32_t* n_scores) {
    if (!s || !counts || !n_counts || !scores || !n_scores) return PE_EINVAL;
    view_take(const_cast<pe_stack*>(s));
    if (!s->metrics_valid) return PE_ESTATE;
    *counts = s->m_counts.data();
    *n_counts = (uint32_t)s->m_counts.size();
    *scores = s->m_scores.data();
    *n_scores = (uint32_t)s->m_scores.size();
    return PE_OK;
}

extern "C" int64_t pe_metric_string(const pe_stack* s, uint32_t key, char* buf, size_t cap) {
    if (!s) return PE_EINVAL;
    if ((key & PE_METRIC_ENGINE_KEY) ? (key & ~PE_METRIC_ENGINE_KEY) >= s->mstrs.size() : key >= s->strs.size())
        return PE_EINVAL;
    const std::string& t = metric_string(s, key);
    if (buf && cap) {
        const size_t k = std::min(cap - 1, t.size());
        std::memcpy(buf, t.data(), k);
        buf[k] = 0;
    }
    return (int64_t)t.size() + 1;
}

extern "C" const char* pe_scorer_name(uint32_t scorer) { return scorer < 7 ? kScorerNames[scorer] : ""; }

// ---- wrappers that log the chain's visits for EvalEligibility -----------------

static int system_place_one(pe_stack* s, uint32_t tgi, double* out_score, uint8_t* out_status, uint32_t* placed) {
    const int rc = system_place_impl(s, tgi, out_score, out_status, placed);
    if (s) sys_deactivate(s);   // rows committed on the device: the per-row cache is stale
    // one single-node Select per row of the list (scheduler_system.go:290-422)
    if (rc == PE_OK) elig_log_span(s, tgi, 0, (uint32_t)s->visit.size());
    return rc;
}

int pe_system_results(const pe_stack* s, const double** score, const uint8_t** status, uint32_t* n) {
    if (!s || !score || !status || !n) return PE_EINVAL;
    if (!s->h_sys_out.p || !s->sys_res_n) return PE_ESTATE;
    const size_t st_off = sizeof(double) * (size_t)s->sys_res_n;
    *score = reinterpret_cast<const double*>(s->h_sys_out.as<uint8_t>());
    *status = s->h_sys_out.as<uint8_t>() + st_off;
    *n = s->sys_res_n;
    return PE_OK;
}

int pe_place_sharded(pe_stack* s, uint32_t tgi, uint32_t count, uint32_t row_begin, uint32_t row_end,
                     pe_ranked_node* out, uint32_t* placed) {
    PE_FLUSH_RESET(s);
    const int rc = place_sharded_impl(s, tgi, count, row_begin, row_end, out, placed);
    if (rc == PE_OK && count) elig_log_span(s, tgi, s->offset, (uint32_t)s->visit.size());   // full passes
    return rc;
}

int pe_get_eligibility(pe_stack* s, uint32_t changed_only, pe_class_feas* out, uint32_t cap, uint32_t* n_out,
                       uint32_t* flags) {
    PE_FLUSH_RESET(s);
    if (!s || !n_out) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    elig_resolve(s);
    elig_size(s);
    if (s->cls_str.size() != s->ncls) {
        s->cls_str.assign(s->ncls, PE_NONE);
        for (const auto& kv : s->cls_of)
            if (kv.second < s->ncls) s->cls_str[kv.second] = kv.first;
    }
    std::vector<pe_class_feas> ents;
    auto push = [&](uint32_t map, uint32_t c, int8_t v) {
        if (v < 0) return;
        ents.push_back(pe_class_feas{map, s->cls_str[c], v ? (uint32_t)PE_CLASS_ELIGIBLE : (uint32_t)PE_CLASS_INELIGIBLE});
    };
    if (changed_only) {
        std::sort(s->ex_dirty.begin(), s->ex_dirty.end());
        s->ex_dirty.erase(std::unique(s->ex_dirty.begin(), s->ex_dirty.end()), s->ex_dirty.end());
        for (const auto& d : s->ex_dirty) {
            if (d.first == PE_NONE) push(PE_NONE, d.second, s->ex_job[d.second]);
            else push(d.first, d.second, s->ex_tg[d.first].st[d.second]);
        }
    } else {
        for (uint32_t c = 0; c < s->ncls; c++) push(PE_NONE, c, s->ex_job[c]);
        for (const auto& kv : s->ex_tg)
            for (uint32_t c = 0; c < (uint32_t)kv.second.st.size(); c++) push(kv.first, c, kv.second.st[c]);
    }
    *n_out = (uint32_t)ents.size();
    if (out && cap) std::memcpy(out, ents.data(), sizeof(pe_class_feas) * std::min<size_t>(cap, ents.size()));
    if (ents.size() <= cap) s->ex_dirty.clear();
    if (flags) {
        bool esc = s->job_escaped;   // HasEscaped (context.go:237-251)
        for (const auto& kv : s->ex_tg_escaped) esc = esc || kv.second;
        *flags = esc ? PE_ELIG_ESCAPED : 0u;
    }
    return PE_OK;
}

int pe_put_eligibility(pe_stack* s, const pe_class_feas* in, uint32_t n) {
    PE_FLUSH_RESET(s);
    if (!s || (!in && n)) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    int rc = spec_flush(s);
    if (rc) return rc;
    s->gen++;
    elig_resolve(s);
    elig_size(s);
    if (s->job_memo.size() != s->ncls) s->job_memo.assign(s->ncls, -1);
    if (s->ref_job_memo.size() != s->ncls) s->ref_job_memo.assign(s->ncls, -1);
    bool changed = false;
    for (uint32_t i = 0; i < n; i++) {
        const auto it = s->cls_of.find(in[i].computed_class);
        if (it == s->cls_of.end() || it->second >= s->ncls) continue;   // a class without nodes here
        const uint32_t c = it->second;
        if (in[i].status != PE_CLASS_ELIGIBLE && in[i].status != PE_CLASS_INELIGIBLE) continue;
        const int8_t v = in[i].status == PE_CLASS_ELIGIBLE ? 1 : 0;
        if (in[i].task_group == PE_NONE) {
            s->ex_job[c] = v;
            if (!s->ex_job_seen[c]) { s->ex_job_seen[c] = 1; s->ex_job_unseen--; }
            if (s->job_memo[c] != v) { s->job_memo[c] = v; changed = true; }
            s->ref_job_memo[c] = v;
        } else {
            const uint32_t name = in[i].task_group;
            pe_stack::ExTg& e = elig_tg(s, name);
            e.st[c] = v;
            if (!e.seen[c]) { e.seen[c] = 1; e.unseen--; }
            auto& memo = s->tg_memo[name];
            if (memo.size() != s->ncls) memo.assign(s->ncls, -1);
            if (memo[c] != v) { memo[c] = v; changed = true; }
            auto& rt = s->ref_tg_memo[name];
            if (rt.size() != s->ncls) rt.assign(s->ncls, -1);
            rt[c] = v;
        }
    }
    if (changed) {
        invalidate_tables(s);
        sys_deactivate(s);   // class verdicts changed under the per-row cache
    }
    return PE_OK;
}

pe_spec_view* pe_spec_view_get(pe_stack* s) { return s ? &s->sview : nullptr; }
pe_system_view* pe_system_view_get(pe_stack* s) { return s ? &s->sysview : nullptr; }

int pe_get_cursor(const pe_stack* s, uint32_t* offset, uint32_t* limit) {
    if (!s) return PE_EINVAL;
    view_take(const_cast<pe_stack*>(s));   // Selects the caller served from the view moved the cursor
    if (offset) *offset = s->offset;
    if (limit) *limit = s->limit;
    return PE_OK;
}

int pe_set_cursor(pe_stack* s, uint32_t tgi, uint32_t offset, uint32_t limit) {
    PE_FLUSH_RESET(s);
    if (!s) return PE_EINVAL;
    if (!s->have_state) return s->fail(PE_ESTATE, "pe_set_state not called");
    if (!s->visit.empty() && offset >= s->visit.size()) return s->fail(PE_EINVAL, "cursor beyond the SetNodes list");
    int rc = spec_flush(s);
    if (rc) return rc;
    s->gen++;
    elig_resolve(s);   // windows before the Go chain's Select, in order
    s->offset = s->visit.empty() ? 0 : offset;
    s->limit = limit;
    if (tgi != PE_NONE) {
        if (!s->have_job || tgi >= s->tgs.size()) return s->fail(PE_EINVAL, "task group index out of range");
        // the Go chain's SpreadIterator.SetTaskGroup ran for this group (spread.go:76-104)
        TgPlan& g = *s->tgs[tgi];
        if (s->cfg.stack_kind == PE_STACK_GENERIC && !s->spread_info_done.count(g.name)) {
            s->spread_info_done.insert(g.name);
            for (auto& sp : g.spreads) s->sum_spread_weights += (int32_t)(int8_t)sp.weight;
            for (auto& sp : s->job_spreads) s->sum_spread_weights += (int32_t)(int8_t)sp.weight;
            for (auto& o : s->tgs) o->psets_built = false;   // every spread weight is over the new sum
        }
    }
    invalidate_tables(s);
    return PE_OK;
}

int pe_flush(pe_stack* s) {
    PE_FLUSH_RESET(s);
    if (!s) return PE_EINVAL;
    return spec_flush(s);
}

int pe_system_spec_stats(const pe_stack* s, uint64_t* out2) {
    if (!s || !out2) return PE_EINVAL;
    out2[0] = s->sys.passes;
    out2[1] = s->sys.served;
    return PE_OK;
}

// ---- one handle over several devices (pe_config.device_count) ---------------

static void kid_log(pe_stack* s, uint8_t kind, uint32_t tgi, int32_t row, const uint32_t* a, uint32_t n) {
    if (s->kids.empty() || !s->kids_valid) return;
    s->replay.push_back(pe_stack::ReplayOp{kind, tgi, row, std::vector<uint32_t>(a, a + n)});
}

// The kids take the plan mutations logged since the last sync, in order, and
// the root's iterator state: they then hold exactly the root's plan.
static int kids_sync(pe_stack* s) {
    if (s->kids.empty()) return PE_OK;
    if (!s->kids_valid) return PE_EUNSUPPORTED;
    for (pe_stack* k : s->kids) {
        int rc = PE_OK;
        if (k->visit != s->visit) rc = pe_set_nodes(k, s->visit.data(), (uint32_t)s->visit.size(), nullptr);
        for (size_t i = 0; i < s->replay.size() && rc == PE_OK; i++) {
            const pe_stack::ReplayOp& op = s->replay[i];
            switch (op.kind) {
                case 0: rc = commit_one(k, op.tgi, op.row); break;
                case 1: rc = commit_preempt_one(k, op.tgi, op.row, op.a.data(), (uint32_t)op.a.size()); break;
                case 2: rc = plan_stop_one(k, op.a.data(), (uint32_t)op.a.size()); break;
                default: rc = plan_pop_update_one(k, op.a[0]); break;
            }
        }
        if (rc == PE_OK) rc = spec_flush(k);
        if (rc) {
            s->kids_valid = false;
            s->replay.clear();
            return PE_EUNSUPPORTED;
        }
        k->offset = s->offset;
        k->limit = s->limit;
        k->tg_memo = s->tg_memo;
        k->job_memo = s->job_memo;
        if (k->spread_info_done != s->spread_info_done || k->sum_spread_weights != s->sum_spread_weights) {
            k->spread_info_done = s->spread_info_done;
            k->sum_spread_weights = s->sum_spread_weights;
            for (auto& g : k->tgs) g->psets_built = false;
        }
        invalidate_tables(k);
    }
    s->replay.clear();
    return PE_OK;
}

// After a call that starts a new evaluation context on every replica.
static void kids_fresh(pe_stack* s, bool all_ok) {
    s->replay.clear();
    s->kids_valid = all_ok;
}

// The full-pass count loop split over the handle's devices: rows
// [n k / N, n (k+1) / N) on replica k, per placement one k_sweep per replica
// whose last workgroup merges the replica's records into one (at slot k of
// its gather buffer), the N records exchanged (ncclAllGather over the group's
// communicators, or device copies in loopback), then every replica's
// k_sweep_step merges the N records and commits the same winner. The
// exchange is timed on every placement (events on the root's stream).
static int multi_place(pe_stack* s, uint32_t tgi, uint32_t count, pe_ranked_node* out, uint32_t* placed) {
    std::vector<pe_stack*> st{s};
    st.insert(st.end(), s->kids.begin(), s->kids.end());
    const uint32_t N = (uint32_t)st.size();
    const uint32_t n = (uint32_t)s->visit.size(), nn = (uint32_t)s->nodes.size();
    std::vector<pe::SweepArgs> A(N), A2(N);
    const uint32_t rows_max = (nn + N - 1) / N;
    const uint32_t blocks = std::max<uint32_t>(
        1, std::min<uint32_t>((rows_max + 255) / 256, (uint32_t)s->n_cu * (uint32_t)s->sweep_per_cu_aux));
    const size_t rec_bytes = sizeof(pe::SweepRec);
    auto strm = [&](uint32_t k) { return s->loopback ? s->stream : st[k]->stream; };
    for (uint32_t k = 0; k < N; k++) {
        pe_stack* x = st[k];
        HIP_TRY(s, hipSetDevice(x->device));
        int rc = flush_counts(x);   // the launches below check the root's pending state only
        if (!rc && x->reset_pending) rc = flush_reset(x);
        if (rc) return k ? s->fail(rc, "replica: " + x->err) : rc;
        rc = prepare_tg(x, tgi, x->visit, x->offset);
        if (rc) return k ? s->fail(rc, "replica: " + x->err) : rc;
        x->limit = 0x7FFFFFFF;
        uint32_t b_unused = 0;
        rc = sweep_setup(x, *x->tgs[tgi], nullptr, (uint32_t)((uint64_t)nn * k / N),
                         (uint32_t)((uint64_t)nn * (k + 1) / N), &A[k], &b_unused);
        if (rc) return k ? s->fail(rc, "replica: " + x->err) : rc;
        HIP_TRY(s, x->d_sweep_recs.ensure(rec_bytes * blocks));
        HIP_TRY(s, x->d_gather.ensure(rec_bytes * N));
        HIP_TRY(s, x->d_sweep_done.ensure(sizeof(uint32_t)));
        A[k].recs = x->d_sweep_recs.as<pe::SweepRec>();
        A[k].merged = x->d_gather.as<pe::SweepRec>() + k;
        A[k].done = x->d_sweep_done.as<uint32_t>();
        A2[k] = A[k];
        A2[k].recs = x->d_gather.as<pe::SweepRec>();
        HIP_TRY(s, upload_visit(x, x->visit));
        HIP_TRY(s, x->d_loop_out.ensure(sizeof(pe_ranked_node) * (size_t)(count + 1)));
        HIP_TRY(s, x->d_loop_state.ensure(8 * sizeof(uint32_t)));
        HIP_TRY(s, hipStreamSynchronize(x->stream));   // uploads on the replica's own stream
        HIP_TRY(s, hipMemsetAsync(x->d_loop_state.p, 0, 8 * sizeof(uint32_t), strm(k)));
        HIP_TRY(s, hipMemsetAsync(x->d_sweep_done.p, 0, sizeof(uint32_t), strm(k)));
        if (A[k].spread_tab) HIP_TRY(s, pe_launch_spread_table(&A[k].tg, x->d_spread_tab.as<double>(), strm(k)));
    }
    uint32_t h_state[5] = {0, 0, 0, 0, 0};
    const uint32_t chunk = 64;
    double x_us = 0, x_min = 1e300, x_max = 0;
    uint32_t x_n = 0;
    HIP_TRY(s, hipSetDevice(s->device));
    if (s->ev_xs.empty()) {   // an event pair around every placement's exchange
        s->ev_xs.resize(2 * chunk, nullptr);
        for (auto& e : s->ev_xs) HIP_TRY(s, hipEventCreate(&e));
    }
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    for (uint32_t p0 = 0; p0 < count && !h_state[0]; p0 += chunk) {
        const uint32_t m = std::min(chunk, count - p0);
        for (uint32_t j = 0; j < m; j++) {
            for (uint32_t k = 0; k < N; k++) {
                HIP_TRY(s, hipSetDevice(st[k]->device));
                HIP_TRY_STATE(s, pe_launch_sweep_local(&A[k], blocks, strm(k)));
            }
            HIP_TRY(s, hipSetDevice(s->device));
            HIP_TRY(s, hipEventRecord(s->ev_xs[2 * j], s->stream));
            if (s->loopback) {
                // every replica's record into every other replica's gather buffer
                for (uint32_t k = 0; k < N; k++)
                    for (uint32_t e = 0; e < N; e++)
                        if (e != k)
                            HIP_TRY(s, hipMemcpyAsync(st[k]->d_gather.as<pe::SweepRec>() + e,
                                                      st[e]->d_gather.as<pe::SweepRec>() + e, rec_bytes,
                                                      hipMemcpyDeviceToDevice, s->stream));
            } else {
                ncclResult_t r = rc_GroupStart();
                for (uint32_t k = 0; k < N && r == ncclSuccess; k++)
                    r = rc_AllGather(A[k].merged, st[k]->d_gather.p, rec_bytes, ncclUint8, s->group_comms[k],
                                     st[k]->stream);
                const ncclResult_t r2 = rc_GroupEnd();
                if (r != ncclSuccess || r2 != ncclSuccess)
                    return s->fail(PE_EHIP, std::string("ncclAllGather: ") + rc_GetErrorString(r != ncclSuccess ? r : r2));
            }
            HIP_TRY(s, hipEventRecord(s->ev_xs[2 * j + 1], s->stream));
            for (uint32_t k = 0; k < N; k++) {
                HIP_TRY(s, hipSetDevice(st[k]->device));
                HIP_TRY_STATE(s, pe_launch_step_only(&A2[k], N, st[k]->d_visit.as<uint32_t>(), n, st[k]->offset,
                                               st[k]->d_loop_out.as<pe_ranked_node>(),
                                               st[k]->d_loop_state.as<uint32_t>(), strm(k)));
            }
        }
        HIP_TRY(s, hipSetDevice(s->device));
        HIP_TRY(s, hipMemcpyAsync(h_state, s->d_loop_state.p, sizeof(h_state), hipMemcpyDeviceToHost, s->stream));
        HIP_TRY(s, hipStreamSynchronize(s->stream));
        for (uint32_t j = 0; j < m; j++) {   // every placement's exchange
            float xms = 0;
            if (hipEventElapsedTime(&xms, s->ev_xs[2 * j], s->ev_xs[2 * j + 1]) != hipSuccess) continue;
            const double us = xms * 1e3;
            x_us += us;
            x_min = std::min(x_min, us);
            x_max = std::max(x_max, us);
            x_n++;
        }
    }
    s->last_exchange_stats[0] = x_n ? x_us / x_n : 0.0;
    s->last_exchange_stats[1] = x_n ? x_min : 0.0;
    s->last_exchange_stats[2] = x_max;
    s->last_exchange_stats[3] = x_n;
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    for (uint32_t k = 1; k < N; k++) {
        HIP_TRY(s, hipSetDevice(st[k]->device));
        HIP_TRY(s, hipStreamSynchronize(strm(k)));
    }
    HIP_TRY(s, hipSetDevice(s->device));
    s->last_exchange_us = s->last_exchange_stats[0];
    const uint32_t p = h_state[1];
    const uint32_t nrec = std::min(count, p + (h_state[0] ? 1u : 0u));
    if (nrec)
        HIP_TRY(s, hipMemcpyAsync(out, s->d_loop_out.p, sizeof(pe_ranked_node) * nrec, hipMemcpyDeviceToHost,
                                  s->stream));
    HIP_TRY(s, hipStreamSynchronize(s->stream));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    for (pe_stack* x : st) {
        for (uint32_t i = 0; i < p; i++) plan_of(x).emplace_back(x->tgs[tgi]->name, (uint32_t)out[i].row);
        invalidate_job_distinct(x, tgi);
        x->offer_row = -1;
        x->gen++;
    }
    elig_log_span(s, tgi, s->offset, n);   // full passes
    if (placed) *placed = p;
    return PE_OK;
}

// Whether tgi's count loop can run split over the replicas (as pe_place_sharded).
static bool multi_place_ok(pe_stack* s, uint32_t tgi, uint32_t count) {
    if (s->kids.empty() || !s->kids_valid || !count || s->cfg.stack_kind != PE_STACK_GENERIC || s->metrics_on)
        return false;
    if (prepare_tg(s, tgi, s->visit, s->offset) != PE_OK) { s->err.clear(); return false; }
    TgPlan& g = *s->tgs[tgi];
    if (!tg_full_scan(s, g) || g.ask.cores > 0 || has_static(g) || !s->visit_unique) return false;
    if (g.n_spread != (int)g.psets.size() || g.psets_dynamic || s->cfg.preempt) return false;
    for (size_t k = 0; k < s->tgs.size(); k++)
        if (k != tgi && s->tgs[k]->name == g.name) return false;
    return s->visit.size() >= 2 * (s->kids.size() + 1);
}

// pe_system_place split over the replicas: contiguous ranges of the list, each
// evaluated and committed by its replica; then every replica commits the
// others' placements, so all of them hold the same plan.
static int multi_system_place(pe_stack* s, uint32_t tgi, double* out_score, uint8_t* out_status, uint32_t* placed) {
    std::vector<pe_stack*> st{s};
    st.insert(st.end(), s->kids.begin(), s->kids.end());
    const uint32_t N = (uint32_t)st.size(), n = (uint32_t)s->visit.size();
    std::vector<uint32_t> lo(N), hi(N);
    for (uint32_t k = 0; k < N; k++) {
        lo[k] = (uint32_t)((uint64_t)n * k / N);
        hi[k] = (uint32_t)((uint64_t)n * (k + 1) / N);
    }
    HIP_TRY(s, hipEventRecord(s->ev0, s->stream));
    for (uint32_t k = 0; k < N; k++) {
        pe_stack* x = st[k];
        HIP_TRY(s, hipSetDevice(x->device));
        int rc = flush_counts(x);   // the launches below check the root's pending state only
        if (!rc && x->reset_pending) rc = flush_reset(x);
        if (rc) return k ? s->fail(rc, "replica: " + x->err) : rc;
        rc = prepare_tg(x, tgi, x->visit, 0);
        if (rc) return k ? s->fail(rc, "replica: " + x->err) : rc;
        TgPlan& g = *x->tgs[tgi];
        HIP_TRY(s, upload_visit(x, x->visit));
        const uint32_t m = hi[k] - lo[k];
        const size_t st_off = sizeof(double) * (size_t)m;
        const size_t bytes = st_off + (((size_t)m + 3) & ~(size_t)3) + 4;
        HIP_TRY(s, x->d_sys_out.ensure(bytes));
        HIP_TRY(s, x->h_sys_out.ensure(bytes));
        uint8_t* dsys = x->d_sys_out.as<uint8_t>();
        HIP_TRY(s, hipMemsetAsync(dsys + bytes - 4, 0, 4, x->stream));
        pe::SystemArgs Sa;
        std::memset(&Sa, 0, sizeof(Sa));
        Sa.soa = soa_of(x);
        Sa.tg = tables_of(g);
        Sa.ask = ask_for(x, g);
        Sa.list = x->d_visit.as<uint32_t>() + lo[k];
        Sa.n_list = m;
        Sa.log10 = x->log10;
        Sa.out_score = reinterpret_cast<double*>(dsys);
        Sa.out_status = dsys + st_off;
        Sa.placed = nullptr;   // counted from the outcomes below
        Sa.commit = 1;
        if (m) HIP_TRY_STATE(s, pe_launch_system(&Sa, x->stream));
        HIP_TRY(s, hipMemcpyAsync(x->h_sys_out.p, dsys, bytes, hipMemcpyDeviceToHost, x->stream));
    }
    std::vector<std::vector<uint32_t>> rows(N);
    uint32_t p = 0;
    for (uint32_t k = 0; k < N; k++) {
        pe_stack* x = st[k];
        HIP_TRY(s, hipSetDevice(x->device));
        HIP_TRY(s, hipStreamSynchronize(x->stream));
        const uint32_t m = hi[k] - lo[k];
        const uint8_t* h = x->h_sys_out.as<uint8_t>();
        const size_t st_off = sizeof(double) * (size_t)m;
        std::memcpy(out_score + lo[k], h, sizeof(double) * m);
        std::memcpy(out_status + lo[k], h + st_off, m);
        for (uint32_t i = 0; i < m; i++)
            if (out_status[lo[k] + i] == 0) rows[k].push_back(s->visit[lo[k] + i]);
        p += (uint32_t)rows[k].size();
    }
    // every replica commits the other ranges' placements
    for (uint32_t k = 0; k < N; k++) {
        pe_stack* x = st[k];
        std::vector<uint32_t> others;
        for (uint32_t e = 0; e < N; e++)
            if (e != k) others.insert(others.end(), rows[e].begin(), rows[e].end());
        HIP_TRY(s, hipSetDevice(x->device));
        if (!others.empty()) {
            TgPlan& g = *x->tgs[tgi];
            HIP_TRY(s, upload_s(x, x->d_commit_rows, others));
            pe::NodeSoA soa = soa_of(x);
            pe::TgTables t = tables_of(g);
            pe::Ask a = ask_for(x, g);
            HIP_TRY_STATE(s, pe_launch_commit_rows(&soa, &t, &a, x->d_commit_rows.as<uint32_t>(), (uint32_t)others.size(),
                                             x->stream));
        }
    }
    for (uint32_t k = 0; k < N; k++) {
        pe_stack* x = st[k];
        HIP_TRY(s, hipSetDevice(x->device));
        HIP_TRY(s, hipStreamSynchronize(x->stream));
        for (uint32_t e = 0; e < N; e++)
            for (uint32_t r : rows[e]) plan_of(x).emplace_back(x->tgs[tgi]->name, r);   // list order
        sys_deactivate(x);
        x->gen++;
    }
    HIP_TRY(s, hipSetDevice(s->device));
    HIP_TRY(s, hipEventRecord(s->ev1, s->stream));
    HIP_TRY(s, hipEventSynchronize(s->ev1));
    float ms = 0;
    HIP_TRY(s, hipEventElapsedTime(&ms, s->ev0, s->ev1));
    s->last_ms = ms;
    s->last_ms_pending = false;
    elig_log_span(s, tgi, 0, n);
    if (placed) *placed = p;
    return PE_OK;
}

static bool multi_system_ok(pe_stack* s, uint32_t tgi) {
    if (s->kids.empty() || !s->kids_valid || s->cfg.stack_kind != PE_STACK_SYSTEM || s->cfg.preempt) return false;
    if (!s->visit_unique || s->visit.size() < s->kids.size() + 1) return false;
    if (prepare_tg(s, tgi, s->visit, 0) != PE_OK) { s->err.clear(); return false; }
    TgPlan& g = *s->tgs[tgi];
    return g.psets.size() == (size_t)g.n_spread && g.ask.cores == 0;
}

int pe_set_state(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes, const pe_alloc_table* allocs) {
    PE_FLUSH_RESET(s);
    const int rc = set_state_one(s, strs, nodes, allocs);
    if (rc || !s || s->kids.empty()) return rc;
    bool ok = true;
    for (pe_stack* k : s->kids) ok = set_state_one(k, strs, nodes, allocs) == PE_OK && ok;
    kids_fresh(s, ok);
    return rc;
}

int pe_update_allocs(pe_stack* s, const pe_strtab* strs, const pe_alloc_table* allocs, const uint32_t* index) {
    PE_FLUSH_RESET(s);
    const int rc = update_allocs_one(s, strs, allocs, index);
    if (rc || !s || s->kids.empty()) return rc;
    bool ok = true;
    for (pe_stack* k : s->kids) ok = update_allocs_one(k, strs, allocs, index) == PE_OK && ok;
    kids_fresh(s, ok);
    return rc;
}

int pe_update_nodes(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes, const uint32_t* index) {
    PE_FLUSH_RESET(s);
    const int rc = update_nodes_one(s, strs, nodes, index);
    if (rc || !s || s->kids.empty()) return rc;
    bool ok = true;
    for (pe_stack* k : s->kids) ok = update_nodes_one(k, strs, nodes, index) == PE_OK && ok;
    kids_fresh(s, ok);
    return rc;
}

int pe_reset_plan(pe_stack* s) {
    const int rc = reset_plan_one(s, s && s->kids.empty());
    if (rc || !s || s->kids.empty()) return rc;
    bool ok = true;
    for (pe_stack* k : s->kids) ok = reset_plan_one(k, false) == PE_OK && ok;
    kids_fresh(s, ok);
    return rc;
}

int pe_set_job(pe_stack* s, const pe_strtab* strs, const pe_job* j) {
    if (s && !s->kids.empty()) (void)kids_sync(s);   // the logged commits name the current job's groups
    const int rc = set_job_one(s, strs, j);
    if (rc || !s || s->kids.empty() || !s->kids_valid) return rc;
    for (pe_stack* k : s->kids)
        if (set_job_one(k, strs, j) != PE_OK) s->kids_valid = false;
    return rc;
}

int pe_commit(pe_stack* s, uint32_t tgi, int32_t row) {
    PE_FLUSH_RESET(s);
    const int rc = commit_one(s, tgi, row);
    if (rc == PE_OK && !s->kids.empty()) kid_log(s, 0, tgi, row, nullptr, 0);
    return rc;
}

int pe_commit_preempt(pe_stack* s, uint32_t tgi, int32_t row, const uint32_t* preempted, uint32_t n_preempted) {
    PE_FLUSH_RESET(s);
    const int rc = commit_preempt_one(s, tgi, row, preempted, n_preempted);
    if (rc == PE_OK && !s->kids.empty()) kid_log(s, 1, tgi, row, preempted, n_preempted);
    return rc;
}

int pe_plan_stop(pe_stack* s, const uint32_t* allocs, uint32_t n) {
    PE_FLUSH_RESET(s);
    const int rc = plan_stop_one(s, allocs, n);
    if (rc == PE_OK && !s->kids.empty()) kid_log(s, 2, 0, 0, allocs, n);
    return rc;
}

int pe_plan_pop_update(pe_stack* s, uint32_t alloc) {
    PE_FLUSH_RESET(s);
    const int rc = plan_pop_update_one(s, alloc);
    if (rc == PE_OK && !s->kids.empty()) kid_log(s, 3, 0, 0, &alloc, 1);
    return rc;
}

int pe_place(pe_stack* s, uint32_t tgi, uint32_t count, pe_ranked_node* out, uint32_t* placed) {
    PE_FLUSH_RESET(s);
    if (!s) return PE_EINVAL;
    s->pre_overflow.clear();
    if (!s->kids.empty() && s->kids_valid) {
        int rc = spec_flush(s);
        if (rc) return rc;
        if (multi_place_ok(s, tgi, count) && kids_sync(s) == PE_OK) {
            s->gen++;
            rc = multi_place(s, tgi, count, out, placed);
            if (rc) s->kids_valid = false;
            return rc;
        }
    }
    uint32_t p = 0;
    const int rc = place_one(s, tgi, count, out, &p);
    if (placed) *placed = p;
    if (rc == PE_OK && !s->kids.empty())   // the placements, as the caller's commits would replay them
        for (uint32_t k = 0; k < p && k < count; k++)
            kid_log(s, 1, tgi, out[k].row, preempted_list(s, k, out[k]), out[k].n_preempted);
    return rc;
}

int pe_preempted_of(const pe_stack* s, uint32_t record, uint32_t* out, uint32_t cap) {
    if (!s) return PE_EINVAL;
    for (auto& e : s->pre_overflow)
        if (e.first == record) {
            const uint32_t k = std::min<uint32_t>(cap, (uint32_t)e.second.size());
            if (k && !out) return PE_EINVAL;
            if (k) std::memcpy(out, e.second.data(), sizeof(uint32_t) * k);
            return (int)e.second.size();
        }
    return PE_ESTATE;
}

int pe_system_place(pe_stack* s, uint32_t tgi, double* out_score, uint8_t* out_status, uint32_t* placed) {
    PE_FLUSH_RESET(s);
    if (!s || (!out_score) != (!out_status)) return PE_EINVAL;
    s->pre_overflow.clear();
    if (!s->kids.empty() && s->kids_valid && out_score) {   // (the staged-results form runs on the root)
        int rc = spec_flush(s);
        if (rc) return rc;
        if (multi_system_ok(s, tgi) && kids_sync(s) == PE_OK) {
            s->gen++;
            rc = multi_system_place(s, tgi, out_score, out_status, placed);
            if (rc) s->kids_valid = false;
            return rc;
        }
    }
    const int rc = system_place_one(s, tgi, out_score, out_status, placed);
    if (!s->kids.empty()) s->kids_valid = false;   // evictions / distinct_property: not replayable
    return rc;
}

uint32_t pe_device_count(const pe_stack* s) { return s ? (uint32_t)s->kids.size() + 1u : 0u; }
