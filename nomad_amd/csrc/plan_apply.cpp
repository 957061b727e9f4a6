// Host side of the plan applier fit check (include/nomad_pe.h, pe_planner_*).
//
// Reference: evaluatePlanPlacements / evaluateNodePlan (nomad/plan_apply.go:439-674),
// AllocsFit (nomad/structs/funcs.go:148-211), NetworkIndex.SetNode and the
// reserved-port helpers (nomad/structs/network.go:92-141, 196-296),
// ParsePortRanges (funcs.go:495-548), DeviceAccounter (nomad/structs/devices.go:22-101).
//
// The host does string work only: interning, ParsePortRanges, the node-side
// SetNode emulation (its collide flag and the reserved (IP, port) set), and the
// flattening of allocs into 32-byte records plus 64-bit keys. Every fit
// decision is made by k_plan_eval on the device (plan_kernels.hip).
#include <chrono>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/nomad_pe.h"
#include "plan_types.h"

hipError_t pe_launch_plan_eval(const pa::PlanArgs* a, int group, hipStream_t st);
hipError_t pe_launch_plan_stage_copy(const void* host_mapped, void* dst, uint64_t bytes, hipStream_t st);
hipError_t pe_launch_plan_patch(pa::NodeRec* nodes, pa::AllocRec* pool, const uint32_t* dead, uint32_t n_dead,
                                const uint32_t* rows, const pa::NodeRec* recs, uint32_t n_rows, hipStream_t st);

namespace {

constexpr uint64_t kMaxValidPort = 65536;   // network.go:22

struct DBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~DBuf() { if (p) (void)hipFree(p); }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(bytes + bytes / 4, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
};

// ParsePortRanges (funcs.go:495-548). Returns false on a parse error. Ports are
// returned ascending and deduplicated; anything >= 65536 is collapsed to a
// single 65536 entry at the end (callers only test port >= maxValidPort, and
// the reference's map order is unspecified, so ascending is one legal order).
bool parse_uint(const std::string& s, uint64_t* out) {   // strconv.ParseUint(s, 10, 0)
    if (s.empty()) return false;
    uint64_t v = 0;
    for (char c : s) {
        if (c < '0' || c > '9') return false;
        const uint64_t d = (uint64_t)(c - '0');
        if (v > (UINT64_MAX - d) / 10) return false;
        v = v * 10 + d;
    }
    *out = v;
    return true;
}

std::string trim(const std::string& s) {
    size_t b = 0, e = s.size();
    while (b < e && (s[b] == ' ' || s[b] == '\t' || s[b] == '\n' || s[b] == '\r' || s[b] == '\v' || s[b] == '\f')) b++;
    while (e > b && (s[e - 1] == ' ' || s[e - 1] == '\t' || s[e - 1] == '\n' || s[e - 1] == '\r' ||
                     s[e - 1] == '\v' || s[e - 1] == '\f')) e--;
    return s.substr(b, e - b);
}

bool parse_port_ranges(const std::string& spec, std::vector<uint32_t>* out) {
    out->clear();
    std::vector<std::string> parts;
    size_t start = 0;
    for (;;) {
        size_t c = spec.find(',', start);
        parts.push_back(spec.substr(start, c == std::string::npos ? std::string::npos : c - start));
        if (c == std::string::npos) break;
        start = c + 1;
    }
    if (parts.size() == 1 && parts[0].empty()) return true;
    std::set<uint32_t> ports;
    for (auto part : parts) {
        part = trim(part);
        std::vector<std::string> rp;
        size_t s0 = 0;
        for (;;) {
            size_t d = part.find('-', s0);
            rp.push_back(part.substr(s0, d == std::string::npos ? std::string::npos : d - s0));
            if (d == std::string::npos) break;
            s0 = d + 1;
        }
        if (rp.size() == 1) {
            uint64_t v;
            if (rp[0].empty() || !parse_uint(rp[0], &v)) return false;
            ports.insert((uint32_t)std::min<uint64_t>(v, kMaxValidPort));
        } else if (rp.size() == 2) {
            uint64_t a, b;
            if (!parse_uint(rp[0], &a) || !parse_uint(rp[1], &b)) return false;
            if (b < a) return false;
            const uint64_t hi = std::min<uint64_t>(b, kMaxValidPort);
            for (uint64_t i = std::min<uint64_t>(a, kMaxValidPort); i <= hi; i++) ports.insert((uint32_t)i);
        } else {
            return false;
        }
    }
    out->assign(ports.begin(), ports.end());
    return true;
}

struct HAlloc {
    uint32_t row;
    uint8_t terminal, bad_port;
    int64_t cpu, mem, disk;
    std::vector<uint64_t> keys;
};

// Page-locked staging for the per-call uploads: the flattening writes its
// records straight here and the copy engine reads them without the runtime's
// pageable bounce.
struct PinBuf {
    void* p = nullptr;
    size_t cap = 0;
    ~PinBuf() { if (p) (void)hipHostFree(p); }
    hipError_t reserve(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) { (void)hipHostFree(p); p = nullptr; cap = 0; }
        size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
};

// Persistent host workers for the per-call flattening (PE_PLAN_THREADS,
// default min(16, cores)). run(fn) calls fn(k) for k in [0, size()), the
// caller taking k = 0. Idle workers spin ~100 us before sleeping, so the
// phases of one call hand over without a futex wake.
class WorkerPool {
  public:
    explicit WorkerPool(int n, int spin_us) : spin_us_(spin_us) {
        for (int k = 1; k < n; k++) workers_.emplace_back([this, k] { loop(k); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            stop_.store(true);
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    int size() const { return (int)workers_.size() + 1; }
    void run(const std::function<void(int)>& fn) {
        if (workers_.empty()) { fn(0); return; }
        {
            std::lock_guard<std::mutex> g(mu_);
            job_ = &fn;
            pending_.store((int)workers_.size(), std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        fn(0);
        while (pending_.load(std::memory_order_acquire) != 0) __builtin_ia32_pause();
    }

  private:
    void loop(int k) {
        uint64_t seen = 0;
        for (;;) {
            uint64_t g;
            auto t0 = std::chrono::steady_clock::now();
            int spins = 0;
            while ((g = gen_.load(std::memory_order_acquire)) == seen && !stop_.load()) {
                __builtin_ia32_pause();
                if ((++spins & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us_)) {
                    std::unique_lock<std::mutex> l(mu_);
                    cv_.wait(l, [&] { return gen_.load() != seen || stop_.load(); });
                }
            }
            if (stop_.load()) return;
            seen = g;
            (*job_)(k);
            pending_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<bool> stop_{false};
    const std::function<void(int)>* job_ = nullptr;
    int spin_us_;
};

// Per-worker memo of DeviceIdTuple ids (allocs of neighbouring nodes repeat a
// handful of tuples); misses go to the planner's map under its lock.
struct TupleMemo {
    std::array<uint32_t, 3> key[8];
    uint32_t id[8];
    int n = 0, next = 0;
};

// One worker's share of a plan: a contiguous range of plan nodes and their
// placed allocs, keys and removals gathered locally, offsets made global in a
// second pass.
struct PlanPart {
    uint32_t n0 = 0, n1 = 0;
    std::vector<uint64_t> keys;
    std::vector<uint32_t> rm;
    std::vector<pa::BigNode> big;
    std::vector<pa::PlanRes> res;   // distinct resource triples of the part's allocs
    uint64_t scratch = 0;
    uint64_t key_base = 0, rm_base = 0, scratch_base = 0, res_base = 0;
    int rc = PE_OK, node_rc = PE_OK;
    const char* msg = nullptr;
    const char* node_msg = nullptr;
    TupleMemo memo;
};

}  // namespace

struct pe_planner {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    std::string err;
    double last_ms = 0;
    // algorithmic bytes of the last evaluate, computed on request (pe_planner_last_bytes)
    mutable uint64_t last_bytes = 0;
    mutable bool bytes_valid = true;
    // the last evaluate's plan columns, removals, plan allocs and resource
    // table (in the pinned staging, valid until the next evaluate)
    const uint32_t *last_row = nullptr, *last_poff = nullptr, *last_rmoff = nullptr, *last_rm = nullptr;
    const pa::PlanAllocRec* last_pa = nullptr;
    const pa::PlanRes* last_res = nullptr;
    uint32_t last_np = 0, last_npa = 0, last_nres = 0;
    uint64_t plan_bytes() const;
    PinBuf h_stage;   // plan node records | plan allocs | keys | removals, one region
    DBuf d_stage;
    std::vector<PlanPart> parts;
    std::unique_ptr<WorkerPool> pool_w;
    int threads = 1, spin_us = 100, copy_kernel = 0;
    WorkerPool& workers() {
        if (!pool_w) pool_w.reset(new WorkerPool(threads, spin_us));
        return *pool_w;
    }
    bool have_state = false;
    int group = 4;    // lanes per plan node in k_plan_eval (PE_PLAN_GROUP: 4 / 8 / 16 / 64; 4 measured fastest)

    std::unordered_map<std::string, uint32_t> sid;
    std::map<std::array<uint32_t, 3>, uint32_t> tuple_id;
    std::vector<uint32_t> xl;   // caller string id -> internal id (current call)

    std::vector<pa::NodeRec> nodes;
    std::vector<uint64_t> node_keys;
    std::vector<HAlloc> allocs;        // caller index order (snapshot, then committed appends)
    std::vector<uint32_t> pool_of;     // caller index -> pool index (kNone: terminal, not in the pool)
    std::vector<pa::AllocRec> pool;
    std::vector<uint64_t> pool_keys;
    std::vector<pa::Chunk> chunks;     // allocs appended by commits since the last compaction

    DBuf d_nodes, d_node_keys, d_pool, d_pool_keys, d_chunks, d_patch_dead, d_patch_rows, d_patch_recs;
    DBuf d_big, d_scratch, d_reason;

    int fail(int code, const std::string& m) { err = m; return code; }

    uint32_t intern(const std::string& s) {
        auto it = sid.find(s);
        if (it != sid.end()) return it->second;
        const uint32_t id = (uint32_t)sid.size();
        sid.emplace(s, id);
        return id;
    }
    // Caller string id -> internal id. A caller that keeps one growing table
    // (ids stable, strings appended) pays only for the new strings: the mapped
    // prefix is recognised by comparing its offsets and bytes.
    std::vector<uint32_t> xl_off;
    std::string xl_bytes;
    int map_strings(const pe_strtab* t) {
        if (!t) { xl.clear(); xl_off.clear(); xl_bytes.clear(); return PE_OK; }
        if (t->count && (!t->offsets || !t->bytes)) return fail(PE_EINVAL, "bad string table");
        size_t keep = 0;
        const size_t have = xl.size();
        if (have && t->count >= have && same_prefix(t, have)) keep = have;
        if (keep == t->count && have) return PE_OK;   // the same table as last call
        xl.resize(keep);
        xl.reserve(t->count);
        for (uint32_t i = (uint32_t)keep; i < t->count; i++)
            xl.push_back(intern(std::string(t->bytes + t->offsets[i], t->offsets[i + 1] - t->offsets[i])));
        xl_off.assign(t->offsets, t->offsets + t->count + 1);
        xl_bytes.assign(t->bytes, t->count ? t->offsets[t->count] : 0);
        if (t->count == 0) xl_off.assign(1, 0);
        return PE_OK;
    }
    // The caller's first `have` strings equal the mapped ones (offsets and
    // bytes); tables past 1 MiB are compared by the workers in slices.
    bool same_prefix(const pe_strtab* t, size_t have) {
        const size_t ob = (have + 1) * 4, bb = xl_bytes.size();
        if (t->offsets[have] != bb) return false;
        const int T = (ob + bb > (1u << 20)) ? threads : 1;
        if (T == 1) return memcmp(t->offsets, xl_off.data(), ob) == 0 && memcmp(t->bytes, xl_bytes.data(), bb) == 0;
        std::atomic<bool> same{true};
        workers().run([&](int k) {
            const size_t o0 = ob * k / T, o1 = ob * (k + 1) / T, b0 = bb * k / T, b1 = bb * (k + 1) / T;
            if (memcmp((const char*)t->offsets + o0, (const char*)xl_off.data() + o0, o1 - o0) != 0 ||
                memcmp(t->bytes + b0, xl_bytes.data() + b0, b1 - b0) != 0)
                same.store(false, std::memory_order_relaxed);
        });
        return same.load();
    }
    bool str(uint32_t caller, uint32_t* out) const {
        if (caller >= xl.size()) return false;
        *out = xl[caller];
        return true;
    }
    const std::string* text(uint32_t caller, const pe_strtab* t, std::string* tmp) const {
        if (!t || caller >= t->count) return nullptr;
        tmp->assign(t->bytes + t->offsets[caller], t->offsets[caller + 1] - t->offsets[caller]);
        return tmp;
    }
    std::mutex tuple_mu;
    TupleMemo memo;   // the single-threaded callers' memo
    uint32_t tuple(uint32_t v, uint32_t ty, uint32_t n, TupleMemo* m) {
        const auto key = std::array<uint32_t, 3>{v, ty, n};
        for (int k = 0; k < m->n; k++)
            if (m->key[k] == key) return m->id[k];
        uint32_t id;
        {
            std::lock_guard<std::mutex> g(tuple_mu);
            auto it = tuple_id.find(key);
            if (it != tuple_id.end()) {
                id = it->second;
            } else {
                id = (uint32_t)tuple_id.size();
                tuple_id.emplace(key, id);
            }
        }
        const int slot = m->n < 8 ? m->n++ : (m->next++ & 7);
        m->key[slot] = key;
        m->id[slot] = id;
        return id;
    }

    // Flatten one alloc of a pe_plan_alloc_table (strings already mapped):
    // resources and flags into *ar, its keys appended to *keys. Thread-safe;
    // an error returns its code and message without touching `err`.
    int flatten_into(const pe_plan_alloc_table* t, uint32_t i, pa::AllocRec* ar, std::vector<uint64_t>* keys,
                     TupleMemo* m, const char** msg) {
        const size_t k0 = keys->size();
        ar->cpu = t->cpu_shares ? t->cpu_shares[i] : 0;
        ar->mem = t->memory_mb ? t->memory_mb[i] : 0;
        ar->disk = t->disk_mb ? t->disk_mb[i] : 0;
        ar->terminal = t->terminal ? (t->terminal[i] != 0) : 0;
        ar->bad_port = 0;
        if (t->core_off && t->core_off[i + 1] > t->core_off[i]) {
            // Flattened.Cpu.ReservedCores is a set (cpuset union, structs.go:3711-3719)
            for (uint32_t j = t->core_off[i]; j < t->core_off[i + 1]; j++)
                keys->push_back(pa::make_key(pa::K_CORE_USED, t->core_id[j]));
            std::sort(keys->begin() + k0, keys->end());
            keys->erase(std::unique(keys->begin() + k0, keys->end()), keys->end());
        }
        if (t->port_off) {
            for (uint32_t j = t->port_off[i]; j < t->port_off[i + 1]; j++) {
                const int64_t v = t->port_value[j];
                if (v < 0 || (uint64_t)v >= kMaxValidPort) { ar->bad_port = 1; continue; }   // network.go:203-205, 222-224
                uint32_t ip;
                if (!str(t->port_ip[j], &ip)) { *msg = "port ip string id out of range"; return PE_EINVAL; }
                keys->push_back(pa::make_key(pa::K_PORT_USED, (uint64_t)ip << 16 | (uint64_t)v));
            }
        }
        if (t->dev_off) {
            for (uint32_t j = t->dev_off[i]; j < t->dev_off[i + 1]; j++) {
                uint32_t v, ty, n, inst;
                if (!str(t->dev_vendor[j], &v) || !str(t->dev_type[j], &ty) || !str(t->dev_name[j], &n) ||
                    !str(t->dev_instance[j], &inst)) {
                    *msg = "device string id out of range";
                    return PE_EINVAL;
                }
                keys->push_back(pa::make_key(pa::K_DEV_USED, (uint64_t)inst << 24 | tuple(v, ty, n, m)));
            }
        }
        const size_t nk = keys->size() - k0;
        if (nk > 0xFFFF) { *msg = "alloc holds more than 65535 cores/ports/devices"; return PE_EINVAL; }
        ar->key_off = (uint32_t)k0;
        ar->n_keys = (uint16_t)nk;
        return PE_OK;
    }
    int flatten(const pe_plan_alloc_table* t, uint32_t i, HAlloc* h) {
        pa::AllocRec ar{};
        const char* msg = nullptr;
        h->keys.clear();
        const int rc = flatten_into(t, i, &ar, &h->keys, &memo, &msg);
        if (rc) return fail(rc, msg);
        h->row = t->node_row ? t->node_row[i] : pa::kNone;
        h->terminal = ar.terminal;
        h->bad_port = ar.bad_port;
        h->cpu = ar.cpu; h->mem = ar.mem; h->disk = ar.disk;
        return PE_OK;
    }
    int plan_part(const pe_plan* plan, PlanPart* w, uint32_t* prow, uint32_t* rmoff, pa::PlanAllocRec* pa_recs);

    // Node static keys and the SetNode collide flag (network.go:92-141).
    int build_node(const pe_plan_node_table* t, const pe_strtab* strs, uint32_t r, pa::NodeRec* nd) {
        memset(nd, 0, sizeof(*nd));
        nd->ready = t->ready ? t->ready[r] != 0 : 1;
        nd->eligible = t->eligible ? t->eligible[r] != 0 : 1;
        nd->cpu = t->cpu_shares[r] - (t->reserved_cpu ? t->reserved_cpu[r] : 0);
        nd->mem = t->memory_mb[r] - (t->reserved_memory_mb ? t->reserved_memory_mb[r] : 0);
        nd->disk = t->disk_mb[r] - (t->reserved_disk_mb ? t->reserved_disk_mb[r] : 0);
        nd->key_off = (uint32_t)node_keys.size();
        if (t->core_off) {
            std::set<uint32_t> cores(t->core_id + t->core_off[r], t->core_id + t->core_off[r + 1]);
            for (uint32_t c : cores) {
                if (c < 64) nd->core_mask |= 1ull << c;
                else node_keys.push_back(pa::make_key(pa::K_CORE_AVAIL, c));
            }
            nd->has_cores = !cores.empty();
        }
        // SetNode: bitmaps per IP; `collide` is assigned (not or-ed) by the
        // ReservedHostPorts step, exactly as network.go:131-133 does.
        std::map<uint32_t, std::set<uint32_t>> used;
        bool collide = false;
        std::string tmp;
        std::vector<uint32_t> ports;
        if (t->addr_off) {
            for (uint32_t j = t->addr_off[r]; j < t->addr_off[r + 1]; j++) {   // AddReservedPortsForIP
                const std::string* spec = text(t->addr_reserved_ports[j], strs, &tmp);
                if (!spec) return fail(PE_EINVAL, "address reserved-ports string id out of range");
                if (!parse_port_ranges(*spec, &ports)) continue;
                uint32_t ip;
                if (!str(t->addr_ip[j], &ip)) return fail(PE_EINVAL, "address string id out of range");
                auto& bm = used[ip];
                for (uint32_t p : ports) {
                    if (p >= kMaxValidPort) { collide = true; break; }
                    if (!bm.insert(p).second) collide = true;
                }
            }
        }
        if (t->reserved_host_ports) {
            const std::string* spec = text(t->reserved_host_ports[r], strs, &tmp);
            if (!spec) return fail(PE_EINVAL, "reserved host ports string id out of range");
            if (!spec->empty()) {   // AddReservedPortRange
                if (!parse_port_ranges(*spec, &ports)) {
                    collide = false;
                } else {
                    if (t->net_off)
                        for (uint32_t j = t->net_off[r]; j < t->net_off[r + 1]; j++) {
                            uint32_t ip;
                            if (!str(t->net_ip[j], &ip)) return fail(PE_EINVAL, "network ip string id out of range");
                            used[ip];
                        }
                    collide = false;
                    for (auto& kv : used) {
                        bool stop = false;
                        for (uint32_t p : ports) {
                            if (p >= kMaxValidPort) { collide = true; stop = true; break; }
                            if (!kv.second.insert(p).second) collide = true;
                        }
                        if (stop) break;
                    }
                }
            }
        }
        nd->setnode_collide = collide;
        for (auto& kv : used)
            for (uint32_t p : kv.second) node_keys.push_back(pa::make_key(pa::K_PORT_NODE, (uint64_t)kv.first << 16 | p));
        // DeviceAccounter: healthy instances per DeviceIdTuple; a later group
        // with the same tuple replaces the earlier one (map assignment, devices.go:38-52).
        if (t->dev_off) {
            std::map<uint32_t, std::set<uint32_t>> inst;
            for (uint32_t g = t->dev_off[r]; g < t->dev_off[r + 1]; g++) {
                uint32_t v, ty, n;
                if (!str(t->dev_vendor[g], &v) || !str(t->dev_type[g], &ty) || !str(t->dev_name[g], &n))
                    return fail(PE_EINVAL, "device string id out of range");
                auto& s = inst[tuple(v, ty, n, &memo)];
                s.clear();
                for (uint32_t k = t->inst_off[g]; k < t->inst_off[g + 1]; k++) {
                    if (!t->inst_healthy[k]) continue;
                    uint32_t id;
                    if (!str(t->inst_id[k], &id)) return fail(PE_EINVAL, "instance string id out of range");
                    s.insert(id);
                }
            }
            for (auto& kv : inst)
                for (uint32_t id : kv.second)
                    node_keys.push_back(pa::make_key(pa::K_DEV_AVAIL, (uint64_t)id << 24 | kv.first));
        }
        nd->n_keys = (uint32_t)node_keys.size() - nd->key_off;
        return PE_OK;
    }

    // Pool: non-terminal allocs grouped by node row (stable in caller order).
    int rebuild_pool() {
        std::vector<uint32_t> order;
        order.reserve(allocs.size());
        for (uint32_t i = 0; i < allocs.size(); i++)
            if (!allocs[i].terminal) order.push_back(i);
        std::stable_sort(order.begin(), order.end(),
                         [&](uint32_t a, uint32_t b) { return allocs[a].row < allocs[b].row; });
        pool.assign(order.size(), pa::AllocRec{});
        pool_keys.clear();
        chunks.clear();
        pool_of.assign(allocs.size(), pa::kNone);
        for (auto& nd : nodes) { nd.alloc_off = 0; nd.alloc_cnt = 0; nd.alloc_keys = 0; nd.ext_head = pa::kNone; }
        for (uint32_t q = 0; q < order.size(); q++) {
            const HAlloc& h = allocs[order[q]];
            pool_of[order[q]] = q;
            pa::AllocRec& ar = pool[q];
            ar.cpu = h.cpu; ar.mem = h.mem; ar.disk = h.disk;
            ar.key_off = (uint32_t)pool_keys.size();
            ar.n_keys = (uint16_t)h.keys.size();
            ar.terminal = 0;
            ar.bad_port = h.bad_port;
            pool_keys.insert(pool_keys.end(), h.keys.begin(), h.keys.end());
            pa::NodeRec& nd = nodes[h.row];
            if (nd.alloc_cnt == 0) nd.alloc_off = q;
            nd.alloc_cnt++;
            nd.alloc_keys += ar.n_keys;
        }
        hipError_t e;
        // headroom for the commits that append to the pool before the next compaction
        const size_t room = std::max<size_t>(pool.size(), 4096);
        const size_t key_room = std::max<size_t>(pool_keys.size(), 16384);
        if ((e = d_pool.reserve((pool.size() + room) * sizeof(pa::AllocRec))) != hipSuccess ||
            (e = d_pool_keys.reserve((pool_keys.size() + key_room) * 8)) != hipSuccess ||
            (e = d_chunks.reserve(std::max<size_t>(nodes.size() / 2, 4096) * sizeof(pa::Chunk))) != hipSuccess ||
            (e = upload(d_nodes, nodes.data(), nodes.size() * sizeof(pa::NodeRec))) != hipSuccess ||
            (e = upload(d_node_keys, node_keys.data(), node_keys.size() * 8)) != hipSuccess ||
            (e = upload(d_pool, pool.data(), pool.size() * sizeof(pa::AllocRec))) != hipSuccess ||
            (e = upload(d_pool_keys, pool_keys.data(), pool_keys.size() * 8)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)
            return fail(PE_EHIP, std::string("planner upload: ") + hipGetErrorString(e));
        return PE_OK;
    }

    // Copy into an existing device buffer at an offset; false when it does not fit.
    bool upload_at(DBuf& b, size_t off, const void* src, size_t bytes, hipError_t* e) {
        *e = hipSuccess;
        if (bytes == 0) return true;
        if (off + bytes > b.cap) return false;
        *e = hipMemcpyAsync((char*)b.p + off, src, bytes, hipMemcpyHostToDevice, stream);
        return true;
    }

    hipError_t upload(DBuf& b, const void* src, size_t bytes) {
        hipError_t e = b.reserve(std::max<size_t>(bytes, 16));
        if (e != hipSuccess || bytes == 0) return e;
        return hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, stream);
    }
};

// What k_plan_eval reads and writes for the last evaluated plan: per plan node
// its row and place_off (4 + 4 B; + 4 B rm_off when the plan removes allocs) and
// 1 reason byte; with a placement on a known node its 64 B record; when the fit
// check runs the node's static keys, every snapshot / chunk alloc record of the
// node (32 B), the keys of those still counted, 4 B per removal and each plan
// alloc (16 B) with its keys; the distinct resource triples once (24 B each)
// (DESIGN.md §9). Computed on the host when asked, against the current snapshot.
uint64_t pe_planner::plan_bytes() const {
    std::set<std::array<int64_t, 3>> distinct;   // the parts' tables may repeat a triple
    for (uint32_t k = 0; k < last_nres; k++) distinct.insert({last_res[k].cpu, last_res[k].mem, last_res[k].disk});
    uint64_t bytes = sizeof(pa::PlanRes) * (uint64_t)distinct.size();
    for (uint32_t i = 0; i < last_np; i++) {
        const uint32_t row = last_row[i], place_off = last_poff[i], place_cnt = last_poff[i + 1] - last_poff[i];
        const uint32_t rm_off = last_rmoff ? last_rmoff[i] : 0, rm_cnt = last_rmoff ? last_rmoff[i + 1] - rm_off : 0;
        bytes += 8 + (last_rmoff ? 4 : 0) + 1;
        if (place_cnt == 0 || row == pa::kNone || (row & ~pa::kBigRow) >= nodes.size()) continue;
        const pa::NodeRec& nd = nodes[row & ~pa::kBigRow];
        bytes += sizeof(pa::NodeRec);
        if (!nd.ready || !nd.eligible) continue;
        bytes += 8ull * nd.n_keys + sizeof(pa::AllocRec) * (uint64_t)nd.alloc_cnt + 4ull * rm_cnt;
        auto count_range = [&](uint32_t off, uint32_t cnt) {
            for (uint32_t q = off; q < off + cnt && q < pool.size(); q++) {
                const bool gone = pool[q].terminal || std::binary_search(last_rm + rm_off, last_rm + rm_off + rm_cnt, q);
                if (!gone) bytes += 8ull * pool[q].n_keys;
            }
        };
        count_range(nd.alloc_off, nd.alloc_cnt);
        for (uint32_t c = nd.ext_head; c != pa::kNone && c < chunks.size(); c = chunks[c].next) {
            bytes += sizeof(pa::Chunk) + sizeof(pa::AllocRec) * (uint64_t)chunks[c].cnt;
            count_range(chunks[c].off, chunks[c].cnt);
        }
        for (uint32_t j = place_off; j < place_off + place_cnt && j < last_npa; j++)
            bytes += sizeof(pa::PlanAllocRec) + (last_pa[j].terminal ? 0 : 8ull * last_pa[j].n_keys);
    }
    return bytes;
}

// Plan nodes [w->n0, w->n1) and their placed allocs: plan alloc records into
// pa_recs (key and resource offsets local to the part), rows into prow and
// removal offsets into rmoff (local to the part), k_plan_eval_big's nodes with
// part-local scratch offsets. Alloc errors take precedence over plan node
// errors, the serial order of evaluate.
int pe_planner::plan_part(const pe_plan* plan, PlanPart* w, uint32_t* prow, uint32_t* rmoff, pa::PlanAllocRec* pa_recs) {
    const pe_plan_alloc_table& pt = plan->allocs;
    w->keys.clear();
    w->rm.clear();
    w->big.clear();
    w->res.clear();
    w->scratch = 0;
    w->rc = w->node_rc = PE_OK;
    for (uint32_t i = w->n0; i < w->n1; i++)
        if (plan->place_off[i + 1] < plan->place_off[i]) {
            w->msg = "place_off not ascending";
            return w->rc = PE_EINVAL;
        }
    const uint32_t a0 = plan->place_off[w->n0], a1 = plan->place_off[w->n1];
    pa::AllocRec ar;
    for (uint32_t j = a0; j < a1; j++) {
        if ((w->rc = flatten_into(&pt, j, &ar, &w->keys, &w->memo, &w->msg))) return w->rc;
        pa::PlanAllocRec& pr = pa_recs[j];
        pr.key_off = ar.key_off;
        pr.n_keys = ar.n_keys;
        pr.terminal = ar.terminal;
        pr.bad_port = ar.bad_port;
        pr._pad = 0;
        // the task group's allocs repeat one triple: compare with the last few
        const size_t nr = w->res.size();
        uint32_t idx = (uint32_t)nr;
        for (size_t k = nr; k > 0 && k + 4 > nr; k--) {
            const pa::PlanRes& r = w->res[k - 1];
            if (r.cpu == ar.cpu && r.mem == ar.mem && r.disk == ar.disk) { idx = (uint32_t)(k - 1); break; }
        }
        if (idx == nr) w->res.push_back(pa::PlanRes{ar.cpu, ar.mem, ar.disk});
        pr.res = idx;
    }
    for (uint32_t i = w->n0; i < w->n1; i++) {
        const uint32_t row = plan->node_row[i];
        if (row != pa::kNone && row >= nodes.size()) {
            w->node_msg = "plan node_row out of range";
            return w->node_rc = PE_EINVAL;
        }
        prow[i] = row;
        const uint32_t place_off = plan->place_off[i], place_cnt = plan->place_off[i + 1] - place_off;
        if (rmoff) {
            rmoff[i] = (uint32_t)w->rm.size();
            const size_t b = w->rm.size();
            for (uint32_t j = plan->remove_off[i]; j < plan->remove_off[i + 1]; j++) {
                const uint32_t a = plan->remove_alloc[j];
                if (a >= allocs.size()) {
                    w->node_msg = "remove_alloc out of range";
                    return w->node_rc = PE_EINVAL;
                }
                if (pool_of[a] != pa::kNone) w->rm.push_back(pool_of[a]);
            }
            std::sort(w->rm.begin() + b, w->rm.end());
            w->rm.erase(std::unique(w->rm.begin() + b, w->rm.end()), w->rm.end());
        }
        if (place_cnt == 0 || row == pa::kNone) continue;
        const pa::NodeRec& nd = nodes[row];
        if (!nd.ready || !nd.eligible) continue;
        uint64_t bound = (uint64_t)nd.n_keys + nd.alloc_keys;   // k_plan_eval's sum
        for (uint32_t j = place_off; j < place_off + place_cnt; j++) bound += pa_recs[j].n_keys;
        if (bound > pa::lds_keys(group)) {
            prow[i] = row | pa::kBigRow;
            w->big.push_back(pa::BigNode{i, (uint32_t)std::min<uint64_t>(w->scratch, 0xFFFFFFFFull)});
            w->scratch += bound;
        }
    }
    return PE_OK;
}

extern "C" {

pe_planner* pe_planner_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    auto* p = new pe_planner();
    p->device = device;
    if (const char* g = getenv("PE_PLAN_GROUP")) {
        const int v = atoi(g);
        if (v == 4 || v == 8 || v == 16 || v == 64) p->group = v;
    }
    p->threads = (int)std::min<unsigned>(16, std::max<unsigned>(1, std::thread::hardware_concurrency()));
    if (const char* g = getenv("PE_PLAN_THREADS")) p->threads = std::max(1, std::min(64, atoi(g)));
    if (const char* g = getenv("PE_PLAN_SPIN_US")) p->spin_us = std::max(0, atoi(g));
    if (const char* g = getenv("PE_PLAN_COPY")) p->copy_kernel = strcmp(g, "kernel") == 0;
    if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&p->e0) != hipSuccess || hipEventCreate(&p->e1) != hipSuccess) {
        delete p;
        return nullptr;
    }
    return p;
}

void pe_planner_destroy(pe_planner* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    if (p->stream) (void)hipStreamSynchronize(p->stream);
    if (p->e0) (void)hipEventDestroy(p->e0);
    if (p->e1) (void)hipEventDestroy(p->e1);
    if (p->stream) (void)hipStreamDestroy(p->stream);
    delete p;
}

const char* pe_planner_last_error(const pe_planner* p) { return p ? p->err.c_str() : "null planner"; }

int pe_planner_set_state(pe_planner* p, const pe_strtab* strs, const pe_plan_node_table* t,
                         const pe_plan_alloc_table* al) {
    if (!p || !t) return PE_EINVAL;
    if (t->n && (!t->cpu_shares || !t->memory_mb || !t->disk_mb)) return p->fail(PE_EINVAL, "node resources missing");
    if (hipSetDevice(p->device) != hipSuccess) return p->fail(PE_EHIP, "hipSetDevice");
    p->have_state = false;
    if (t->n >= pa::kBigRow) return p->fail(PE_EINVAL, "snapshot of 2^31 nodes or more");
    int rc = p->map_strings(strs);
    if (rc) return rc;
    p->nodes.assign(t->n, pa::NodeRec{});
    p->node_keys.clear();
    for (uint32_t r = 0; r < t->n; r++)
        if ((rc = p->build_node(t, strs, r, &p->nodes[r]))) return rc;
    p->allocs.clear();
    if (al) {
        p->allocs.resize(al->count);
        for (uint32_t i = 0; i < al->count; i++) {
            if ((rc = p->flatten(al, i, &p->allocs[i]))) return rc;
            if (p->allocs[i].row >= t->n) return p->fail(PE_EINVAL, "alloc node_row out of range");
        }
    }
    if ((rc = p->rebuild_pool())) return rc;
    p->have_state = true;
    return PE_OK;
}

int pe_planner_evaluate(pe_planner* p, const pe_strtab* strs, const pe_plan* plan, uint8_t* reason,
                        uint32_t* n_fit) {
    if (!p || !plan || (plan->n_nodes && (!reason || !plan->node_row || !plan->place_off))) return PE_EINVAL;
    if (!p->have_state) return p->fail(PE_ESTATE, "pe_planner_set_state not called");
    if (hipSetDevice(p->device) != hipSuccess) return p->fail(PE_EHIP, "hipSetDevice");
    const bool prof = getenv("PE_PLAN_PROF") != nullptr;
    auto tnow = [] { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
    double t[6] = {tnow(), 0, 0, 0, 0, 0};
    int rc = p->map_strings(strs);
    if (rc) return rc;
    t[1] = tnow();
    const uint32_t np = plan->n_nodes;
    const pe_plan_alloc_table& pt = plan->allocs;
    if (np && plan->place_off[np] > pt.count) return p->fail(PE_EINVAL, "place_off exceeds plan allocs");
    const uint32_t na = np ? plan->place_off[np] : 0;

    // Flatten into one pinned staging region, one part per worker over
    // contiguous plan node ranges (balanced by plan nodes + placed allocs);
    // the parts' key / removal / scratch / resource offsets are then made
    // global and their keys, removals and resource triples gathered behind
    // each other; one copy to the device. Alloc errors take precedence over
    // plan node errors (the serial order: every alloc is flattened before the
    // plan nodes are walked).
    auto span = [](const uint32_t* off, uint32_t n) -> uint64_t {
        return off && n && off[n] > off[0] ? off[n] - off[0] : 0;
    };
    const uint64_t key_cap = span(pt.core_off, na) + span(pt.port_off, na) + span(pt.dev_off, na);
    const uint64_t rm_cap = plan->remove_off ? span(plan->remove_off, np) : 0;
    if (key_cap > 0xFFFFFFFFull || rm_cap > 0xFFFFFFFFull) return p->fail(PE_ENOMEM, "plan too large");
    const bool has_rm = rm_cap > 0;
    // staging layout (host and device alike, 256-B aligned parts): rows,
    // place_off, rm_off (plans with removals), plan allocs, keys (up to the
    // offsets' bound), resource triples, removals
    auto al = [](uint64_t x) { return (x + 255) & ~255ull; };
    const uint64_t o_poff = al(4ull * np);
    const uint64_t o_rmoff = al(o_poff + 4ull * (np + 1));
    const uint64_t o_pa = al(o_rmoff + (has_rm ? 4ull * (np + 1) : 0));
    const uint64_t o_keys = al(o_pa + (uint64_t)na * sizeof(pa::PlanAllocRec));
    const uint64_t o_res = al(o_keys + key_cap * 8);
    const uint64_t o_rm = al(o_res + (uint64_t)std::max<uint32_t>(na, 1) * sizeof(pa::PlanRes));
    const uint64_t stage_bytes = al(o_rm + rm_cap * 4) + 256;
    hipError_t e;
    if ((e = p->h_stage.reserve(stage_bytes)) != hipSuccess || (e = p->d_stage.reserve(stage_bytes)) != hipSuccess ||
        (e = p->d_reason.reserve(std::max<uint32_t>(np, 1))) != hipSuccess)
        return p->fail(PE_EHIP, std::string("planner staging: ") + hipGetErrorString(e));
    char* const hs = (char*)p->h_stage.p;
    char* const ds = (char*)p->d_stage.p;
    auto* prow = (uint32_t*)hs;
    auto* poff = (uint32_t*)(hs + o_poff);
    auto* rmoff = has_rm ? (uint32_t*)(hs + o_rmoff) : nullptr;
    auto* pa_recs = (pa::PlanAllocRec*)(hs + o_pa);
    auto* pkeys = (uint64_t*)(hs + o_keys);
    auto* pres = (pa::PlanRes*)(hs + o_res);
    auto* rm = (uint32_t*)(hs + o_rm);
    // ranges of [0, np) balanced by plan nodes + placed allocs
    auto split = [&](int k, int parts) -> uint32_t {
        if (k == parts) return np;
        const uint64_t goal = ((uint64_t)np + plan->place_off[np]) * k / parts;
        uint32_t a = 0, b = np;   // first i with i + place_off[i] >= goal (binary search)
        while (a < b) {
            const uint32_t m = a + (b - a) / 2;
            if ((uint64_t)m + plan->place_off[m] < goal) a = m + 1;
            else b = m;
        }
        return a;
    };
    const int T = np == 0 ? 0 : (np + na >= 8192) ? p->threads : 1;
    if ((int)p->parts.size() < T) p->parts.resize(T);
    for (int k = 0; k < T; k++) {
        p->parts[k].n0 = split(k, T);
        p->parts[k].n1 = split(k + 1, T);
    }
    auto part = [&](int k) { if (k < T) p->plan_part(plan, &p->parts[k], prow, rmoff, pa_recs); };
    if (T > 1) p->workers().run(part);
    else if (T == 1) part(0);
    for (int k = 0; k < T; k++)
        if (p->parts[k].rc) return p->fail(p->parts[k].rc, p->parts[k].msg);
    for (int k = 0; k < T; k++)
        if (p->parts[k].node_rc) return p->fail(p->parts[k].node_rc, p->parts[k].node_msg);
    t[2] = tnow();
    uint64_t nkeys = 0, nrm = 0, scratch = 0, nres = 0;
    std::vector<pa::BigNode> big;
    for (int k = 0; k < T; k++) {
        PlanPart& w = p->parts[k];
        w.key_base = nkeys;
        w.rm_base = nrm;
        w.scratch_base = scratch;
        w.res_base = nres;
        nkeys += w.keys.size();
        nrm += w.rm.size();
        nres += w.res.size();
        for (const pa::BigNode& b : w.big) big.push_back(pa::BigNode{b.p, (uint32_t)(b.scratch_off + scratch)});
        scratch += w.scratch;
    }
    if (scratch > 0xFFFFFFF0ull) return p->fail(PE_ENOMEM, "plan key scratch too large");
    if (nkeys > key_cap || nrm > rm_cap) return p->fail(PE_EINVAL, "plan offsets not ascending");
    auto gather = [&](int k) {
        if (k >= T) return;
        const PlanPart& w = p->parts[k];
        if (w.n0 == w.n1) return;
        const uint32_t kb = (uint32_t)w.key_base, rb = (uint32_t)w.rm_base, resb = (uint32_t)w.res_base;
        for (uint32_t j = plan->place_off[w.n0]; j < plan->place_off[w.n1]; j++) {
            pa_recs[j].key_off += kb;
            pa_recs[j].res += resb;
        }
        memcpy(poff + w.n0, plan->place_off + w.n0, 4ull * (w.n1 - w.n0));
        if (rmoff)
            for (uint32_t i = w.n0; i < w.n1; i++) rmoff[i] += rb;
        if (!w.keys.empty()) memcpy(pkeys + kb, w.keys.data(), w.keys.size() * 8);
        if (!w.res.empty()) memcpy(pres + resb, w.res.data(), w.res.size() * sizeof(pa::PlanRes));
        if (!w.rm.empty()) memcpy(rm + rb, w.rm.data(), w.rm.size() * 4);
    };
    if (T > 1) p->workers().run(gather);
    else if (T == 1) gather(0);
    poff[np] = np ? plan->place_off[np] : 0;
    if (rmoff) rmoff[np] = (uint32_t)nrm;
    t[3] = tnow();
    // host -> device: one copy-engine transfer of everything up to the last
    // resource triple (+ the removals), or k_plan_stage_copy reading the
    // mapped staging (PE_PLAN_COPY=kernel)
    void* hs_dev = nullptr;
    if (p->copy_kernel && hipHostGetDevicePointer(&hs_dev, hs, 0) != hipSuccess) hs_dev = nullptr;
    auto h2d = [&](uint64_t off, uint64_t bytes) -> hipError_t {
        if (!bytes) return hipSuccess;
        if (hs_dev) return pe_launch_plan_stage_copy((const char*)hs_dev + off, ds + off, bytes, p->stream);
        return hipMemcpyAsync(ds + off, hs + off, bytes, hipMemcpyHostToDevice, p->stream);
    };
    if ((np && (e = h2d(0, o_res + nres * sizeof(pa::PlanRes))) != hipSuccess) ||
        (e = h2d(o_rm, nrm * 4)) != hipSuccess ||
        (e = p->upload(p->d_big, big.data(), big.size() * sizeof(pa::BigNode))) != hipSuccess ||
        (e = p->d_scratch.reserve(std::max<uint64_t>(scratch, 1) * 8)) != hipSuccess) {
        (void)hipStreamSynchronize(p->stream);
        return p->fail(PE_EHIP, std::string("planner plan upload: ") + hipGetErrorString(e));
    }
    t[4] = tnow();
    pa::PlanArgs a{};
    a.nodes = (const pa::NodeRec*)p->d_nodes.p;
    a.chunks = (const pa::Chunk*)p->d_chunks.p;
    a.pool = (const pa::AllocRec*)p->d_pool.p;
    a.node_keys = (const uint64_t*)p->d_node_keys.p;
    a.pool_keys = (const uint64_t*)p->d_pool_keys.p;
    a.prow = (const uint32_t*)ds;
    a.poff = (const uint32_t*)(ds + o_poff);
    a.rmoff = rmoff ? (const uint32_t*)(ds + o_rmoff) : nullptr;
    a.n_plan = np;
    a.rm = (const uint32_t*)(ds + o_rm);
    a.pallocs = (const pa::PlanAllocRec*)(ds + o_pa);
    a.pres = (const pa::PlanRes*)(ds + o_res);
    a.pkeys = (const uint64_t*)(ds + o_keys);
    a.scratch = (uint64_t*)p->d_scratch.p;
    a.big = (const pa::BigNode*)p->d_big.p;
    a.n_big = (uint32_t)big.size();
    a.reason = (uint8_t*)p->d_reason.p;
    if ((e = hipEventRecord(p->e0, p->stream)) != hipSuccess || (e = pe_launch_plan_eval(&a, p->group, p->stream)) != hipSuccess ||
        (e = hipEventRecord(p->e1, p->stream)) != hipSuccess ||
        (np && (e = hipMemcpyAsync(reason, a.reason, np, hipMemcpyDeviceToHost, p->stream)) != hipSuccess) ||
        (e = hipStreamSynchronize(p->stream)) != hipSuccess)
        return p->fail(PE_EHIP, std::string("planner evaluate: ") + hipGetErrorString(e));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, p->e0, p->e1);
    p->last_ms = ms;
    p->last_row = prow;
    p->last_poff = poff;
    p->last_rmoff = rmoff;
    p->last_rm = rm;
    p->last_pa = pa_recs;
    p->last_np = np;
    p->last_npa = na;
    p->last_nres = (uint32_t)nres;
    p->last_res = pres;
    p->bytes_valid = false;
    if (prof) {
        t[5] = tnow();
        fprintf(stderr, "planner evaluate us: strings %.1f flatten %.1f gather %.1f upload %.1f "
                        "kernel+reasons %.1f (kernel %.1f, %d threads)\n", t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4],
                ms * 1e3, T);
    }
    uint32_t fit = 0;
    for (uint32_t i = 0; i < np; i++) fit += reason[i] == PE_PLAN_FIT;
    if (n_fit) *n_fit = fit;
    return PE_OK;
}

int pe_planner_commit(pe_planner* p, const pe_strtab* strs, const pe_plan* plan, const uint8_t* keep) {
    if (!p || !plan || (plan->n_nodes && (!keep || !plan->node_row || !plan->place_off))) return PE_EINVAL;
    if (!p->have_state) return p->fail(PE_ESTATE, "pe_planner_set_state not called");
    if (hipSetDevice(p->device) != hipSuccess) return p->fail(PE_EHIP, "hipSetDevice");
    int rc = p->map_strings(strs);
    if (rc) return rc;
    const pe_plan_alloc_table& pt = plan->allocs;
    for (uint32_t i = 0; i < plan->n_nodes; i++) {   // validate before changing anything
        if (!keep[i]) continue;
        const uint32_t row = plan->node_row[i];
        if (plan->place_off[i + 1] > plan->place_off[i] && (row == pa::kNone || row >= p->nodes.size()))
            return p->fail(PE_EINVAL, "commit places allocs on a node outside the snapshot");
        if (plan->remove_off)
            for (uint32_t j = plan->remove_off[i]; j < plan->remove_off[i + 1]; j++)
                if (plan->remove_alloc[j] >= p->allocs.size()) return p->fail(PE_EINVAL, "remove_alloc out of range");
    }
    // Incremental: removed allocs turn terminal in place, placed allocs are
    // appended to the pool as one chunk per node (chained from the node's
    // record); the device gets the appended records and a small patch.
    const size_t pool0 = p->pool.size(), keys0 = p->pool_keys.size(), chunks0 = p->chunks.size();
    std::vector<uint32_t> dead, rows;
    HAlloc h;
    for (uint32_t i = 0; i < plan->n_nodes; i++) {
        if (!keep[i]) continue;
        const uint32_t row = plan->node_row[i];
        if (plan->remove_off)
            for (uint32_t j = plan->remove_off[i]; j < plan->remove_off[i + 1]; j++) {
                const uint32_t a = plan->remove_alloc[j];
                if (p->allocs[a].terminal) continue;
                p->allocs[a].terminal = 1;
                if (p->pool_of[a] != pa::kNone) {
                    dead.push_back(p->pool_of[a]);
                    p->pool[p->pool_of[a]].terminal = 1;
                }
            }
        const uint32_t b = plan->place_off[i], e = plan->place_off[i + 1];
        if (e == b) continue;
        pa::NodeRec& nd = p->nodes[row];
        pa::Chunk ch{(uint32_t)p->pool.size(), e - b, nd.ext_head, 0};
        for (uint32_t j = b; j < e; j++) {
            if ((rc = p->flatten(&pt, j, &h))) return rc;   // validated by the evaluate of this plan
            h.row = row;
            pa::AllocRec ar{};
            ar.cpu = h.cpu; ar.mem = h.mem; ar.disk = h.disk;
            ar.key_off = (uint32_t)p->pool_keys.size();
            ar.n_keys = (uint16_t)h.keys.size();
            ar.terminal = h.terminal;
            ar.bad_port = h.bad_port;
            p->pool_keys.insert(p->pool_keys.end(), h.keys.begin(), h.keys.end());
            nd.alloc_keys += ar.n_keys;
            p->pool_of.push_back((uint32_t)p->pool.size());
            p->pool.push_back(ar);
            p->allocs.push_back(h);
        }
        if (nd.ext_head == ch.next) rows.push_back(row);   // first chunk of this commit for the row
        nd.ext_head = (uint32_t)p->chunks.size();
        p->chunks.push_back(ch);
    }
    hipError_t e = hipSuccess;
    const bool fits =
        p->upload_at(p->d_pool, pool0 * sizeof(pa::AllocRec), p->pool.data() + pool0,
                     (p->pool.size() - pool0) * sizeof(pa::AllocRec), &e) && e == hipSuccess &&
        p->upload_at(p->d_pool_keys, keys0 * 8, p->pool_keys.data() + keys0, (p->pool_keys.size() - keys0) * 8, &e) &&
        e == hipSuccess &&
        p->upload_at(p->d_chunks, chunks0 * sizeof(pa::Chunk), p->chunks.data() + chunks0,
                     (p->chunks.size() - chunks0) * sizeof(pa::Chunk), &e) && e == hipSuccess;
    if (e != hipSuccess) return p->fail(PE_EHIP, std::string("planner commit upload: ") + hipGetErrorString(e));
    if (!fits) return p->rebuild_pool();   // append room used up: compact
    std::vector<pa::NodeRec> recs(rows.size());
    for (size_t k = 0; k < rows.size(); k++) recs[k] = p->nodes[rows[k]];
    if ((e = p->upload(p->d_patch_dead, dead.data(), dead.size() * 4)) != hipSuccess ||
        (e = p->upload(p->d_patch_rows, rows.data(), rows.size() * 4)) != hipSuccess ||
        (e = p->upload(p->d_patch_recs, recs.data(), recs.size() * sizeof(pa::NodeRec))) != hipSuccess ||
        (e = pe_launch_plan_patch((pa::NodeRec*)p->d_nodes.p, (pa::AllocRec*)p->d_pool.p,
                                  (const uint32_t*)p->d_patch_dead.p, (uint32_t)dead.size(),
                                  (const uint32_t*)p->d_patch_rows.p, (const pa::NodeRec*)p->d_patch_recs.p,
                                  (uint32_t)rows.size(), p->stream)) != hipSuccess ||
        (e = hipStreamSynchronize(p->stream)) != hipSuccess)
        return p->fail(PE_EHIP, std::string("planner commit patch: ") + hipGetErrorString(e));
    return PE_OK;
}

double pe_planner_kernel_ms(const pe_planner* p) { return p ? p->last_ms : 0; }
uint64_t pe_planner_last_bytes(const pe_planner* p) {
    if (!p) return 0;
    if (!p->bytes_valid) {
        p->last_bytes = p->plan_bytes();
        p->bytes_valid = true;
    }
    return p->last_bytes;
}
uint32_t pe_planner_snapshot_allocs(const pe_planner* p) { return p ? (uint32_t)p->allocs.size() : 0; }

}  // extern "C"
