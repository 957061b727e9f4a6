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
#include <cstdlib>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/nomad_pe.h"
#include "plan_types.h"

hipError_t pe_launch_plan_eval(const pa::PlanArgs* a, int group, hipStream_t st);
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
    std::vector<pa::PlanNodeRec> last_pn;
    std::vector<uint32_t> last_rm;
    std::vector<pa::AllocRec> last_pa;
    uint64_t plan_bytes() const;
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
    DBuf d_pn, d_rm, d_pallocs, d_pkeys, d_big, d_scratch, d_reason;

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
        if (have && t->count >= have && memcmp(t->offsets, xl_off.data(), (have + 1) * 4) == 0 &&
            memcmp(t->bytes, xl_bytes.data(), xl_bytes.size()) == 0)
            keep = have;
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
    std::array<uint32_t, 3> last_tuple{{PE_NONE, PE_NONE, PE_NONE}};
    uint32_t last_tuple_id = 0;
    uint32_t tuple(uint32_t v, uint32_t ty, uint32_t n) {
        auto key = std::array<uint32_t, 3>{v, ty, n};
        if (key == last_tuple) return last_tuple_id;   // allocs of a node repeat their device type
        last_tuple = key;
        auto it = tuple_id.find(key);
        if (it != tuple_id.end()) return last_tuple_id = it->second;
        const uint32_t id = (uint32_t)tuple_id.size();
        tuple_id.emplace(key, id);
        return last_tuple_id = id;
    }

    // Flatten one alloc of a pe_plan_alloc_table (strings already mapped).
    int flatten(const pe_plan_alloc_table* t, uint32_t i, HAlloc* h) {
        h->row = t->node_row ? t->node_row[i] : pa::kNone;
        h->terminal = t->terminal ? (t->terminal[i] != 0) : 0;
        h->cpu = t->cpu_shares ? t->cpu_shares[i] : 0;
        h->mem = t->memory_mb ? t->memory_mb[i] : 0;
        h->disk = t->disk_mb ? t->disk_mb[i] : 0;
        h->bad_port = 0;
        h->keys.clear();
        if (t->core_off && t->core_off[i + 1] > t->core_off[i]) {
            // Flattened.Cpu.ReservedCores is a set (cpuset union, structs.go:3711-3719)
            const size_t b = h->keys.size();
            for (uint32_t j = t->core_off[i]; j < t->core_off[i + 1]; j++)
                h->keys.push_back(pa::make_key(pa::K_CORE_USED, t->core_id[j]));
            std::sort(h->keys.begin() + b, h->keys.end());
            h->keys.erase(std::unique(h->keys.begin() + b, h->keys.end()), h->keys.end());
        }
        if (t->port_off) {
            for (uint32_t j = t->port_off[i]; j < t->port_off[i + 1]; j++) {
                const int64_t v = t->port_value[j];
                if (v < 0 || (uint64_t)v >= kMaxValidPort) { h->bad_port = 1; continue; }   // network.go:203-205, 222-224
                uint32_t ip;
                if (!str(t->port_ip[j], &ip)) return fail(PE_EINVAL, "port ip string id out of range");
                h->keys.push_back(pa::make_key(pa::K_PORT_USED, (uint64_t)ip << 16 | (uint64_t)v));
            }
        }
        if (t->dev_off) {
            for (uint32_t j = t->dev_off[i]; j < t->dev_off[i + 1]; j++) {
                uint32_t v, ty, n, inst;
                if (!str(t->dev_vendor[j], &v) || !str(t->dev_type[j], &ty) || !str(t->dev_name[j], &n) ||
                    !str(t->dev_instance[j], &inst))
                    return fail(PE_EINVAL, "device string id out of range");
                h->keys.push_back(pa::make_key(pa::K_DEV_USED, (uint64_t)inst << 24 | tuple(v, ty, n)));
            }
        }
        if (h->keys.size() > 0xFFFF) return fail(PE_EINVAL, "alloc holds more than 65535 cores/ports/devices");
        return PE_OK;
    }

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
                auto& s = inst[tuple(v, ty, n)];
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

// What k_plan_eval reads and writes for the last evaluated plan: 32 B plan
// node record + 1 reason byte per plan node; with a placement on a known node
// its 64 B record; when the fit check runs the node's static keys, every
// snapshot / chunk alloc record of the node (32 B), the keys of those still
// counted, 4 B per removal and each plan alloc with its keys.
// Computed on the host when asked, against the current snapshot.
uint64_t pe_planner::plan_bytes() const {
    uint64_t bytes = 0;
    for (const pa::PlanNodeRec& r : last_pn) {
        bytes += sizeof(pa::PlanNodeRec) + 1;
        if (r.place_cnt == 0 || r.row == pa::kNone || r.row >= nodes.size()) continue;
        const pa::NodeRec& nd = nodes[r.row];
        bytes += sizeof(pa::NodeRec);
        if (!nd.ready || !nd.eligible) continue;
        bytes += 8ull * nd.n_keys + sizeof(pa::AllocRec) * (uint64_t)nd.alloc_cnt + 4ull * r.rm_cnt;
        auto count_range = [&](uint32_t off, uint32_t cnt) {
            for (uint32_t q = off; q < off + cnt && q < pool.size(); q++) {
                const bool gone = pool[q].terminal ||
                                  std::binary_search(last_rm.begin() + r.rm_off, last_rm.begin() + r.rm_off + r.rm_cnt, q);
                if (!gone) bytes += 8ull * pool[q].n_keys;
            }
        };
        count_range(nd.alloc_off, nd.alloc_cnt);
        for (uint32_t c = nd.ext_head; c != pa::kNone && c < chunks.size(); c = chunks[c].next) {
            bytes += sizeof(pa::Chunk) + sizeof(pa::AllocRec) * (uint64_t)chunks[c].cnt;
            count_range(chunks[c].off, chunks[c].cnt);
        }
        for (uint32_t j = r.place_off; j < r.place_off + r.place_cnt && j < last_pa.size(); j++)
            bytes += sizeof(pa::AllocRec) + (last_pa[j].terminal ? 0 : 8ull * last_pa[j].n_keys);
    }
    return bytes;
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

    std::vector<pa::PlanNodeRec> pn(np);
    std::vector<uint32_t> rm, big;
    std::vector<pa::AllocRec> pa_recs(pt.count);
    std::vector<uint64_t> pkeys;
    HAlloc h;
    for (uint32_t i = 0; i < pt.count; i++) {
        if ((rc = p->flatten(&pt, i, &h))) return rc;
        pa::AllocRec& ar = pa_recs[i];
        ar.cpu = h.cpu; ar.mem = h.mem; ar.disk = h.disk;
        ar.key_off = (uint32_t)pkeys.size();
        ar.n_keys = (uint16_t)h.keys.size();
        ar.terminal = h.terminal;
        ar.bad_port = h.bad_port;
        pkeys.insert(pkeys.end(), h.keys.begin(), h.keys.end());
    }
    t[2] = tnow();
    uint64_t scratch = 0;
    for (uint32_t i = 0; i < np; i++) {
        pa::PlanNodeRec& r = pn[i];
        r.row = plan->node_row[i];
        if (r.row != pa::kNone && r.row >= p->nodes.size()) return p->fail(PE_EINVAL, "plan node_row out of range");
        r.place_off = plan->place_off[i];
        r.place_cnt = plan->place_off[i + 1] - plan->place_off[i];
        r.rm_off = (uint32_t)rm.size();
        if (plan->remove_off) {
            const size_t b = rm.size();
            for (uint32_t j = plan->remove_off[i]; j < plan->remove_off[i + 1]; j++) {
                const uint32_t a = plan->remove_alloc[j];
                if (a >= p->allocs.size()) return p->fail(PE_EINVAL, "remove_alloc out of range");
                if (p->pool_of[a] != pa::kNone) rm.push_back(p->pool_of[a]);
            }
            std::sort(rm.begin() + b, rm.end());
            rm.erase(std::unique(rm.begin() + b, rm.end()), rm.end());
        }
        r.rm_cnt = (uint32_t)rm.size() - r.rm_off;
        r.scratch_off = pa::kNone;
        if (r.place_cnt == 0 || r.row == pa::kNone) continue;
        const pa::NodeRec& nd = p->nodes[r.row];
        if (!nd.ready || !nd.eligible) continue;
        uint64_t bound = (uint64_t)nd.n_keys + nd.alloc_keys;
        for (uint32_t j = r.place_off; j < r.place_off + r.place_cnt; j++) bound += pa_recs[j].n_keys;
        r.key_bound = (uint32_t)std::min<uint64_t>(bound, 0xFFFFFFFFull);
        if (bound > pa::lds_keys(p->group)) {
            big.push_back(i);
            r.scratch_off = (uint32_t)scratch;
            scratch += bound;
            if (scratch > 0xFFFFFFF0ull) return p->fail(PE_ENOMEM, "plan key scratch too large");
        }
    }
    t[3] = tnow();
    hipError_t e;
    if ((e = p->upload(p->d_pn, pn.data(), pn.size() * sizeof(pa::PlanNodeRec))) != hipSuccess ||
        (e = p->upload(p->d_rm, rm.data(), rm.size() * 4)) != hipSuccess ||
        (e = p->upload(p->d_pallocs, pa_recs.data(), pa_recs.size() * sizeof(pa::AllocRec))) != hipSuccess ||
        (e = p->upload(p->d_pkeys, pkeys.data(), pkeys.size() * 8)) != hipSuccess ||
        (e = p->upload(p->d_big, big.data(), big.size() * 4)) != hipSuccess ||
        (e = p->d_scratch.reserve(std::max<uint64_t>(scratch, 1) * 8)) != hipSuccess ||
        (e = p->d_reason.reserve(std::max<uint32_t>(np, 1))) != hipSuccess)
        return p->fail(PE_EHIP, std::string("planner plan upload: ") + hipGetErrorString(e));
    t[4] = tnow();
    pa::PlanArgs a{};
    a.nodes = (const pa::NodeRec*)p->d_nodes.p;
    a.chunks = (const pa::Chunk*)p->d_chunks.p;
    a.pool = (const pa::AllocRec*)p->d_pool.p;
    a.node_keys = (const uint64_t*)p->d_node_keys.p;
    a.pool_keys = (const uint64_t*)p->d_pool_keys.p;
    a.pn = (const pa::PlanNodeRec*)p->d_pn.p;
    a.n_plan = np;
    a.rm = (const uint32_t*)p->d_rm.p;
    a.pallocs = (const pa::AllocRec*)p->d_pallocs.p;
    a.pkeys = (const uint64_t*)p->d_pkeys.p;
    a.scratch = (uint64_t*)p->d_scratch.p;
    a.big = (const uint32_t*)p->d_big.p;
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
    p->last_pn = std::move(pn);
    p->last_rm = std::move(rm);
    p->last_pa = std::move(pa_recs);
    p->bytes_valid = false;
    if (prof) {
        t[5] = tnow();
        fprintf(stderr, "planner evaluate us: strings %.1f flatten %.1f nodes %.1f upload %.1f kernel+reasons %.1f "
                        "(kernel %.1f)\n", t[1] - t[0], t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], ms * 1e3);
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
