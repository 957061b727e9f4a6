// ORACLE — test infrastructure only. Never linked or loaded by the product.
//
// C++ restatement of the reference placement stack with the reference's lazy
// pull semantics, object for object:
//   scheduler/stack.go        GenericStack / SystemStack (Select, SetNodes, SetJob)
//   scheduler/feasible.go     StaticIterator, FeasibilityWrapper, checkers,
//                             DistinctHosts / DistinctProperty iterators
//   scheduler/rank.go         FeasibleRank, BinPack, JobAntiAffinity,
//                             NodeReschedulingPenalty, NodeAffinity, ScoreNormalization
//   scheduler/spread.go       SpreadIterator (+ evenSpreadScoreBoost)
//   scheduler/propertyset.go  propertySet
//   scheduler/select.go       LimitIterator, MaxScoreIterator
//   scheduler/context.go      EvalContext.ProposedAllocs, EvalEligibility
//   nomad/structs/funcs.go    AllocsFit, ScoreFitBinPack, ScoreFitSpread
//   nomad/structs/network.go  NetworkIndex feasibility (ports counted, bandwidth)
// Randomness (shuffleNodes, random port values) is an input / not modelled:
// the caller passes the already-shuffled node order.
//   scheduler/device.go       deviceAllocator.AssignDevice (+ DeviceAccounter, devices.go)
//   scheduler/preemption.go   Preemptor (PreemptForTaskGroup, PreemptForDevice),
//                             PreemptionScoringIterator (rank.go:775-844)
// Go map iteration order (ProposedAllocs, device groups, preemption device
// groups) is replaced by a fixed order: allocs by ascending id (state table
// order, then plan order), device groups in node order.
// sort.Slice is Go 1.16's quickSort_func (go.mod: go 1.16), restated below.
// Modelled as the reference does: PreemptForNetwork (bandwidth, dynamic and
// static ports), reserved cores, static reserved port asks, nodes and
// preempted lists of any length (pe_preempted_of). Out of the oracle's scope
// (returns PE_EUNSUPPORTED): CSI volumes.
#include "oracle.h"
#include "gomath.h"
#include "semantics.h"

#include <string>
#include <vector>
#include <map>
#include <unordered_map>
#include <set>
#include <memory>
#include <cmath>
#include <climits>
#include <stdexcept>
#include <new>
#include <cfloat>
#include <algorithm>

namespace {

using orasem::Val;

struct Unsupported : std::runtime_error {
    explicit Unsupported(const std::string& m) : std::runtime_error(m) {}
};

static const int32_t kDynPortCapacity = 32000 - 20000 + 1;   // IndexesInRange is inclusive

struct DriverInfo { bool detected, healthy, nil; };
struct NetRes { std::string mode, device; int32_t mbits; std::string ip, cidr_ip; };   // cidr_ip: yieldIP's one address

struct ODev {
    std::string vendor, type, name;
    int healthy;
    std::map<std::string, orasem::Attr> attrs;
};

struct ONode {
    int row;
    std::string id, name, dc, node_class, computed_class;
    int64_t cpu, mem, disk, rcpu, rmem, rdisk;
    std::map<std::string, std::string> attrs, meta;
    std::map<std::string, DriverInfo> drivers;
    std::vector<NetRes> nets;
    std::vector<std::string> aliases;
    int32_t reserved_dyn;
    std::map<std::string, bool> host_volumes;   // name -> read only
    int n_devices;
    std::vector<ODev> devs;
    std::vector<uint16_t> rcores, nrsv_cores;   // ReservableCpuCores, ReservedResources.Cpu.ReservedCpuCores
    uint32_t total_cores = 0;                   // TotalCpuCores
    struct Addr { std::string alias, ip; std::vector<int> reserved; };
    std::vector<Addr> addrs;                    // NodeNetworks[*].Addresses[*] in node order
    std::vector<int> reserved_host_ports;       // ReservedResources.Networks.ReservedHostPorts
};

struct OAlloc {
    uint64_t id;
    int node_row;
    std::string ns, job_id, tg;
    bool terminal;
    int32_t priority;
    int64_t cpu, mem, disk;
    int32_t mbits, dyn_ports;
    std::vector<std::pair<int, int>> devs;   // (device group on the node, instances held)
    int32_t max_parallel = 0;
    int state_index = -1;                    // row of the state alloc table (-1: plan alloc)
    std::vector<uint16_t> cores;             // Flattened.Cpu.ReservedCores (a set)
    std::vector<std::pair<std::string, int>> ports;   // (HostIP, port) held (NetworkIndex.AddAllocs)
    bool has_net = false;                    // Flattened.Networks non-empty
    std::string dev;                         // Device of its networks (Networks[0].Device): the key of its
                                             // UsedBandwidth and of its PreemptForNetwork group
};

struct OConstraint { std::string l, r, op; };
struct OAffinity { std::string l, r, op; int32_t weight; };
struct ODevReq {   // structs.RequestedDevice
    std::string name;
    uint64_t count;
    std::vector<OConstraint> constraints;
    std::vector<OAffinity> affinities;
};

struct OTask {
    std::string name, driver;
    int64_t cpu, mem, mem_max;
    int32_t cores;
    uint32_t lifecycle;
    bool has_network; int32_t net_mbits, net_dyn, net_reserved;
    std::vector<std::pair<int, std::string>> rports;   // the task network's ReservedPorts (Value, Label)
    std::vector<const pe_constraint*> constraints;
    std::vector<const pe_affinity*> affinities;
    int n_devices;
    std::vector<ODevReq> devices;
};
struct OSpreadTarget { std::string value; int32_t percent; };
struct OSpread { std::string attribute; int8_t weight; std::vector<OSpreadTarget> targets; };

struct OTaskGroup {
    std::string name;
    int32_t count;
    int64_t disk;
    std::vector<OConstraint> constraints;
    std::vector<OAffinity> affinities;
    std::vector<OSpread> spreads;
    std::vector<OTask> tasks;
    std::vector<std::vector<OConstraint>> task_constraints;
    std::vector<std::vector<OAffinity>> task_affinities;
    bool has_network; std::string net_mode, net_host_network;
    int32_t net_dyn, net_reserved;
    std::vector<std::pair<int, std::string>> rports;     // ReservedPorts (Value, Label)
    std::vector<std::pair<std::string, bool>> volumes;   // host volume requests (source, read only)
    bool csi;
};

struct OJob {
    std::string id, ns;
    uint32_t type;
    int32_t priority;
    uint64_t version;
    std::vector<OConstraint> constraints;
    std::vector<OAffinity> affinities;
    std::vector<OSpread> spreads;
    std::vector<OTaskGroup> tgs;
};

// ---------------------------------------------------------------------------
// AllocMetric (structs.go:9826-10026) — counters only
// Per-row outcome trace of one Select (oracle_full_pass): 1 filtered,
// 2 exhausted, 0 option with its FinalScore.
static thread_local uint8_t* g_trace_status = nullptr;
static thread_local double* g_trace_score = nullptr;

// NodeScoreMeta (structs.go:10030-10035) and kheap.ScoreHeap
// (lib/kheap/score_heap.go) over Go's container/heap (up / down / Fix / Pop).
struct NodeScoreMeta {
    std::string node_id;
    std::map<std::string, double> scores;
    double norm = 0;
};

struct GoScoreHeap {
    std::vector<NodeScoreMeta> items;
    int capacity = 5;   // MaxRetainedNodeScores
    bool Less(int i, int j) const { return items[i].norm < items[j].norm; }
    void Swap(int i, int j) { std::swap(items[i], items[j]); }
    int Len() const { return (int)items.size(); }
    void up(int j) {
        for (;;) {
            int i = (j - 1) / 2;   // Go integer division truncates toward zero
            if (i == j || !Less(j, i)) break;
            Swap(i, j);
            j = i;
        }
    }
    bool down(int i0, int n) {
        int i = i0;
        for (;;) {
            int j1 = 2 * i + 1;
            if (j1 >= n || j1 < 0) break;
            int j = j1;
            int j2 = j1 + 1;
            if (j2 < n && Less(j2, j1)) j = j2;
            if (!Less(j, i)) break;
            Swap(i, j);
            i = j;
        }
        return i > i0;
    }
    void Fix(int i) { if (!down(i, Len())) up(i); }
    void HeapPush(const NodeScoreMeta& x) {   // heap.Push(h, x)
        if (Len() < capacity) {
            items.push_back(x);
        } else if (x.norm > items[0].norm) {
            items[0] = x;
            Fix(0);
        }
        up(Len() - 1);
    }
    NodeScoreMeta HeapPop() {                  // heap.Pop(h)
        int n = Len() - 1;
        Swap(0, n);
        down(0, n);
        NodeScoreMeta it = items.back();
        items.pop_back();
        return it;
    }
    std::vector<NodeScoreMeta> GetItemsReverse() {
        std::vector<NodeScoreMeta> ret(Len());
        int i = Len() - 1;
        while (Len() > 0) ret[i--] = HeapPop();
        return ret;
    }
};

struct Metrics {
    uint32_t evaluated = 0, filtered = 0, exhausted = 0;
    std::map<std::string, int> class_filtered, constraint_filtered, class_exhausted, dimension_exhausted;
    std::unique_ptr<NodeScoreMeta> meta;
    GoScoreHeap top;
    void ScoreNode(const ONode* n, const std::string& name, double score) {   // structs.go:9977-10001
        if (!meta || meta->node_id != n->id) {
            meta.reset(new NodeScoreMeta());
            meta->node_id = n->id;
        }
        if (name == "normalized-score") {
            meta->norm = score;
            top.HeapPush(*meta);
            meta.reset();
        } else {
            meta->scores[name] = score;
        }
    }
    void EvaluateNode() { evaluated++; }
    void FilterNode(const ONode* n, const std::string& c) {   // structs.go:9907-9921
        filtered++;
        if (n && !n->node_class.empty()) class_filtered[n->node_class]++;
        if (!c.empty()) constraint_filtered[c]++;
        if (g_trace_status && n) g_trace_status[n->row] = 1;
    }
    void ExhaustedNode(const ONode* n, const std::string& d) {   // structs.go:9923-9937
        exhausted++;
        if (n && !n->node_class.empty()) class_exhausted[n->node_class]++;
        if (!d.empty()) dimension_exhausted[d]++;
        if (g_trace_status && n) g_trace_status[n->row] = 2;
    }
    // "KIND\tKEY\tCOUNT\n" lines, KIND in CF/KF/CE/DE, maps in key order
    std::string Text() const {
        std::string out;
        auto put = [&](const char* k, const std::map<std::string, int>& m) {
            for (auto& kv : m) out += std::string(k) + "\t" + kv.first + "\t" + std::to_string(kv.second) + "\n";
        };
        put("CF", class_filtered); put("KF", constraint_filtered);
        put("CE", class_exhausted); put("DE", dimension_exhausted);
        GoScoreHeap h = top;   // PopulateScoreMetaData
        auto items = h.GetItemsReverse();
        char num[64];
        for (size_t i = 0; i < items.size(); i++) {
            snprintf(num, sizeof num, "%.17g", items[i].norm);
            out += "SM\t" + std::to_string(i) + "\t" + items[i].node_id + "\t" + num + "\t";
            bool first = true;
            for (auto& kv : items[i].scores) {
                snprintf(num, sizeof num, "%.17g", kv.second);
                out += (first ? "" : ",") + kv.first + "=" + num;
                first = false;
            }
            out += "\n";
        }
        return out;
    }
};

enum ClassFeas { kUnknown = 0, kIneligible = 1, kEligible = 2, kEscaped = 3 };

// EvalEligibility (context.go:190-345)
struct Eligibility {
    std::map<std::string, int> job;
    bool job_escaped = false;
    std::map<std::string, std::map<std::string, int>> tgs;
    std::map<std::string, bool> tg_escaped;

    static bool target_escapes(const std::string& t) {
        return t.rfind("${node.unique.", 0) == 0 || t.rfind("${attr.unique.", 0) == 0 ||
               t.rfind("${meta.unique.", 0) == 0;
    }
    static bool any_escaped(const std::vector<OConstraint>& cs) {
        for (auto& c : cs) if (target_escapes(c.l) || target_escapes(c.r)) return true;
        return false;
    }
    void SetJob(const OJob& j) {
        job_escaped = any_escaped(j.constraints);
        for (auto& tg : j.tgs) {
            std::vector<OConstraint> cs = tg.constraints;
            for (auto& tc : tg.task_constraints) cs.insert(cs.end(), tc.begin(), tc.end());
            tg_escaped[tg.name] = any_escaped(cs);
        }
    }
    int JobStatus(const std::string& cls) {
        if (job_escaped) return kEscaped;
        auto it = job.find(cls);
        return it == job.end() ? kUnknown : it->second;
    }
    void SetJobEligibility(bool e, const std::string& cls) { job[cls] = e ? kEligible : kIneligible; }
    int TaskGroupStatus(const std::string& tg, const std::string& cls) {
        auto e = tg_escaped.find(tg);
        if (e != tg_escaped.end() && e->second) return kEscaped;
        auto it = tgs.find(tg);
        if (it != tgs.end()) {
            auto jt = it->second.find(cls);
            if (jt != it->second.end()) return jt->second;
        }
        return kUnknown;
    }
    void SetTaskGroupEligibility(bool e, const std::string& tg, const std::string& cls) {
        tgs[tg][cls] = e ? kEligible : kIneligible;
    }
};

// ---------------------------------------------------------------------------
// State + Plan + EvalContext
struct State {
    std::vector<std::string> strs;
    std::vector<ONode> nodes;
    std::vector<OAlloc> allocs;
    std::vector<std::vector<int>> allocs_by_node;   // indices into allocs
};

struct Plan {
    std::map<int, std::vector<OAlloc>> node_allocation;   // NodeAllocation
    std::map<int, std::vector<OAlloc>> node_update;       // NodeUpdate (stops)
    std::map<int, std::vector<OAlloc>> node_preemptions;  // NodePreemptions
};

struct EvalContext {
    const State* state = nullptr;
    Plan plan;
    Metrics metrics;
    Eligibility elig;
    orasem::Caches caches;
    uint64_t next_alloc_id = 1ull << 40;

    void Reset() { metrics = Metrics(); }

    // EvalContext.ProposedAllocs (context.go:120-157): non-terminal state allocs
    // of the node, minus planned stops, plus planned placements (by ID).
    std::vector<const OAlloc*> ProposedAllocs(int row) const {
        std::map<uint64_t, const OAlloc*> ids;
        std::set<uint64_t> removed;
        auto up = plan.node_update.find(row);
        if (up != plan.node_update.end()) for (auto& a : up->second) removed.insert(a.id);
        auto pp = plan.node_preemptions.find(row);
        if (pp != plan.node_preemptions.end()) for (auto& a : pp->second) removed.insert(a.id);
        for (int ai : state->allocs_by_node[row]) {
            const OAlloc& a = state->allocs[ai];
            if (a.terminal) continue;              // AllocsByNodeTerminal(ws, node, false)
            if (removed.count(a.id)) continue;
            ids[a.id] = &a;
        }
        auto pa = plan.node_allocation.find(row);
        if (pa != plan.node_allocation.end()) for (auto& a : pa->second) ids[a.id] = &a;
        std::vector<const OAlloc*> out;
        for (auto& kv : ids) out.push_back(kv.second);
        return out;
    }
};

// resolveTarget (feasible.go:748-781)
static Val resolve_target(const std::string& target, const ONode& n, bool* found) {
    Val v; v.is_nil = false;
    if (target.rfind("${", 0) != 0) { *found = true; v.s = target; return v; }
    if (target == "${node.unique.id}") { *found = true; v.s = n.id; return v; }
    if (target == "${node.datacenter}") { *found = true; v.s = n.dc; return v; }
    if (target == "${node.unique.name}") { *found = true; v.s = n.name; return v; }
    if (target == "${node.class}") { *found = true; v.s = n.node_class; return v; }
    auto strip = [&](const std::string& pre) {
        std::string s = target.substr(pre.size());
        if (!s.empty() && s.back() == '}') s.pop_back();
        return s;
    };
    if (target.rfind("${attr.", 0) == 0) {
        auto it = n.attrs.find(strip("${attr."));
        *found = it != n.attrs.end();
        v.s = *found ? it->second : "";
        return v;
    }
    if (target.rfind("${meta.", 0) == 0) {
        auto it = n.meta.find(strip("${meta."));
        *found = it != n.meta.end();
        v.s = *found ? it->second : "";
        return v;
    }
    *found = false; v.is_nil = true;
    return v;
}

static bool meets_constraint(EvalContext& ctx, const OConstraint& c, const ONode& n) {
    bool lf, rf;
    Val l = resolve_target(c.l, n, &lf), r = resolve_target(c.r, n, &rf);
    return orasem::check_constraint(ctx.caches, c.op, l, r, lf, rf);
}

// getProperty (propertyset.go:339-355)
static bool get_property(const ONode* n, const std::string& prop, std::string* out) {
    if (!n || prop.empty()) return false;
    bool ok;
    Val v = resolve_target(prop, *n, &ok);
    if (!ok || v.is_nil) return false;
    *out = v.s;
    return true;
}

// ---------------------------------------------------------------------------
// Feasibility checkers
struct Checker { virtual ~Checker() {} virtual bool Feasible(const ONode& n) = 0; };

struct ConstraintChecker : Checker {
    EvalContext* ctx; std::vector<OConstraint> cs;
    bool Feasible(const ONode& n) override {
        for (auto& c : cs) {
            if (!meets_constraint(*ctx, c, n)) {
                ctx->metrics.FilterNode(&n, c.l + " " + c.op + " " + c.r);
                return false;
            }
        }
        return true;
    }
};

// DriverChecker (feasible.go:433-500); drivers visited in sorted order (the
// Go map order is random but the result is order independent).
struct DriverChecker : Checker {
    EvalContext* ctx; std::set<std::string> drivers;
    bool has(const ONode& n) {
        for (auto& d : drivers) {
            auto it = n.drivers.find(d);
            if (it != n.drivers.end()) {
                if (it->second.nil) return false;
                if (it->second.detected && it->second.healthy) continue;
                return false;
            }
            auto at = n.attrs.find("driver." + d);
            if (at == n.attrs.end()) return false;
            // strconv.ParseBool
            const std::string& v = at->second;
            bool enabled;
            if (v == "1" || v == "t" || v == "T" || v == "true" || v == "TRUE" || v == "True") enabled = true;
            else if (v == "0" || v == "f" || v == "F" || v == "false" || v == "FALSE" || v == "False") enabled = false;
            else return false;
            if (!enabled) return false;
        }
        return true;
    }
    bool Feasible(const ONode& n) override {
        if (has(n)) return true;
        ctx->metrics.FilterNode(&n, "missing drivers");
        return false;
    }
};

// HostVolumeChecker (feasible.go:130-207)
struct HostVolumeChecker : Checker {
    EvalContext* ctx; std::map<std::string, std::vector<bool>> volumes;   // source -> read only flags
    bool has(const ONode& n) {
        if (volumes.empty()) return true;
        if (volumes.size() > n.host_volumes.size()) return false;
        for (auto& kv : volumes) {
            auto it = n.host_volumes.find(kv.first);
            if (it == n.host_volumes.end()) return false;
            if (!it->second) continue;
            for (bool ro : kv.second) if (!ro) return false;
        }
        return true;
    }
    bool Feasible(const ONode& n) override {
        if (has(n)) return true;
        ctx->metrics.FilterNode(&n, "missing compatible host volumes");
        return false;
    }
};

// ---------------------------------------------------------------------------
// Devices: RequestedDevice.ID + DeviceIdTuple.Matches (structs.go:2738-2761,
// 3130-3148), resolveDeviceTarget / nodeDeviceMatches (feasible.go:1278-1330).
static bool device_id_matches(const ODev& d, const std::string& req) {
    if (req.empty()) return false;   // RequestedDevice.ID() == nil
    std::vector<std::string> parts;
    size_t start = 0;
    while (parts.size() < 2) {
        size_t k = req.find('/', start);
        if (k == std::string::npos) break;
        parts.push_back(req.substr(start, k - start));
        start = k + 1;
    }
    parts.push_back(req.substr(start));
    std::string vendor, type, name;
    if (parts.size() == 1) type = parts[0];
    else if (parts.size() == 2) { vendor = parts[0]; type = parts[1]; }
    else { vendor = parts[0]; type = parts[1]; name = parts[2]; }
    if (!name.empty() && name != d.name) return false;
    if (!vendor.empty() && vendor != d.vendor) return false;
    if (!type.empty() && type != d.type) return false;
    return true;
}

static orasem::Attr resolve_device_target(const std::string& t, const ODev& d, bool* found) {
    orasem::Attr a;
    *found = true;
    if (t.rfind("${", 0) != 0) return orasem::parse_attribute(t);
    if (t == "${device.model}") { a.kind = orasem::Attr::Str; a.s = d.name; return a; }
    if (t == "${device.vendor}") { a.kind = orasem::Attr::Str; a.s = d.vendor; return a; }
    if (t == "${device.type}") { a.kind = orasem::Attr::Str; a.s = d.type; return a; }
    if (t.rfind("${device.attr.", 0) == 0) {
        std::string k = t.substr(14);
        if (!k.empty() && k.back() == '}') k.pop_back();
        auto it = d.attrs.find(k);
        if (it == d.attrs.end()) { *found = false; return a; }
        return it->second;
    }
    *found = false;
    return a;
}

static bool dev_check(orasem::Caches& c, const std::string& op, const std::string& l, const std::string& r,
                      const ODev& d) {
    bool lf, rf;
    orasem::Attr lv = resolve_device_target(l, d, &lf), rv = resolve_device_target(r, d, &rf);
    return orasem::check_attribute_constraint(c, op, lv, rv, lf, rf);
}

static bool node_device_matches(orasem::Caches& c, const ODev& d, const ODevReq& req) {
    if (!device_id_matches(d, req.name)) return false;
    for (auto& k : req.constraints)
        if (!dev_check(c, k.op, k.l, k.r, d)) return false;
    return true;
}

// DeviceChecker (feasible.go:1171-1274). The reference walks a map of device
// groups; groups are visited here in node order.
struct DeviceChecker : Checker {
    EvalContext* ctx = nullptr;
    std::vector<const ODevReq*> required;
    bool has(const ONode& n) {
        if (required.empty()) return true;
        if (n.devs.empty()) return false;
        std::vector<int64_t> avail(n.devs.size(), 0);
        for (size_t g = 0; g < n.devs.size(); g++) avail[g] = n.devs[g].healthy;
        for (const ODevReq* req : required) {
            bool ok = false;
            for (size_t g = 0; g < n.devs.size(); g++) {
                if (n.devs[g].healthy == 0) continue;   // not in the `available` map
                if (avail[g] == 0) continue;
                if ((uint64_t)avail[g] < req->count) continue;
                if (node_device_matches(ctx->caches, n.devs[g], *req)) {
                    avail[g] -= (int64_t)req->count;
                    ok = true;
                    break;
                }
            }
            if (!ok) return false;
        }
        return true;
    }
    bool Feasible(const ONode& n) override {
        if (has(n)) return true;
        ctx->metrics.FilterNode(&n, "missing devices");
        return false;
    }
};

// deviceAllocator over a DeviceAccounter (device.go:13-131, devices.go:25-100),
// counted per device group: instances in use by proposed allocs / reservations.
struct DevAlloc {
    const ONode* n = nullptr;
    std::vector<int64_t> used;
    explicit DevAlloc(const ONode* node) : n(node), used(node->devs.size(), 0) {}
    int64_t free_count(size_t g) const { return std::max<int64_t>(0, (int64_t)n->devs[g].healthy - used[g]); }
    void AddAllocs(const std::vector<const OAlloc*>& allocs) {
        for (const OAlloc* a : allocs) {
            if (a->terminal) continue;
            for (auto& d : a->devs)
                if (d.first >= 0 && (size_t)d.first < used.size()) used[(size_t)d.first] += d.second;
        }
    }
    // AddReserved of an offer: marks `count` instances used; instances already
    // in use (an offer made by a fresh allocator after preemption, rank.go:470)
    // do not change the free count.
    void AddReserved(int g, int64_t count) { used[(size_t)g] += std::min<int64_t>(count, free_count((size_t)g)); }
    // AssignDevice: best-scoring matching group with enough free instances;
    // equal scores -> the later group (map order in the reference).
    bool Assign(orasem::Caches& c, const ODevReq& req, int* group, double* matched, std::string* err) const {
        if (n->devs.empty()) { *err = "no devices available"; return false; }
        if (req.count == 0) { *err = "invalid request of zero devices"; return false; }
        int offer = -1;
        double offer_score = 0, offer_matched = 0;
        for (size_t g = 0; g < n->devs.size(); g++) {
            if ((uint64_t)free_count(g) < req.count) continue;
            if (!node_device_matches(c, n->devs[g], req)) continue;
            double choice = 0, sum = 0;
            if (!req.affinities.empty()) {
                double total = 0;
                for (auto& a : req.affinities) {
                    total += std::fabs((double)a.weight);
                    if (!dev_check(c, a.op, a.l, a.r, n->devs[g])) continue;
                    choice += (double)a.weight;
                    sum += (double)a.weight;
                }
                choice /= total;
            }
            if (offer >= 0 && choice < offer_score) continue;
            offer = (int)g;
            offer_score = choice;
            offer_matched = sum;
        }
        if (offer < 0) { *err = "no devices match request"; return false; }
        *group = offer;
        *matched = offer_matched;
        return true;
    }
};

// NetworkChecker (feasible.go:339-429)
struct NetworkChecker : Checker {
    EvalContext* ctx; std::string mode = "host"; std::vector<std::string> port_networks; bool has_ports = false;
    bool has_network(const ONode& n) {
        for (auto& nw : n.nets) {
            std::string m = nw.mode.empty() ? "host" : nw.mode;
            if (m == mode) return true;
        }
        return false;
    }
    bool Feasible(const ONode& n) override {
        if (!has_network(n)) {
            if (mode == "bridge") {
                auto it = n.attrs.find("nomad.version");
                if (it != n.attrs.end()) {
                    orasem::Version v;
                    if (orasem::new_version(it->second, true, &v)) {
                        orasem::Version c; orasem::new_version("0.12", false, &c);
                        if (orasem::prerelease_check(v, c) && orasem::version_compare(v, c) == -1) return true;
                    }
                }
            }
            ctx->metrics.FilterNode(&n, "missing network");
            return false;
        }
        if (has_ports) {
            for (auto& hn : port_networks) {
                if (hn.empty()) continue;
                bool ok; Val v = resolve_target(hn, n, &ok);
                if (!ok) { ctx->metrics.FilterNode(&n, "invalid host network"); return false; }
                bool found = false;
                for (auto& a : n.aliases) if (a == v.s) { found = true; break; }
                if (!found) { ctx->metrics.FilterNode(&n, "missing host network"); return false; }
            }
        }
        return true;
    }
};

// ---------------------------------------------------------------------------
// Feasible iterators
struct FeasibleIterator { virtual ~FeasibleIterator() {} virtual const ONode* Next() = 0; virtual void Reset() = 0; };

// StaticIterator (feasible.go:74-117)
struct StaticIterator : FeasibleIterator {
    EvalContext* ctx; std::vector<const ONode*> nodes; int offset = 0, seen = 0;
    const ONode* Next() override {
        int n = (int)nodes.size();
        if (offset == n || seen == n) {
            if (seen != n) offset = 0;
            else return nullptr;
        }
        int o = offset;
        offset++; seen++;
        ctx->metrics.EvaluateNode();
        return nodes[o];
    }
    void Reset() override { seen = 0; }
    void SetNodes(const std::vector<const ONode*>& ns) { nodes = ns; offset = 0; seen = 0; }
};

// FeasibilityWrapper (feasible.go:1026-1169); no availability checkers (CSI excluded).
struct FeasibilityWrapper : FeasibleIterator {
    EvalContext* ctx; FeasibleIterator* source;
    std::vector<Checker*> job_checkers, tg_checkers;
    std::string tg;
    const ONode* Next() override {
        Eligibility& e = ctx->elig;
        for (;;) {
        outer:
            const ONode* option = source->Next();
            if (!option) return nullptr;
            bool job_escaped = false, job_unknown = false;
            switch (e.JobStatus(option->computed_class)) {
                case kIneligible: ctx->metrics.FilterNode(option, "computed class ineligible"); continue;
                case kEscaped: job_escaped = true; break;
                case kUnknown: job_unknown = true; break;
            }
            for (Checker* c : job_checkers) {
                if (!c->Feasible(*option)) {
                    if (!job_escaped) e.SetJobEligibility(false, option->computed_class);
                    goto outer;
                }
            }
            if (!job_escaped && job_unknown) e.SetJobEligibility(true, option->computed_class);
            bool tg_escaped = false, tg_unknown = false;
            switch (e.TaskGroupStatus(tg, option->computed_class)) {
                case kIneligible: ctx->metrics.FilterNode(option, "computed class ineligible"); continue;
                case kEligible: return option;    // available() is always true without CSI
                case kEscaped: tg_escaped = true; break;
                case kUnknown: tg_unknown = true; break;
            }
            for (Checker* c : tg_checkers) {
                if (!c->Feasible(*option)) {
                    if (!tg_escaped) e.SetTaskGroupEligibility(false, tg, option->computed_class);
                    goto outer;
                }
            }
            if (!tg_escaped && tg_unknown) e.SetTaskGroupEligibility(true, tg, option->computed_class);
            return option;
        }
    }
    void Reset() override { source->Reset(); }
};

// DistinctHostsIterator (feasible.go:502-599)
struct DistinctHostsIterator : FeasibleIterator {
    EvalContext* ctx; FeasibleIterator* source;
    const OJob* job = nullptr; const OTaskGroup* tg = nullptr;
    bool tg_dh = false, job_dh = false;
    static bool has_dh(const std::vector<OConstraint>& cs) {
        for (auto& c : cs) if (c.op == "distinct_hosts") return true;
        return false;
    }
    void SetJob(const OJob* j) { job = j; job_dh = has_dh(j->constraints); }
    void SetTaskGroup(const OTaskGroup* t) { tg = t; tg_dh = has_dh(t->constraints); }
    bool satisfies(const ONode& n) {
        if (!(job_dh || tg_dh)) return true;
        for (const OAlloc* a : ctx->ProposedAllocs(n.row)) {
            bool jc = a->job_id == job->id, tc = a->tg == tg->name;
            if ((job_dh && jc) || (jc && tc)) return false;
        }
        return true;
    }
    const ONode* Next() override {
        for (;;) {
            const ONode* o = source->Next();
            if (!o || !(job_dh || tg_dh)) return o;
            if (!satisfies(*o)) { ctx->metrics.FilterNode(o, "distinct_hosts"); continue; }
            return o;
        }
    }
    void Reset() override { source->Reset(); }
};

// propertySet (propertyset.go:14-355)
struct PropertySet {
    EvalContext* ctx;
    std::string job_id, ns, task_group, target;
    uint64_t allowed = 0;
    bool error = false; std::string error_msg;
    std::map<std::string, uint64_t> existing, proposed, cleared;

    bool keep(const OAlloc& a, bool filter_terminal) const {
        if (filter_terminal && a.terminal) return false;
        if (!task_group.empty() && a.tg != task_group) return false;
        return true;
    }
    void populate_existing() {
        // AllocsByJob(ws, ns, jobID, false): the job's allocs in the state store
        for (const OAlloc& a : ctx->state->allocs) {
            if (a.ns != ns || a.job_id != job_id) continue;
            if (!keep(a, true)) continue;
            std::string v;
            if (get_property(&ctx->state->nodes[a.node_row], target, &v)) existing[v]++;
        }
    }
    void PopulateProposed() {
        proposed.clear(); cleared.clear();
        for (auto& kv : ctx->plan.node_update)
            for (auto& a : kv.second) {
                if (!keep(a, false)) continue;
                std::string v;
                if (get_property(&ctx->state->nodes[a.node_row], target, &v)) cleared[v]++;
            }
        for (auto& kv : ctx->plan.node_allocation)
            for (auto& a : kv.second) {
                if (!keep(a, true)) continue;
                std::string v;
                if (get_property(&ctx->state->nodes[a.node_row], target, &v)) proposed[v]++;
            }
        for (auto& kv : proposed) {
            auto it = cleared.find(kv.first);
            if (it == cleared.end()) continue;
            if (it->second == 0) cleared.erase(it);
            else if (it->second > 1) it->second--;
        }
    }
    void set_target(const std::string& attr, uint64_t allowed_count, const std::string& tg) {
        if (!tg.empty()) task_group = tg;
        target = attr;
        allowed = allowed_count;
        populate_existing();
        PopulateProposed();
    }
    void SetConstraint(const OConstraint& c, const std::string& tg) {
        uint64_t allowed_count = 1;
        if (!c.r.empty()) {
            // strconv.ParseUint(v, 10, 64)
            bool ok = !c.r.empty();
            unsigned __int128 v = 0;
            for (char ch : c.r) {
                if (ch < '0' || ch > '9') { ok = false; break; }
                v = v * 10 + (ch - '0');
                if (v > UINT64_MAX) { ok = false; break; }
            }
            if (!ok) { error = true; error_msg = "failed to convert RTarget"; return; }
            allowed_count = (uint64_t)v;
        }
        set_target(c.l, allowed_count, tg);
    }
    std::map<std::string, uint64_t> CombinedUse() const {
        std::map<std::string, uint64_t> use;
        for (auto& kv : existing) use[kv.first] += kv.second;
        for (auto& kv : proposed) use[kv.first] += kv.second;
        for (auto& kv : cleared) {
            auto it = use.find(kv.first);
            if (it == use.end()) continue;
            it->second = it->second >= kv.second ? it->second - kv.second : 0;
        }
        return use;
    }
    // UsedCount: returns false with an error message when unresolvable
    bool UsedCount(const ONode& n, std::string* value, uint64_t* used, std::string* err) const {
        if (error) { *err = error_msg; return false; }
        if (!get_property(&n, target, value)) { *err = "missing property \"" + target + "\""; return false; }
        auto use = CombinedUse();
        auto it = use.find(*value);
        *used = it == use.end() ? 0 : it->second;
        return true;
    }
    bool SatisfiesDistinctProperties(const ONode& n, std::string* reason) const {
        std::string v, err; uint64_t used = 0;
        if (!UsedCount(n, &v, &used, &err)) { *reason = err; return false; }
        if (used < allowed) return true;
        *reason = "distinct_property: " + target + "=" + v + " used by " + std::to_string(used) + " allocs";
        return false;
    }
};

// DistinctPropertyIterator (feasible.go:601-704)
struct DistinctPropertyIterator : FeasibleIterator {
    EvalContext* ctx; FeasibleIterator* source;
    const OJob* job = nullptr; const OTaskGroup* tg = nullptr;
    bool has = false;
    std::vector<std::unique_ptr<PropertySet>> job_sets;
    std::map<std::string, std::vector<std::unique_ptr<PropertySet>>> group_sets;
    void SetJob(const OJob* j) {
        job = j;
        for (auto& c : j->constraints) {
            if (c.op != "distinct_property") continue;
            auto p = std::make_unique<PropertySet>();
            p->ctx = ctx; p->job_id = j->id; p->ns = j->ns;
            p->SetConstraint(c, "");
            job_sets.push_back(std::move(p));
        }
    }
    void SetTaskGroup(const OTaskGroup* t) {
        tg = t;
        if (!group_sets.count(t->name)) {
            auto& v = group_sets[t->name];
            for (auto& c : t->constraints) {
                if (c.op != "distinct_property") continue;
                auto p = std::make_unique<PropertySet>();
                p->ctx = ctx; p->job_id = job->id; p->ns = job->ns;
                p->SetConstraint(c, t->name);
                v.push_back(std::move(p));
            }
        }
        has = !job_sets.empty() || !group_sets[t->name].empty();
    }
    bool satisfies(const ONode& n, std::vector<std::unique_ptr<PropertySet>>& sets) {
        for (auto& ps : sets) {
            std::string reason;
            if (!ps->SatisfiesDistinctProperties(n, &reason)) { ctx->metrics.FilterNode(&n, reason); return false; }
        }
        return true;
    }
    const ONode* Next() override {
        for (;;) {
            const ONode* o = source->Next();
            if (!o || !has) return o;
            if (!satisfies(*o, job_sets) || !satisfies(*o, group_sets[tg->name])) continue;
            return o;
        }
    }
    void Reset() override {
        source->Reset();
        for (auto& p : job_sets) p->PopulateProposed();
        for (auto& kv : group_sets) for (auto& p : kv.second) p->PopulateProposed();
    }
};

// ---------------------------------------------------------------------------
// Rank iterators
struct RankedNode {
    const ONode* node;
    double final_score = 0;
    std::vector<double> scores;
    std::vector<const OAlloc*> preempted;   // PreemptedAllocs
    std::vector<std::pair<int, int>> offers; // device offers (group, instances) per request
    std::vector<uint16_t> cores;             // Cpu.ReservedCores of the tasks, in task order
    int64_t cpu = 0;                         // the alloc's CpuShares (SharesPerCore x cores for core tasks)
    std::vector<std::pair<std::string, int>> ports;   // static ports of the offer (HostIP, value)
    std::string net_dev;                     // Device of the task network's offer (AssignNetwork)
};

struct RankIterator { virtual ~RankIterator() {} virtual RankedNode* Next() = 0; virtual void Reset() = 0; };

// FeasibleRankIterator (rank.go:77-107)
struct FeasibleRankIterator : RankIterator {
    FeasibleIterator* source;
    std::vector<std::unique_ptr<RankedNode>> pool;
    RankedNode* Next() override {
        const ONode* o = source->Next();
        if (!o) return nullptr;
        pool.push_back(std::make_unique<RankedNode>());
        pool.back()->node = o;
        return pool.back().get();
    }
    void Reset() override { source->Reset(); pool.clear(); }
};

// The task group's resource ask: AllocatedResources.Comparable() (structs.go:3445-3487)
struct Ask { int64_t cpu, mem, disk; };
// spc >= 0: tasks asking reserved cores hold SharesPerCore x cores CpuShares
// (rank.go:461-463); spc < 0: their Resources.CPU (a commit without a Select)
static Ask tg_ask(const OTaskGroup& tg, bool oversub, int64_t spc = -1) {
    (void)oversub;
    int64_t sc_cpu = 0, sc_mem = 0, eph_cpu = 0, eph_mem = 0, main_cpu = 0, main_mem = 0, ps_cpu = 0, ps_mem = 0;
    for (auto& t : tg.tasks) {
        const int64_t cpu = (t.cores > 0 && spc >= 0) ? spc * t.cores : t.cpu;
        switch (t.lifecycle) {
            case PE_LC_MAIN: main_cpu += cpu; main_mem += t.mem; break;
            case PE_LC_PRESTART: eph_cpu += cpu; eph_mem += t.mem; break;
            case PE_LC_PRESTART_SIDECAR: sc_cpu += cpu; sc_mem += t.mem; break;
            case PE_LC_POSTSTOP: ps_cpu += cpu; ps_mem += t.mem; break;
            default: break;   // poststart hooks are not counted by Comparable()
        }
    }
    eph_cpu = std::max(eph_cpu, main_cpu); eph_mem = std::max(eph_mem, main_mem);
    eph_cpu = std::max(eph_cpu, ps_cpu); eph_mem = std::max(eph_mem, ps_mem);
    return Ask{sc_cpu + eph_cpu, sc_mem + eph_mem, tg.disk};
}

// structs.ParsePortRanges (funcs.go:495-548) as NetworkIndex uses it: a spec
// that does not parse reserves nothing; ports >= 65536 are dropped (the
// reference stops at the first one in map order; ascending is one legal order).
static std::vector<int> parse_port_ranges(const std::string& spec) {
    std::set<int> ports;
    if (spec.empty()) return {};
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
        for (uint64_t v = lo; v <= hi && v < 65536; v++) ports.insert((int)v);
        b = e + 1;
    }
    return std::vector<int>(ports.begin(), ports.end());
}

// NetworkIndex contribution of an alloc of this task group (network.go:144-193):
// allocs with task-group ports only count their ports; otherwise task networks.
static void tg_net_contrib(const OTaskGroup& tg, int32_t* mbits, int32_t* dyn) {
    *mbits = 0; *dyn = 0;
    if (tg.has_network && tg.net_dyn + tg.net_reserved > 0) {
        *dyn = tg.net_dyn;
        for (auto& p : tg.rports) *dyn += (p.first >= 20000 && p.first <= 32000) ? 1 : 0;
        return;
    }
    for (auto& t : tg.tasks) if (t.has_network) { *mbits += t.net_mbits; *dyn += t.net_dyn; }
}

// Go 1.16 sort.Slice (sort/zsortfunc.go: quickSort_func with doPivot_func,
// medianOfThree_func, heapSort_func, insertionSort_func). Not stable: the
// order of equal elements is part of the reference's behaviour.
template <class T, class Less>
struct GoSort {
    std::vector<T>& d;
    Less less;
    bool L(int i, int j) { return less(d[(size_t)i], d[(size_t)j]); }
    void S(int i, int j) { std::swap(d[(size_t)i], d[(size_t)j]); }
    void insertion(int a, int b) {
        for (int i = a + 1; i < b; i++)
            for (int j = i; j > a && L(j, j - 1); j--) S(j, j - 1);
    }
    void sift(int lo, int hi, int first) {
        int root = lo;
        for (;;) {
            int child = 2 * root + 1;
            if (child >= hi) return;
            if (child + 1 < hi && L(first + child, first + child + 1)) child++;
            if (!L(first + root, first + child)) return;
            S(first + root, first + child);
            root = child;
        }
    }
    void heap(int a, int b) {
        int first = a, lo = 0, hi = b - a;
        for (int i = (hi - 1) / 2; i >= 0; i--) sift(i, hi, first);
        for (int i = hi - 1; i >= 0; i--) { S(first, first + i); sift(lo, i, first); }
    }
    void median3(int m1, int m0, int m2) {
        if (L(m1, m0)) S(m1, m0);
        if (L(m2, m1)) { S(m2, m1); if (L(m1, m0)) S(m1, m0); }
    }
    void pivot(int lo, int hi, int* midlo, int* midhi) {
        int m = (int)((unsigned)(lo + hi) >> 1);
        if (hi - lo > 40) {
            int s = (hi - lo) / 8;
            median3(lo, lo + s, lo + 2 * s);
            median3(m, m - s, m + s);
            median3(hi - 1, hi - 1 - s, hi - 1 - 2 * s);
        }
        median3(lo, m, hi - 1);
        int pv = lo, a = lo + 1, c = hi - 1;
        for (; a < c && L(a, pv); a++) {}
        int b = a;
        for (;;) {
            for (; b < c && !L(pv, b); b++) {}
            for (; b < c && L(pv, c - 1); c--) {}
            if (b >= c) break;
            S(b, c - 1);
            b++; c--;
        }
        bool protect = hi - c < 5;
        if (!protect && hi - c < (hi - lo) / 4) {
            int dups = 0;
            if (!L(pv, hi - 1)) { S(c, hi - 1); c++; dups++; }
            if (!L(b - 1, pv)) { b--; dups++; }
            if (!L(m, pv)) { S(m, b - 1); b--; dups++; }
            protect = dups > 1;
        }
        if (protect) {
            for (;;) {
                for (; a < b && !L(b - 1, pv); b--) {}
                for (; a < b && L(a, pv); a++) {}
                if (a >= b) break;
                S(a, b - 1);
                a++; b--;
            }
        }
        S(pv, b - 1);
        *midlo = b - 1; *midhi = c;
    }
    void quick(int a, int b, int depth) {
        while (b - a > 12) {
            if (depth == 0) { heap(a, b); return; }
            depth--;
            int mlo, mhi;
            pivot(a, b, &mlo, &mhi);
            if (mlo - a < b - mhi) { quick(a, mlo, depth); a = mhi; }
            else { quick(mhi, b, depth); b = mlo; }
        }
        if (b - a > 1) {
            for (int i = a + 6; i < b; i++) if (L(i, i - 6)) S(i, i - 6);
            insertion(a, b);
        }
    }
};
template <class T, class Less>
static void go_sort_slice(std::vector<T>& v, Less less) {
    int n = (int)v.size(), depth = 0;
    for (int i = n; i > 0; i >>= 1) depth++;
    GoSort<T, Less> g{v, less};
    g.quick(0, n, depth * 2);
}

// structs.RemoveAllocs (funcs.go:47-64): swap-with-last removal (reorders).
static std::vector<const OAlloc*> remove_allocs(std::vector<const OAlloc*> v, const std::vector<const OAlloc*>& rm) {
    std::set<uint64_t> ids;
    for (auto* a : rm) ids.insert(a->id);
    int n = (int)v.size();
    for (int i = 0; i < n; i++) {
        if (ids.count(v[(size_t)i]->id)) {
            v[(size_t)i] = v[(size_t)n - 1];
            i--; n--;
        }
    }
    v.resize((size_t)n);
    return v;
}

// ComparableResources restricted to the dimensions Superset checks (cpu,
// memory, disk; structs.go:3891-3906).
struct CRes {
    int64_t cpu = 0, mem = 0, disk = 0;
    void add(const CRes& o) { cpu += o.cpu; mem += o.mem; disk += o.disk; }
    void sub(const CRes& o) { cpu -= o.cpu; mem -= o.mem; disk -= o.disk; }
    bool superset(const CRes& o) const { return cpu >= o.cpu && mem >= o.mem && disk >= o.disk; }
};
static CRes res_of(const OAlloc* a) { return CRes{a->cpu, a->mem, a->disk}; }

// basicResourceDistance / scoreForTaskGroup (preemption.go:603-651)
static double basic_distance(const CRes& ask, const CRes& used) {
    double mc = 0, cc = 0, dc = 0;
    if (ask.mem > 0) mc = ((double)ask.mem - (double)used.mem) / (double)ask.mem;
    if (ask.cpu > 0) cc = ((double)ask.cpu - (double)used.cpu) / (double)ask.cpu;
    if (ask.disk > 0) dc = ((double)ask.disk - (double)used.disk) / (double)ask.disk;
    return std::sqrt(gomath::pow(mc, 2) + gomath::pow(cc, 2) + gomath::pow(dc, 2));
}
static double score_for_tg(const CRes& ask, const CRes& used, int max_parallel, int num_preempted) {
    double pen = 0.0;
    if (max_parallel > 0 && num_preempted >= max_parallel) pen = (double)((num_preempted + 1) - max_parallel) * 50.0;
    return basic_distance(ask, used) + pen;
}

// filterAndGroupPreemptibleAllocs (preemption.go:661-697)
static std::vector<std::pair<int, std::vector<const OAlloc*>>> group_preemptible(int job_priority,
                                                                              const std::vector<const OAlloc*>& cur) {
    std::map<int, std::vector<const OAlloc*>> by;
    for (const OAlloc* a : cur) {
        if (job_priority - a->priority < 10) continue;
        by[a->priority].push_back(a);
    }
    std::vector<std::pair<int, std::vector<const OAlloc*>>> out(by.begin(), by.end());   // ascending priority
    return out;
}

// Preemptor (preemption.go:96-557) for one node of a BinPack pass.
struct Preemptor {
    int job_priority = 0;
    std::string job_id, job_ns;
    CRes remaining;
    std::vector<const OAlloc*> current;
    std::map<std::pair<std::string, std::string>, std::map<std::string, int>> preemptions;

    void SetNode(const ONode& n) { remaining = CRes{n.cpu - n.rcpu, n.mem - n.rmem, n.disk - n.rdisk}; }
    void SetPreemptions(const Plan& plan) {
        preemptions.clear();
        for (auto& kv : plan.node_preemptions)
            for (auto& a : kv.second) preemptions[{a.job_id, a.ns}][a.tg]++;
    }
    void SetCandidates(const std::vector<const OAlloc*>& allocs) {
        current.clear();
        for (const OAlloc* a : allocs) {
            if (a->job_id == job_id && a->ns == job_ns) continue;
            current.push_back(a);
        }
    }
    int num_preemptions(const OAlloc* a) const {
        auto it = preemptions.find({a->job_id, a->ns});
        if (it == preemptions.end()) return 0;
        auto jt = it->second.find(a->tg);
        return jt == it->second.end() ? 0 : jt->second;
    }

    // PreemptForTaskGroup (preemption.go:194-264)
    std::vector<const OAlloc*> ForTaskGroup(const CRes& ask) {
        CRes needed = ask;
        for (const OAlloc* a : current) remaining.sub(res_of(a));
        auto groups = group_preemptible(job_priority, current);
        std::vector<const OAlloc*> best;
        bool met = false;
        CRes available = remaining;
        for (auto& grp : groups) {
            auto& v = grp.second;
            while (!v.empty() && !met) {
                int idx = -1;
                double bd = DBL_MAX;
                for (size_t i = 0; i < v.size(); i++) {
                    double d = score_for_tg(needed, res_of(v[i]), v[i]->max_parallel, num_preemptions(v[i]));
                    if (d < bd) { bd = d; idx = (int)i; }
                }
                if (idx < 0) idx = 0;
                const OAlloc* closest = v[(size_t)idx];
                available.add(res_of(closest));
                met = available.superset(ask);
                best.push_back(closest);
                v[(size_t)idx] = v.back();
                v.pop_back();
                needed.sub(res_of(closest));
            }
            if (met) break;
        }
        if (!met) return {};
        // filterSuperset (preemption.go:699-731)
        go_sort_slice(best, [&](const OAlloc* x, const OAlloc* y) {
            return basic_distance(ask, res_of(x)) > basic_distance(ask, res_of(y));
        });
        CRes avail = remaining;
        std::vector<const OAlloc*> out;
        for (const OAlloc* a : best) {
            out.push_back(a);
            avail.add(res_of(a));
            if (avail.superset(ask)) break;
        }
        return out;
    }

    // PreemptForNetwork (preemption.go:270-455) for an ask of `needed` MBits and
    // the ReservedPorts values `ports`: candidates grouped by their network's
    // device (deviceToAllocs), filteredReservedPorts per device, the device's
    // AvailBandwidth and the NetworkIndex's UsedBandwidth of it. The reference
    // ranges over the deviceToAllocs map: with candidates on two devices its
    // answer depends on Go's map order, which is not modelled (Unsupported).
    // An alloc's ReservedPorts are the values of the ports it holds.
    std::vector<const OAlloc*> ForNetwork(int32_t needed, const std::map<std::string, int32_t>& avail_bw,
                                          const std::map<std::string, int32_t>& used_bw,
                                          const std::vector<int>& ports = {}) {
        if (current.empty()) return {};
        std::map<std::string, std::vector<const OAlloc*>> by_dev;
        std::map<std::string, std::set<int>> filtered_by_dev;   // ports of allocs too close in priority
        for (const OAlloc* a : current) {
            if (!a->has_net) continue;
            if (job_priority - a->priority < 10) {
                for (auto& pp : a->ports) filtered_by_dev[a->dev].insert(pp.second);
                continue;
            }
            by_dev[a->dev].push_back(a);
        }
        if (by_dev.empty()) return {};
        if (by_dev.size() > 1) throw Unsupported("network preemption candidates on several network devices (map order)");
        const std::string& device = by_dev.begin()->first;
        std::vector<const OAlloc*> dev = by_dev.begin()->second;
        const std::set<int>& filtered = filtered_by_dev[device];
        auto at = [](const std::map<std::string, int32_t>& m, const std::string& k) {
            auto it = m.find(k);
            return it == m.end() ? 0 : it->second;
        };
        const int32_t total = at(avail_bw, device);
        if (total < needed) return {};
        const int32_t free_bw = total - at(used_bw, device);
        int32_t pbw = 0;
        std::vector<const OAlloc*> best;
        if (!ports.empty()) {
            // the reserved ports first: usedPortToAlloc (the last holder in
            // candidate order wins), a port held by a filtered alloc fails
            std::map<int, const OAlloc*> holder;
            for (const OAlloc* a : dev)
                for (auto& pp : a->ports) holder[pp.second] = a;
            for (int v : ports) {
                auto it = holder.find(v);
                if (it != holder.end()) {
                    for (const OAlloc* b : best)
                        if (b == it->second) throw Unsupported("one alloc holding two static ports of the ask");
                    pbw += it->second->mbits;
                    best.push_back(it->second);
                } else if (filtered.count(v)) {
                    return {};
                }
            }
            dev = remove_allocs(dev, best);
        }
        bool met = pbw + free_bw >= needed;
        auto distance = [&](const OAlloc* a) {   // networkResourceDistance (preemption.go:627-635)
            return std::fabs((double)((int64_t)needed - (int64_t)a->mbits) / (double)needed);
        };
        if (!met) {
            for (auto& grp : group_preemptible(job_priority, dev)) {
                auto v = grp.second;
                go_sort_slice(v, [&](const OAlloc* x, const OAlloc* y) {   // distanceComparatorForNetwork
                    auto score = [&](const OAlloc* a) {                   // scoreForNetwork
                        double pen = 0.0;
                        const int num = num_preemptions(a);
                        if (a->max_parallel > 0 && num >= a->max_parallel)
                            pen = (double)((num + 1) - a->max_parallel) * 50.0;
                        return distance(a) + pen;
                    };
                    return score(x) < score(y);
                });
                for (const OAlloc* a : v) {
                    pbw += a->mbits;
                    best.push_back(a);
                    if (pbw + free_bw >= needed) { met = true; break; }
                }
                if (met) break;
            }
        }
        if (!met) return {};
        // filterSuperset with the network resource (MeetsRequirements is false
        // while either MBits figure is 0)
        go_sort_slice(best, [&](const OAlloc* x, const OAlloc* y) { return distance(x) > distance(y); });
        int32_t avail = free_bw;
        std::vector<const OAlloc*> out;
        for (const OAlloc* a : best) {
            out.push_back(a);
            avail += a->mbits;
            if (avail != 0 && needed != 0 && avail >= needed) break;
        }
        return out;
    }

    // PreemptForDevice + selectBestAllocs (preemption.go:472-601); device groups
    // in node order (a map in the reference).
    std::vector<const OAlloc*> ForDevice(orasem::Caches& c, const ONode& n, const ODevReq& req, const DevAlloc& da) {
        struct Grp { std::vector<const OAlloc*> allocs; std::map<uint64_t, int64_t> inst; bool used = false; };
        std::vector<Grp> grps(n.devs.size());
        for (const OAlloc* a : current) {
            for (auto& d : a->devs) {
                if (d.first < 0 || (size_t)d.first >= n.devs.size()) continue;
                if (!node_device_matches(c, n.devs[(size_t)d.first], req)) continue;
                Grp& g = grps[(size_t)d.first];
                g.used = true;
                g.allocs.push_back(a);
                g.inst[a->id] += d.second;
            }
        }
        const int64_t needed = (int64_t)req.count;
        struct Opt { std::vector<const OAlloc*> allocs; const std::map<uint64_t, int64_t>* inst; };
        std::vector<Opt> options;
        for (size_t gi = 0; gi < grps.size(); gi++) {
            if (!grps[gi].used) continue;
            auto byp = group_preemptible(job_priority, grps[gi].allocs);
            int64_t cnt = 0;
            std::vector<const OAlloc*> pre;
            bool done = false;
            for (auto& grp : byp) {
                for (const OAlloc* a : grp.second) {
                    cnt += grps[gi].inst[a->id];
                    pre.push_back(a);
                    if (cnt + da.free_count(gi) >= needed) { options.push_back(Opt{pre, &grps[gi].inst}); done = true; break; }
                }
                if (done) break;
            }
        }
        if (options.empty()) return {};
        int best_prio = INT32_MAX;
        std::vector<const OAlloc*> best;
        for (auto& o : options) {
            const auto& inst = *o.inst;
            go_sort_slice(o.allocs, [&](const OAlloc* x, const OAlloc* y) {
                return inst.at(x->id) > inst.at(y->id);
            });
            std::set<int> prios;
            int net = 0;
            int64_t got = 0;
            std::vector<const OAlloc*> filtered;
            for (const OAlloc* a : o.allocs) {
                if (got >= needed) break;
                got += inst.at(a->id);
                filtered.push_back(a);
                if (prios.insert(a->priority).second) net += a->priority;
            }
            if (net < best_prio) { best_prio = net; best = filtered; }
        }
        return best;
    }
};

// netPriority / preemptionScore (rank.go:808-844)
static double preemption_score(const std::vector<const OAlloc*>& allocs) {
    int sum = 0;
    double mx = 0.0;
    for (const OAlloc* a : allocs) {
        if ((double)a->priority > mx) mx = (double)a->priority;
        sum += a->priority;
    }
    const double net = mx + ((double)sum / mx);
    return 1.0 / (1 + gomath::exp(0.0048 * (net - 2048.0)));
}

// BinPackIterator (rank.go:149-531)
struct BinPackIterator : RankIterator {
    EvalContext* ctx; RankIterator* source;
    bool evict = false; int32_t priority = 0; std::string job_id, job_ns;
    const OTaskGroup* tg = nullptr;
    bool spread_algo = false, oversub = false;

    // NetworkIndex SetNode + AddAllocs: dynamic-range ports in use (counted
    // per node) and UsedBandwidth per device (network.go:92-230)
    static void index_usage(const ONode& n, const std::vector<const OAlloc*>& proposed, int32_t* dyn,
                            std::map<std::string, int32_t>* used_bw) {
        *dyn = n.reserved_dyn;
        used_bw->clear();
        for (const OAlloc* a : proposed) {
            if (a->terminal) continue;
            *dyn += a->dyn_ports;
            if (a->mbits) (*used_bw)[a->dev] += a->mbits;
        }
    }
    // AvailBandwidth: per device, the MBits of the last AvailNetworks entry
    // naming it (SetNode, network.go:108-114)
    static std::map<std::string, int32_t> avail_bandwidth(const ONode& n) {
        std::map<std::string, int32_t> m;
        for (auto& nw : n.nets) if (!nw.device.empty()) m[nw.device] = nw.mbits;
        return m;
    }

    static double score_fit(bool spread, const ONode& n, int64_t ucpu, int64_t umem) {
        double node_cpu = (double)n.cpu, node_mem = (double)n.mem;
        node_cpu -= (double)n.rcpu; node_mem -= (double)n.rmem;
        double fc = 1 - ((double)ucpu / node_cpu);
        double fm = 1 - ((double)umem / node_mem);
        double total = gomath::pow(10, fc) + gomath::pow(10, fm);
        double s = spread ? total - 2 : 20.0 - total;
        if (s > 18.0) s = 18.0; else if (s < 0) s = 0;
        return s;
    }

    RankedNode* Next() override {
        for (;;) {
            RankedNode* option = source->Next();
            if (!option) return nullptr;
            const ONode& n = *option->node;
            auto proposed = ctx->ProposedAllocs(n.row);
            // NetworkIndex: SetNode + AddAllocs
            int32_t used_dyn = 0;
            std::map<std::string, int32_t> used_bw;
            const std::map<std::string, int32_t> avail_bw = avail_bandwidth(n);
            index_usage(n, proposed, &used_dyn, &used_bw);
            DevAlloc dev(&n);
            dev.AddAllocs(proposed);
            double total_dev_w = 0.0, sum_dev_match = 0.0;
            std::vector<const OAlloc*> to_preempt;
            Preemptor pre;
            pre.job_priority = priority; pre.job_id = job_id; pre.job_ns = job_ns;
            pre.SetNode(n);
            pre.SetPreemptions(ctx->plan);
            option->ports.clear();
            option->net_dev.clear();
            // UsedPorts[ip] of the NetworkIndex (network.go:92-293): SetNode keys the
            // AvailNetworks' IP fields and the addresses (their ReservedPorts), then
            // marks ReservedHostPorts on every key; AddAllocs marks the proposed
            // allocs' ports; this BinPack's offers so far (option->ports) are added
            // by AddReservedPorts / AddReserved (idx_offers; a rebuilt index drops them).
            std::vector<std::pair<std::string, int>> idx_offers;
            auto port_used = [&](const std::vector<const OAlloc*>& prop, const std::string& ip, int v) {
                bool keyed = false;
                for (auto& nw : n.nets) if (!nw.device.empty() && nw.ip == ip) keyed = true;
                for (auto& ad : n.addrs)
                    if (ad.ip == ip) {
                        keyed = true;
                        for (int r : ad.reserved) if (r == v) return true;
                    }
                if (keyed) for (int r : n.reserved_host_ports) if (r == v) return true;
                for (const OAlloc* x : prop) {
                    if (x->terminal) continue;
                    for (auto& pp : x->ports) if (pp.first == ip && pp.second == v) return true;
                }
                for (auto& o : idx_offers) if (o.first == ip && o.second == v) return true;
                return false;
            };
            if (tg->has_network) {
                // AssignPorts (network.go:317-404): ReservedPorts first, on the first
                // address of the port's host network, then one free port in
                // [MinDynamicPort, MaxDynamicPort] per dynamic port; "" = an offer
                std::vector<int> rport_values;
                for (auto& rp : tg->rports) rport_values.push_back(rp.first);
                std::vector<std::pair<std::string, int>> offer;
                int32_t static_dyn = 0;
                auto assign_ports = [&](const std::vector<const OAlloc*>& prop) -> std::string {
                    offer.clear();
                    static_dyn = 0;
                    for (auto& rp : tg->rports) {
                        const ONode::Addr* ad = nullptr;
                        for (auto& x : n.addrs) if (x.alias == tg->net_host_network) { ad = &x; break; }
                        if (!ad) return "no addresses available for \"" + tg->net_host_network + "\" network";
                        if (rp.first < 0 || rp.first >= 65536) return "invalid port " + std::to_string(rp.first) + " (out of range)";
                        if (port_used(prop, ad->ip, rp.first))
                            return "reserved port collision " + rp.second + "=" + std::to_string(rp.first);
                        offer.push_back({ad->ip, rp.first});
                        static_dyn += (rp.first >= 20000 && rp.first <= 32000) ? 1 : 0;
                    }
                    if (tg->net_dyn > 0) {   // reservedIdx: the dynamic picks skip the static ones
                        bool has_addr = false;
                        for (auto& x : n.aliases) if (x == tg->net_host_network) { has_addr = true; break; }
                        if (!has_addr) return "no addresses available";
                        if (kDynPortCapacity - used_dyn - static_dyn < 1) return "dynamic port selection failed";
                    }
                    return "";
                };
                std::string perr = assign_ports(proposed);
                if (!perr.empty()) {
                    if (!evict) {
                        ctx->metrics.ExhaustedNode(&n, "network: " + perr);
                        continue;
                    }
                    // PreemptForNetwork on the group's ask (rank.go:273-300); nil skips
                    // the node without an ExhaustedNode, and so does a failed retry
                    pre.SetCandidates(proposed);
                    auto np = pre.ForNetwork(0, avail_bw, used_bw, rport_values);
                    if (np.empty()) continue;
                    to_preempt.insert(to_preempt.end(), np.begin(), np.end());
                    proposed = remove_allocs(proposed, np);
                    index_usage(n, proposed, &used_dyn, &used_bw);   // a new NetworkIndex
                    if (!assign_ports(proposed).empty()) continue;
                }
                used_dyn += static_dyn + tg->net_dyn;   // AddReservedPorts(offer)
                option->ports.insert(option->ports.end(), offer.begin(), offer.end());
                idx_offers.insert(idx_offers.end(), offer.begin(), offer.end());
            }
            bool skip = false;
            option->offers.clear();
            option->cores.clear();
            int64_t spc = -1;
            for (auto& t : tg->tasks) {
                if (t.has_network) {
                    // AssignNetwork over the node's AvailNetworks (device != "", yieldIP
                    // over the CIDR): bandwidth, ReservedPorts on the address, dynamic
                    std::vector<int> rport_values;
                    for (auto& rp : t.rports) rport_values.push_back(rp.first);
                    const std::string* yield_ip = nullptr;
                    const std::string* yield_dev = nullptr;
                    auto assign_network = [&](const std::vector<const OAlloc*>& prop, std::string* err) {
                        *err = "no networks available";
                        for (auto& nw : n.nets) {   // yieldIP: the AvailNetworks in node order
                            if (nw.device.empty()) continue;
                            auto ub = used_bw.find(nw.device);
                            const int32_t used = ub == used_bw.end() ? 0 : ub->second;
                            if (used + t.net_mbits > avail_bw.at(nw.device)) { *err = "bandwidth exceeded"; continue; }
                            if (!t.rports.empty()) {
                                if (nw.cidr_ip.empty()) throw Unsupported("task static ports on a network that is not one address");
                                bool bad = false;
                                for (auto& rp : t.rports) {
                                    if (rp.first < 0 || rp.first >= 65536) {
                                        *err = "invalid port " + std::to_string(rp.first) + " (out of range)";
                                        bad = true;
                                        break;
                                    }
                                    if (port_used(prop, nw.cidr_ip, rp.first)) {
                                        *err = "reserved port collision " + rp.second + "=" + std::to_string(rp.first);
                                        bad = true;
                                        break;
                                    }
                                }
                                if (bad) continue;
                            }
                            if (kDynPortCapacity - used_dyn < t.net_dyn) { *err = "dynamic port selection failed"; continue; }
                            yield_ip = &nw.cidr_ip;
                            yield_dev = &nw.device;
                            return true;
                        }
                        return false;
                    };
                    std::string err;
                    bool ok = assign_network(proposed, &err);
                    if (!ok && evict) {
                        // PreemptForNetwork on the task's ask (rank.go:343-379); the
                        // rebuilt index holds the remaining proposed allocs only
                        pre.SetCandidates(proposed);
                        auto np = pre.ForNetwork(t.net_mbits, avail_bw, used_bw, rport_values);
                        if (np.empty()) { skip = true; break; }
                        to_preempt.insert(to_preempt.end(), np.begin(), np.end());
                        proposed = remove_allocs(proposed, np);
                        index_usage(n, proposed, &used_dyn, &used_bw);
                        idx_offers.clear();   // the rebuilt index holds no earlier offers
                        std::string err2;
                        if (!assign_network(proposed, &err2)) { skip = true; break; }
                    }
                    if (!ok && !evict) { ctx->metrics.ExhaustedNode(&n, "network: " + err); skip = true; break; }
                    used_bw[*yield_dev] += t.net_mbits;   // AddReserved(offer)
                    used_dyn += t.net_dyn;
                    option->net_dev = *yield_dev;
                    for (auto& rp : t.rports) {
                        option->ports.push_back({*yield_ip, rp.first});
                        idx_offers.push_back({*yield_ip, rp.first});
                    }
                }
                // devices (rank.go:366-414)
                for (auto& req : t.devices) {
                    int g = -1; double matched = 0; std::string err;
                    if (!dev.Assign(ctx->caches, req, &g, &matched, &err)) {
                        if (!evict) { ctx->metrics.ExhaustedNode(&n, "devices: " + err); skip = true; break; }
                        pre.SetCandidates(proposed);
                        auto dp = pre.ForDevice(ctx->caches, n, req, dev);
                        if (dp.empty()) { skip = true; break; }
                        to_preempt.insert(to_preempt.end(), dp.begin(), dp.end());
                        proposed = remove_allocs(proposed, to_preempt);
                        // a fresh allocator (shadowing the outer one, rank.go:400-402)
                        DevAlloc inner(&n);
                        inner.AddAllocs(proposed);
                        if (!inner.Assign(ctx->caches, req, &g, &matched, &err)) { skip = true; break; }
                    }
                    dev.AddReserved(g, (int64_t)req.count);
                    option->offers.push_back({g, (int)req.count});
                    if (!req.affinities.empty()) {
                        for (auto& a : req.affinities) total_dev_w += std::fabs((double)a.weight);
                        sum_dev_match += matched;
                    }
                }
                if (skip) break;
                if (t.cores > 0) {   // reserved cores (rank.go:437-466)
                    std::set<uint16_t> allocated(option->cores.begin(), option->cores.end());
                    for (const OAlloc* a : proposed) allocated.insert(a->cores.begin(), a->cores.end());
                    std::vector<uint16_t> avail;   // cpuset ToSlice: ascending
                    for (uint16_t c : std::set<uint16_t>(n.rcores.begin(), n.rcores.end()))
                        if (!allocated.count(c)) avail.push_back(c);
                    if ((int64_t)avail.size() < (int64_t)t.cores) {   // no preemption for cores ("TODO")
                        ctx->metrics.ExhaustedNode(&n, "cores");
                        skip = true;
                        break;
                    }
                    option->cores.insert(option->cores.end(), avail.begin(), avail.begin() + t.cores);
                    if (n.total_cores == 0) throw Unsupported("TotalCpuCores = 0 (SharesPerCore divides by it)");
                    spc = n.cpu / (int64_t)n.total_cores;   // SharesPerCore (structs.go:3047-3049)
                }
            }
            if (skip) continue;
            Ask ask = tg_ask(*tg, oversub, spc);
            option->cpu = ask.cpu;
            // AllocsFit(node, proposed + ask): used over non-terminal allocs
            int64_t ucpu = ask.cpu, umem = ask.mem, udisk = ask.disk;
            for (const OAlloc* a : proposed) { if (a->terminal) continue; ucpu += a->cpu; umem += a->mem; udisk += a->disk; }
            int64_t acpu = n.cpu - n.rcpu, amem = n.mem - n.rmem, adisk = n.disk - n.rdisk;
            const char* dim = nullptr;
            // reserved cores: overlap between allocs, then Superset's cores
            // check against ReservableCpuCores - ReservedCpuCores (funcs.go:148-180,
            // structs.go:3891-3906)
            bool core_overlap = false, core_outside = false;
            {
                std::set<uint16_t> used;
                auto add = [&](const std::vector<uint16_t>& cs) {
                    for (uint16_t c : std::set<uint16_t>(cs.begin(), cs.end()))
                        if (!used.insert(c).second) core_overlap = true;
                };
                for (const OAlloc* a : proposed) if (!a->terminal) add(a->cores);
                add(option->cores);
                std::set<uint16_t> av(n.rcores.begin(), n.rcores.end());
                for (uint16_t c : n.nrsv_cores) av.erase(c);
                if (!av.empty())
                    for (uint16_t c : used) core_outside = core_outside || !av.count(c);
            }
            if (core_overlap) dim = "cores";
            else if (acpu < ucpu) dim = "cpu";
            else if (core_outside) dim = "cores";
            else if (amem < umem) dim = "memory";
            else if (adisk < udisk) dim = "disk";
            if (dim) {
                if (!evict) { ctx->metrics.ExhaustedNode(&n, dim); continue; }
                pre.SetCandidates(proposed);
                auto tp = pre.ForTaskGroup(CRes{ask.cpu, ask.mem, ask.disk});
                to_preempt.insert(to_preempt.end(), tp.begin(), tp.end());
                if (tp.empty()) { ctx->metrics.ExhaustedNode(&n, dim); continue; }
            }
            option->preempted = to_preempt;
            // the score uses the utilisation computed before any preemption (rank.go:505-516)
            double fitness = score_fit(spread_algo, n, ucpu, umem);
            option->scores.push_back(fitness / 18.0);
            ctx->metrics.ScoreNode(&n, "binpack", fitness / 18.0);
            if (total_dev_w != 0) {
                option->scores.push_back(sum_dev_match / total_dev_w);
                ctx->metrics.ScoreNode(&n, "devices", sum_dev_match / total_dev_w);
            }
            return option;
        }
    }
    void Reset() override { source->Reset(); }
};

// JobAntiAffinityIterator (rank.go:533-601)
struct JobAntiAffinityIterator : RankIterator {
    EvalContext* ctx; RankIterator* source;
    std::string job_id, tg; int desired = 0;
    RankedNode* Next() override {
        RankedNode* o = source->Next();
        if (!o) return nullptr;
        int coll = 0;
        for (const OAlloc* a : ctx->ProposedAllocs(o->node->row))
            if (a->job_id == job_id && a->tg == tg) coll++;
        if (coll > 0) {
            o->scores.push_back(-1 * (double)(coll + 1) / (double)desired);
            ctx->metrics.ScoreNode(o->node, "job-anti-affinity", o->scores.back());
        } else {
            ctx->metrics.ScoreNode(o->node, "job-anti-affinity", 0);
        }
        return o;
    }
    void Reset() override { source->Reset(); }
};

// NodeReschedulingPenaltyIterator (rank.go:603-646)
struct NodeReschedulingPenaltyIterator : RankIterator {
    EvalContext* ctx = nullptr; RankIterator* source; std::set<int> penalty;
    RankedNode* Next() override {
        RankedNode* o = source->Next();
        if (!o) return nullptr;
        if (penalty.count(o->node->row)) {
            o->scores.push_back(-1);
            ctx->metrics.ScoreNode(o->node, "node-reschedule-penalty", -1);
        } else {
            ctx->metrics.ScoreNode(o->node, "node-reschedule-penalty", 0);
        }
        return o;
    }
    void Reset() override { penalty.clear(); source->Reset(); }
};

// NodeAffinityIterator (rank.go:648-735)
struct NodeAffinityIterator : RankIterator {
    EvalContext* ctx; RankIterator* source;
    std::vector<OAffinity> job_affs, affs;
    void SetJob(const OJob* j) { job_affs = j->affinities; }
    void SetTaskGroup(const OTaskGroup* t) {
        affs.insert(affs.end(), job_affs.begin(), job_affs.end());
        affs.insert(affs.end(), t->affinities.begin(), t->affinities.end());
        for (auto& ta : t->task_affinities) affs.insert(affs.end(), ta.begin(), ta.end());
    }
    bool has() const { return !affs.empty(); }
    RankedNode* Next() override {
        RankedNode* o = source->Next();
        if (!o) return nullptr;
        if (!has()) { ctx->metrics.ScoreNode(o->node, "node-affinity", 0); return o; }
        double sum_w = 0.0;
        for (auto& a : affs) sum_w += std::fabs((double)a.weight);
        double total = 0.0;
        for (auto& a : affs) {
            bool lf, rf;
            Val l = resolve_target(a.l, *o->node, &lf), r = resolve_target(a.r, *o->node, &rf);
            if (orasem::check_constraint(ctx->caches, a.op, l, r, lf, rf)) total += (double)a.weight;
        }
        double norm = total / sum_w;
        if (total != 0.0) {
            o->scores.push_back(norm);
            ctx->metrics.ScoreNode(o->node, "node-affinity", norm);
        }
        return o;
    }
    void Reset() override { source->Reset(); affs.clear(); }
};

// SpreadIterator (spread.go:13-257)
struct SpreadInfo { int8_t weight; std::map<std::string, double> desired; };
struct SpreadIterator : RankIterator {
    EvalContext* ctx; RankIterator* source;
    const OJob* job = nullptr; const OTaskGroup* tg = nullptr;
    std::vector<OSpread> job_spreads;
    std::map<std::string, std::map<std::string, SpreadInfo>> tg_spread_info;
    int32_t sum_spread_weights = 0;
    bool has_spread = false;
    std::map<std::string, std::vector<std::unique_ptr<PropertySet>>> group_sets;

    void SetJob(const OJob* j) { job = j; if (!j->spreads.empty()) job_spreads = j->spreads; }
    void compute_spread_info(const OTaskGroup* t) {
        std::map<std::string, SpreadInfo> infos;
        double total = (double)t->count;
        std::vector<OSpread> combined = t->spreads;
        combined.insert(combined.end(), job_spreads.begin(), job_spreads.end());
        for (auto& sp : combined) {
            SpreadInfo si; si.weight = sp.weight;
            double sum = 0.0;
            for (auto& st : sp.targets) {
                double d = ((double)st.percent / (double)100) * total;
                si.desired[st.value] = d;
                sum += d;
            }
            if (sum > 0 && sum < total) si.desired["*"] = total - sum;
            infos[sp.attribute] = si;
            sum_spread_weights += (int32_t)sp.weight;
        }
        tg_spread_info[t->name] = infos;
    }
    void SetTaskGroup(const OTaskGroup* t) {
        tg = t;
        if (!group_sets.count(t->name)) {
            auto& v = group_sets[t->name];
            for (auto& sp : job_spreads) {
                auto p = std::make_unique<PropertySet>();
                p->ctx = ctx; p->job_id = job->id; p->ns = job->ns;
                p->set_target(sp.attribute, 0, t->name);
                v.push_back(std::move(p));
            }
            for (auto& sp : t->spreads) {
                auto p = std::make_unique<PropertySet>();
                p->ctx = ctx; p->job_id = job->id; p->ns = job->ns;
                p->set_target(sp.attribute, 0, t->name);
                v.push_back(std::move(p));
            }
        }
        has_spread = !group_sets[t->name].empty();
        if (!tg_spread_info.count(t->name)) compute_spread_info(t);
    }
    static double even_boost(const PropertySet& ps, const ONode& n) {
        auto use = ps.CombinedUse();
        if (use.empty()) return 0.0;
        std::string v;
        if (!get_property(&n, ps.target, &v)) return -1.0;
        uint64_t cur = use.count(v) ? use[v] : 0;
        uint64_t mn = 0, mx = 0;
        for (auto& kv : use) {
            if (mn == 0 || kv.second < mn) mn = kv.second;
            if (mx == 0 || kv.second > mx) mx = kv.second;
        }
        double delta_boost;
        if (mn == 0) delta_boost = -1.0;
        else { int64_t d = (int64_t)(mn - cur); delta_boost = (double)d / (double)mn; }
        if (cur != mn) return delta_boost;
        if (mn == mx) return -1.0;
        if (mn == 0) return 1.0;
        int64_t d = (int64_t)(mx - mn);
        return (double)d / (double)mn;
    }
    RankedNode* Next() override {
        for (;;) {
            RankedNode* o = source->Next();
            if (!o || !has_spread) return o;
            double total = 0.0;
            auto& infos = tg_spread_info[tg->name];
            for (auto& ps : group_sets[tg->name]) {
                std::string v, err; uint64_t used = 0;
                bool ok = ps->UsedCount(*o->node, &v, &used, &err);
                used += 1;
                if (!ok) { total -= 1.0; continue; }
                auto it = infos.find(ps->target);
                SpreadInfo empty{0, {}};
                const SpreadInfo& sd = it == infos.end() ? empty : it->second;
                if (sd.desired.empty()) { total += even_boost(*ps, *o->node); continue; }
                auto dit = sd.desired.find(v);
                double desired;
                if (dit == sd.desired.end()) {
                    auto star = sd.desired.find("*");
                    if (star == sd.desired.end()) { total -= 1.0; continue; }
                    desired = star->second;
                } else desired = dit->second;
                double w = (double)sd.weight / (double)sum_spread_weights;
                double boost = ((desired - (double)used) / desired) * w;
                total += boost;
            }
            if (total != 0.0) {
                o->scores.push_back(total);
                ctx->metrics.ScoreNode(o->node, "allocation-spread", total);
            }
            return o;
        }
    }
    void Reset() override {
        source->Reset();
        for (auto& kv : group_sets) for (auto& p : kv.second) p->PopulateProposed();
    }
};

// PreemptionScoringIterator (rank.go:773-806)
struct PreemptionScoringIterator : RankIterator {
    EvalContext* ctx = nullptr;
    RankIterator* source;
    RankedNode* Next() override {
        RankedNode* o = source->Next();
        if (!o || o->preempted.empty()) return o;
        o->scores.push_back(preemption_score(o->preempted));
        if (ctx) ctx->metrics.ScoreNode(o->node, "preemption", o->scores.back());
        return o;
    }
    void Reset() override { source->Reset(); }
};

// ScoreNormalizationIterator (rank.go:737-771)
struct ScoreNormalizationIterator : RankIterator {
    EvalContext* ctx = nullptr;
    RankIterator* source;
    RankedNode* Next() override {
        RankedNode* o = source->Next();
        if (!o || o->scores.empty()) return o;
        double sum = 0.0;
        for (double s : o->scores) sum += s;
        o->final_score = sum / (double)o->scores.size();
        if (ctx) ctx->metrics.ScoreNode(o->node, "normalized-score", o->final_score);
        if (g_trace_status) { g_trace_status[o->node->row] = 0; g_trace_score[o->node->row] = o->final_score; }
        return o;
    }
    void Reset() override { source->Reset(); }
};

// LimitIterator (select.go:5-74)
struct LimitIterator : RankIterator {
    RankIterator* source; int limit; int max_skip; double threshold;
    int seen = 0; std::vector<RankedNode*> skipped; size_t skipped_index = 0;
    RankedNode* next_option() {
        RankedNode* s = source->Next();
        if (!s && skipped_index < skipped.size()) return skipped[skipped_index++];
        return s;
    }
    RankedNode* Next() override {
        if (seen == limit) return nullptr;
        RankedNode* o = next_option();
        if (!o) return nullptr;
        if ((int)skipped.size() < max_skip) {
            while (o && o->final_score <= threshold && (int)skipped.size() < max_skip) {
                skipped.push_back(o);
                o = source->Next();
            }
        }
        seen++;
        if (!o) return next_option();
        return o;
    }
    void Reset() override { source->Reset(); seen = 0; skipped.clear(); skipped_index = 0; }
};

// MaxScoreIterator (select.go:76-116)
struct MaxScoreIterator : RankIterator {
    RankIterator* source; RankedNode* max = nullptr;
    RankedNode* Next() override {
        if (max) return nullptr;
        for (;;) {
            RankedNode* o = source->Next();
            if (!o) return max;
            if (!max || o->final_score > max->final_score) max = o;
        }
    }
    void Reset() override { source->Reset(); max = nullptr; }
};

// StaticRankIterator (rank.go:109-147), for the LimitIterator KAT helper
struct StaticRankIterator : RankIterator {
    std::vector<RankedNode*> nodes; int offset = 0, seen = 0, pulled = 0;
    RankedNode* Next() override {
        int n = (int)nodes.size();
        if (offset == n || seen == n) {
            if (seen != n) offset = 0;
            else return nullptr;
        }
        int o = offset; offset++; seen++; pulled++;
        return nodes[o];
    }
    void Reset() override { seen = 0; }
};

}  // namespace

// ---------------------------------------------------------------------------
// The stack handle
struct oracle_stack {
    pe_config cfg;
    std::string err;
    // PreemptedAllocs past PE_MAX_PREEMPT of the last record-producing call:
    // (record index, full list), as the engine's pe_preempted_of
    std::vector<std::pair<uint32_t, std::vector<uint32_t>>> pre_overflow;
    uint32_t cur_rec = 0;
    State state;
    EvalContext ctx;
    OJob job; bool have_job = false;
    std::vector<const ONode*> base_nodes;

    // chain
    StaticIterator source;
    ConstraintChecker job_constraint, tg_constraint;
    DriverChecker tg_drivers;
    HostVolumeChecker tg_volumes;
    DeviceChecker tg_devices;
    NetworkChecker tg_network;
    FeasibilityWrapper wrapped;
    DistinctHostsIterator distinct_hosts;
    DistinctPropertyIterator distinct_property;
    FeasibleRankIterator rank_source;
    BinPackIterator bin_pack;
    JobAntiAffinityIterator job_anti_aff;
    NodeReschedulingPenaltyIterator penalty;
    NodeAffinityIterator node_affinity;
    SpreadIterator spread;
    PreemptionScoringIterator preempt_score;
    ScoreNormalizationIterator score_norm;
    LimitIterator limit;
    MaxScoreIterator max_score;
    bool have_job_version = false; uint64_t job_version = 0;
    int offer_row = -1;                                // device offers of the last Select's pick
    std::vector<std::pair<int, int>> offers;
    std::vector<uint16_t> offer_cores;                 // and its reserved cores / CpuShares / static ports
    int64_t offer_cpu = 0;
    std::vector<std::pair<std::string, int>> offer_ports;
    std::string offer_net_dev;

    explicit oracle_stack(const pe_config& c) : cfg(c) {
        ctx.state = &state;
        source.ctx = &ctx;
        job_constraint.ctx = &ctx; tg_constraint.ctx = &ctx;
        tg_drivers.ctx = &ctx; tg_volumes.ctx = &ctx; tg_network.ctx = &ctx; tg_devices.ctx = &ctx;
        wrapped.ctx = &ctx; wrapped.source = &source;
        wrapped.job_checkers = {&job_constraint};
        wrapped.tg_checkers = {&tg_drivers, &tg_constraint, &tg_volumes, &tg_devices, &tg_network};
        bool generic = c.stack_kind == PE_STACK_GENERIC;
        distinct_hosts.ctx = &ctx; distinct_hosts.source = &wrapped;
        distinct_property.ctx = &ctx;
        distinct_property.source = generic ? (FeasibleIterator*)&distinct_hosts : (FeasibleIterator*)&wrapped;
        rank_source.source = &distinct_property;   // quota iterator is a no-op in OSS
        bin_pack.ctx = &ctx; bin_pack.source = &rank_source;
        bin_pack.evict = !generic && c.preempt;
        bin_pack.spread_algo = c.algorithm == PE_ALGO_SPREAD;
        bin_pack.oversub = c.memory_oversubscription != 0;
        job_anti_aff.ctx = &ctx; job_anti_aff.source = &bin_pack;
        penalty.ctx = &ctx; penalty.source = &job_anti_aff;
        node_affinity.ctx = &ctx; node_affinity.source = &penalty;
        spread.ctx = &ctx; spread.source = &node_affinity;
        preempt_score.ctx = &ctx; preempt_score.source = &spread;
        score_norm.ctx = &ctx; score_norm.source = generic ? (RankIterator*)&preempt_score : (RankIterator*)&bin_pack;
        limit.source = &score_norm; limit.limit = 2; limit.max_skip = 3; limit.threshold = 0.0;
        max_score.source = &limit;
    }
    const OTaskGroup& tg(uint32_t i) const { return job.tgs.at(i); }
};

static std::string S(const State& st, uint32_t id) {
    if (id == PE_NONE || id >= st.strs.size()) return std::string();
    return st.strs[id];
}

extern "C" {

oracle_stack* oracle_create(const pe_config* cfg) {
    if (!cfg) return nullptr;
    return new oracle_stack(*cfg);
}
void oracle_destroy(oracle_stack* s) { delete s; }
const char* oracle_last_error(const oracle_stack* s) { return s ? s->err.c_str() : "null handle"; }

int oracle_set_state(oracle_stack* s, const pe_strtab* strs, const pe_node_table* nt,
                     const pe_alloc_table* at) {
    State& st = s->state;
    st = State();
    for (uint32_t i = 0; i < strs->count; i++)
        st.strs.emplace_back(strs->bytes + strs->offsets[i], strs->offsets[i + 1] - strs->offsets[i]);
    st.nodes.resize(nt->n);
    for (uint32_t i = 0; i < nt->n; i++) {
        ONode& n = st.nodes[i];
        n.row = (int)i;
        n.id = S(st, nt->id[i]); n.name = S(st, nt->name[i]); n.dc = S(st, nt->datacenter[i]);
        n.node_class = S(st, nt->node_class[i]); n.computed_class = S(st, nt->computed_class[i]);
        n.cpu = nt->cpu_shares[i]; n.mem = nt->memory_mb[i]; n.disk = nt->disk_mb[i];
        n.rcpu = nt->reserved_cpu[i]; n.rmem = nt->reserved_memory_mb[i]; n.rdisk = nt->reserved_disk_mb[i];
        for (uint32_t k = nt->attr_off[i]; k < nt->attr_off[i + 1]; k++) n.attrs[S(st, nt->attr_key[k])] = S(st, nt->attr_val[k]);
        for (uint32_t k = nt->meta_off[i]; k < nt->meta_off[i + 1]; k++) n.meta[S(st, nt->meta_key[k])] = S(st, nt->meta_val[k]);
        for (uint32_t k = nt->drv_off[i]; k < nt->drv_off[i + 1]; k++) {
            uint8_t f = nt->drv_flags[k];
            n.drivers[S(st, nt->drv_name[k])] = DriverInfo{(f & 1) != 0, (f & 2) != 0, (f & 4) != 0};
        }
        for (uint32_t k = nt->net_off[i]; k < nt->net_off[i + 1]; k++) {
            auto ip_of = [&](const uint32_t* col) {
                return (col && col[k] != PE_NONE) ? S(st, col[k]) : std::string();
            };
            n.nets.push_back(NetRes{S(st, nt->net_mode[k]), S(st, nt->net_device[k]), nt->net_mbits[k],
                                    ip_of(nt->net_ip), ip_of(nt->net_cidr_ip)});
        }
        for (uint32_t k = nt->alias_off[i]; k < nt->alias_off[i + 1]; k++) n.aliases.push_back(S(st, nt->alias_name[k]));
        n.reserved_dyn = nt->reserved_dyn_ports ? nt->reserved_dyn_ports[i] : 0;
        if (nt->hv_off)
            for (uint32_t k = nt->hv_off[i]; k < nt->hv_off[i + 1]; k++) n.host_volumes[S(st, nt->hv_name[k])] = nt->hv_read_only[k] != 0;
        n.n_devices = nt->dev_off ? (int)(nt->dev_off[i + 1] - nt->dev_off[i]) : 0;
        for (int k = 0; k < n.n_devices; k++) {
            const uint32_t g = nt->dev_off[i] + (uint32_t)k;
            ODev d;
            d.vendor = S(st, nt->dev_vendor[g]); d.type = S(st, nt->dev_type[g]); d.name = S(st, nt->dev_name[g]);
            d.healthy = (int)nt->dev_healthy[g];
            for (uint32_t q = nt->dev_attr_off[g]; nt->dev_attr_off && q < nt->dev_attr_off[g + 1]; q++) {
                const pe_attr& pa = nt->dev_attr_val[q];
                orasem::Attr a;
                a.unit = S(st, pa.unit);
                switch (pa.kind) {
                    case PE_ATTR_INT: a.kind = orasem::Attr::Int; a.i = pa.i; break;
                    case PE_ATTR_FLOAT: a.kind = orasem::Attr::Float; a.f = pa.f; break;
                    case PE_ATTR_BOOL: a.kind = orasem::Attr::Bool; a.b = pa.i != 0; a.unit.clear(); break;
                    default: a.kind = orasem::Attr::Str; a.s = S(st, pa.s); a.unit.clear(); break;
                }
                d.attrs[S(st, nt->dev_attr_key[q])] = a;
            }
            n.devs.push_back(d);
        }
        if (nt->core_off)
            n.rcores.assign(nt->core_id + nt->core_off[i], nt->core_id + nt->core_off[i + 1]);
        if (nt->rsv_core_off)
            n.nrsv_cores.assign(nt->rsv_core_id + nt->rsv_core_off[i], nt->rsv_core_id + nt->rsv_core_off[i + 1]);
        n.total_cores = nt->total_cores ? nt->total_cores[i] : 0;
        for (uint32_t k = nt->addr_off ? nt->addr_off[i] : 0; nt->addr_off && k < nt->addr_off[i + 1]; k++) {
            ONode::Addr a;
            a.alias = S(st, nt->addr_alias[k]);
            a.ip = S(st, nt->addr_ip[k]);
            if (nt->addr_rsv_ports && nt->addr_rsv_ports[k] != PE_NONE) a.reserved = parse_port_ranges(S(st, nt->addr_rsv_ports[k]));
            n.addrs.push_back(a);
        }
        if (nt->rsv_host_ports && nt->rsv_host_ports[i] != PE_NONE)
            n.reserved_host_ports = parse_port_ranges(S(st, nt->rsv_host_ports[i]));
    }
    st.allocs.resize(at ? at->count : 0);
    st.allocs_by_node.assign(nt->n, {});
    for (uint32_t i = 0; at && i < at->count; i++) {
        OAlloc& a = st.allocs[i];
        a.id = i + 1;
        a.node_row = (int)at->node_row[i];
        if (a.node_row < 0 || a.node_row >= (int)nt->n) { s->err = "alloc node_row out of range"; return PE_EINVAL; }
        a.ns = S(st, at->ns[i]); a.job_id = S(st, at->job_id[i]); a.tg = S(st, at->task_group[i]);
        a.terminal = at->terminal[i] != 0; a.priority = at->priority[i];
        a.cpu = at->cpu_shares[i]; a.mem = at->memory_mb[i]; a.disk = at->disk_mb[i];
        a.mbits = at->net_mbits[i]; a.dyn_ports = at->dyn_ports[i];
        a.state_index = (int)i;
        const bool held_ports = at->port_off && at->port_off[i + 1] > at->port_off[i];
        a.has_net = at->has_network ? at->has_network[i] != 0 : (a.mbits > 0 || a.dyn_ports > 0 || held_ports);
        if (at->net_device && at->net_device[i] != PE_NONE) {
            a.dev = S(st, at->net_device[i]);
        } else {   // the node's first host network device (pe_alloc_table.net_device)
            const ONode& nd = st.nodes[(size_t)a.node_row];
            for (auto& nw : nd.nets) if (!nw.device.empty()) { a.dev = nw.device; break; }
        }
        a.max_parallel = at->max_parallel ? at->max_parallel[i] : 0;
        if (at->dev_off)
            for (uint32_t k = at->dev_off[i]; k < at->dev_off[i + 1]; k++)
                a.devs.push_back({(int)at->dev_group[k], (int)at->dev_count[k]});
        if (at->core_off) a.cores.assign(at->core_id + at->core_off[i], at->core_id + at->core_off[i + 1]);
        if (at->port_off)
            for (uint32_t k = at->port_off[i]; k < at->port_off[i + 1]; k++) a.ports.push_back({S(st, at->port_ip[k]), at->port_value[k]});
        st.allocs_by_node[a.node_row].push_back((int)i);
    }
    s->ctx.plan = Plan();
    return PE_OK;
}

}  // extern "C"

// Fresh EvalContext on the same snapshot: the chain and the eligibility memo
// are rebuilt, exactly as a new eval would construct them.
extern "C" int oracle_reset_plan(oracle_stack* s) {
    State saved = std::move(s->state);
    pe_config cfg = s->cfg;
    s->~oracle_stack();
    new (s) oracle_stack(cfg);
    s->state = std::move(saved);
    s->ctx.state = &s->state;
    return PE_OK;
}

extern "C" {

static std::vector<OConstraint> conv_constraints(const State& st, const pe_constraint* base, uint32_t off, uint32_t cnt) {
    std::vector<OConstraint> out;
    for (uint32_t i = 0; i < cnt; i++) out.push_back(OConstraint{S(st, base[off + i].ltarget), S(st, base[off + i].rtarget), S(st, base[off + i].operand)});
    return out;
}
static std::vector<OAffinity> conv_affinities(const State& st, const pe_affinity* base, uint32_t off, uint32_t cnt) {
    std::vector<OAffinity> out;
    for (uint32_t i = 0; i < cnt; i++) out.push_back(OAffinity{S(st, base[off + i].ltarget), S(st, base[off + i].rtarget), S(st, base[off + i].operand), base[off + i].weight});
    return out;
}
static std::vector<OSpread> conv_spreads(const State& st, const pe_job* j, uint32_t off, uint32_t cnt) {
    std::vector<OSpread> out;
    for (uint32_t i = 0; i < cnt; i++) {
        const pe_spread& sp = j->spreads[off + i];
        OSpread o; o.attribute = S(st, sp.attribute); o.weight = (int8_t)sp.weight;
        for (uint32_t k = 0; k < sp.target_count; k++) {
            const pe_spread_target& t = j->spread_targets[sp.target_off + k];
            o.targets.push_back(OSpreadTarget{S(st, t.value), t.percent});
        }
        out.push_back(o);
    }
    return out;
}

int oracle_set_job(oracle_stack* s, const pe_strtab* strs, const pe_job* j) {
    State& st = s->state;
    for (uint32_t i = (uint32_t)st.strs.size(); strs && i < strs->count; i++)
        st.strs.emplace_back(strs->bytes + strs->offsets[i], strs->offsets[i + 1] - strs->offsets[i]);
    OJob job;
    job.id = S(st, j->id); job.ns = S(st, j->ns); job.type = j->type; job.priority = j->priority; job.version = j->version;
    job.constraints = conv_constraints(st, j->constraints, j->constraint_off, j->constraint_count);
    job.affinities = conv_affinities(st, j->affinities, j->affinity_off, j->affinity_count);
    job.spreads = conv_spreads(st, j, j->spread_off, j->spread_count);
    for (uint32_t g = 0; g < j->tg_count; g++) {
        const pe_task_group& t = j->task_groups[g];
        OTaskGroup tg;
        tg.name = S(st, t.name); tg.count = t.count; tg.disk = t.ephemeral_disk_mb;
        tg.constraints = conv_constraints(st, j->constraints, t.constraint_off, t.constraint_count);
        tg.affinities = conv_affinities(st, j->affinities, t.affinity_off, t.affinity_count);
        tg.spreads = conv_spreads(st, j, t.spread_off, t.spread_count);
        tg.has_network = t.has_network != 0; tg.net_mode = S(st, t.net_mode);
        tg.net_host_network = S(st, t.net_host_network);
        if (tg.net_host_network.empty()) tg.net_host_network = "default";
        tg.net_dyn = t.net_dyn_ports; tg.net_reserved = t.net_reserved_ports;
        for (uint32_t k = 0; k < t.rport_count && j->rport_value; k++)
            tg.rports.push_back({j->rport_value[t.rport_off + k], S(st, j->rport_label[t.rport_off + k])});
        for (uint32_t k = 0; k < t.volume_count; k++)
            tg.volumes.push_back({S(st, j->volume_source[t.volume_off + k]), j->volume_read_only[t.volume_off + k] != 0});
        tg.csi = t.has_csi_volumes != 0;
        for (uint32_t k = 0; k < t.task_count; k++) {
            const pe_task& pt = j->tasks[t.task_off + k];
            OTask ot;
            ot.name = S(st, pt.name); ot.driver = S(st, pt.driver);
            ot.cpu = pt.cpu; ot.mem = pt.memory_mb; ot.mem_max = pt.memory_max_mb; ot.cores = pt.cores;
            ot.lifecycle = pt.lifecycle;
            ot.has_network = pt.has_network != 0; ot.net_mbits = pt.net_mbits; ot.net_dyn = pt.net_dyn_ports; ot.net_reserved = pt.net_reserved_ports;
            for (int32_t q = 0; ot.has_network && q < pt.net_reserved_ports; q++) {
                if (!j->rport_value) throw Unsupported("task static ports without their values");
                ot.rports.push_back({j->rport_value[pt.rport_off + (uint32_t)q],
                                     j->rport_label ? S(st, j->rport_label[pt.rport_off + (uint32_t)q]) : std::string()});
            }
            ot.n_devices = (int)pt.device_count;
            for (uint32_t q = 0; q < pt.device_count; q++) {
                const pe_device_request& r = j->devices[pt.device_off + q];
                ODevReq dr;
                dr.name = S(st, r.name); dr.count = r.count;
                dr.constraints = conv_constraints(st, j->device_constraints, r.constraint_off, r.constraint_count);
                dr.affinities = conv_affinities(st, j->device_affinities, r.affinity_off, r.affinity_count);
                ot.devices.push_back(dr);
            }
            tg.tasks.push_back(ot);
            tg.task_constraints.push_back(conv_constraints(st, j->constraints, pt.constraint_off, pt.constraint_count));
            tg.task_affinities.push_back(conv_affinities(st, j->affinities, pt.affinity_off, pt.affinity_count));
        }
        job.tgs.push_back(tg);
    }
    // GenericStack.SetJob skips when the job version is unchanged (stack.go:94-96)
    if (s->cfg.stack_kind == PE_STACK_GENERIC && s->have_job_version && s->job_version == job.version) return PE_OK;
    s->have_job_version = true; s->job_version = job.version;
    s->job = job; s->have_job = true;
    const OJob* jp = &s->job;
    s->job_constraint.cs = jp->constraints;
    if (s->cfg.stack_kind == PE_STACK_GENERIC) s->distinct_hosts.SetJob(jp);
    s->distinct_property.SetJob(jp);
    s->bin_pack.priority = jp->priority; s->bin_pack.job_id = jp->id; s->bin_pack.job_ns = jp->ns;
    s->job_anti_aff.job_id = jp->id;
    s->node_affinity.SetJob(jp);
    s->spread.SetJob(jp);
    s->ctx.elig.SetJob(*jp);
    return PE_OK;
}

int oracle_set_nodes(oracle_stack* s, const uint32_t* rows, uint32_t n, uint32_t* limit_out) {
    std::vector<const ONode*> ns;
    for (uint32_t i = 0; i < n; i++) {
        if (rows[i] >= s->state.nodes.size()) { s->err = "row out of range"; return PE_EINVAL; }
        ns.push_back(&s->state.nodes[rows[i]]);
    }
    s->base_nodes = ns;
    s->source.SetNodes(ns);
    int lim = 2;
    if (s->cfg.stack_kind == PE_STACK_GENERIC && !s->cfg.batch && n > 0) {
        int log_limit = (int)std::ceil(std::log2((double)n));
        if (log_limit > lim) lim = log_limit;
    }
    s->limit.limit = lim;
    if (limit_out) *limit_out = (uint32_t)lim;
    return PE_OK;
}

// taskGroupConstraints (util.go:843-858) + per-tg parameterisation (stack.go:139-163)
static void set_task_group(oracle_stack* s, const OTaskGroup& tg, bool system) {
    std::vector<OConstraint> cs = tg.constraints;
    std::set<std::string> drivers;
    for (size_t k = 0; k < tg.tasks.size(); k++) {
        drivers.insert(tg.tasks[k].driver);
        cs.insert(cs.end(), tg.task_constraints[k].begin(), tg.task_constraints[k].end());
    }
    if (tg.csi) throw Unsupported("CSI volumes");
    s->tg_drivers.drivers = drivers;
    s->tg_constraint.cs = cs;
    s->tg_devices.required.clear();
    for (auto& t : tg.tasks) for (auto& r : t.devices) s->tg_devices.required.push_back(&r);
    s->tg_volumes.volumes.clear();
    for (auto& v : tg.volumes) s->tg_volumes.volumes[v.first].push_back(v.second);
    if (tg.has_network) {
        s->tg_network.mode = tg.net_mode.empty() ? "host" : tg.net_mode;
        s->tg_network.has_ports = true;   // c.ports is a non-nil slice after SetNetwork
        s->tg_network.port_networks.assign((size_t)(tg.net_dyn + tg.net_reserved), tg.net_host_network);
    }
    s->wrapped.tg = tg.name;
    if (!system) {
        s->distinct_hosts.SetTaskGroup(&tg);
    }
    s->distinct_property.SetTaskGroup(&tg);
    s->bin_pack.tg = &tg;
}

static void fill_out(pe_ranked_node* out, RankedNode* o, oracle_stack* s) {
    std::memset(out, 0, sizeof(*out));
    out->row = o ? o->node->row : -1;
    if (o) {
        out->final_score = o->final_score;
        out->n_scores = (uint32_t)std::min<size_t>(o->scores.size(), PE_MAX_SCORES);
        for (uint32_t i = 0; i < out->n_scores; i++) out->scores[i] = o->scores[i];
    }
    out->nodes_evaluated = s->ctx.metrics.evaluated;
    out->nodes_filtered = s->ctx.metrics.filtered;
    out->nodes_exhausted = s->ctx.metrics.exhausted;
    out->new_offset = s->source.nodes.empty() ? 0 : (uint32_t)(s->source.offset % (int)s->source.nodes.size());
    if (o) {
        out->n_preempted = (uint32_t)o->preempted.size();
        std::vector<uint32_t> full;
        for (size_t i = 0; i < o->preempted.size(); i++) {
            const uint32_t a = (uint32_t)o->preempted[i]->state_index;
            if (i < PE_MAX_PREEMPT) out->preempted[i] = a;
            full.push_back(a);
        }
        if (full.size() > PE_MAX_PREEMPT) s->pre_overflow.emplace_back(s->cur_rec, std::move(full));
        if (o->offers.size() > PE_MAX_DEVICE_REQ) throw Unsupported("more than PE_MAX_DEVICE_REQ device requests");
        out->n_device_offers = (uint32_t)o->offers.size();
        for (size_t i = 0; i < o->offers.size(); i++) out->device_offer_group[i] = (uint32_t)o->offers[i].first;
        for (uint16_t c : o->cores)
            if (c < 256) out->reserved_cores[c >> 6] |= 1ull << (c & 63);
    }
}

static RankedNode* generic_select(oracle_stack* s, uint32_t tgi, const pe_select_options* opts) {
    if (opts && opts->preferred_count > 0) {
        std::vector<const ONode*> original = s->source.nodes;
        std::vector<const ONode*> pref;
        for (uint32_t i = 0; i < opts->preferred_count; i++) pref.push_back(&s->state.nodes.at(opts->preferred_rows[i]));
        s->source.SetNodes(pref);
        pe_select_options o2 = *opts; o2.preferred_count = 0; o2.preferred_rows = nullptr;
        RankedNode* r = generic_select(s, tgi, &o2);
        if (r) { s->source.SetNodes(original); return r; }
        s->source.SetNodes(original);
        return generic_select(s, tgi, &o2);
    }
    s->max_score.Reset();
    s->ctx.Reset();
    const OTaskGroup& tg = s->tg(tgi);
    set_task_group(s, tg, false);
    if (opts) s->bin_pack.evict = opts->preempt != 0;
    s->job_anti_aff.tg = tg.name; s->job_anti_aff.desired = tg.count;
    if (opts) for (uint32_t i = 0; i < opts->penalty_count; i++) s->penalty.penalty.insert((int)opts->penalty_rows[i]);
    s->node_affinity.SetTaskGroup(&tg);
    s->spread.SetTaskGroup(&tg);
    if (s->node_affinity.has() || s->spread.has_spread) s->limit.limit = INT32_MAX;
    return s->max_score.Next();
}

static RankedNode* system_select(oracle_stack* s, uint32_t tgi) {
    s->score_norm.Reset();
    s->ctx.Reset();
    const OTaskGroup& tg = s->tg(tgi);
    set_task_group(s, tg, true);
    return s->score_norm.Next();
}

static int select_rec(oracle_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out,
                      uint32_t rec);

int oracle_select(oracle_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out) {
    s->pre_overflow.clear();
    return select_rec(s, tgi, opts, out, 0);
}

// The full PreemptedAllocs of record `rec` of the last call (engine: pe_preempted_of).
int oracle_preempted_of(const oracle_stack* s, uint32_t rec, uint32_t* out, uint32_t cap) {
    for (auto& e : s->pre_overflow)
        if (e.first == rec) {
            const size_t k = std::min<size_t>(cap, e.second.size());
            for (size_t i = 0; i < k; i++) out[i] = e.second[i];
            return (int)e.second.size();
        }
    return PE_ESTATE;
}

static const uint32_t* full_preempted(const oracle_stack* s, uint32_t rec, const pe_ranked_node& r) {
    if (r.n_preempted <= PE_MAX_PREEMPT) return r.preempted;
    for (auto& e : s->pre_overflow)
        if (e.first == rec && e.second.size() == r.n_preempted) return e.second.data();
    return nullptr;
}

static int select_rec(oracle_stack* s, uint32_t tgi, const pe_select_options* opts, pe_ranked_node* out,
                      uint32_t rec) {
    s->cur_rec = rec;
    if (!s->have_job || tgi >= s->job.tgs.size()) { s->err = "select before set_job / bad tg"; return PE_ESTATE; }
    try {
        RankedNode* o = s->cfg.stack_kind == PE_STACK_GENERIC ? generic_select(s, tgi, opts) : system_select(s, tgi);
        fill_out(out, o, s);
        s->offer_row = o ? o->node->row : -1;
        if (o) {
            s->offers = o->offers; s->offer_cores = o->cores; s->offer_cpu = o->cpu; s->offer_ports = o->ports;
            s->offer_net_dev = o->net_dev;
        }
    } catch (const Unsupported& e) {
        s->err = std::string("unsupported: ") + e.what();
        return PE_EUNSUPPORTED;
    }
    return PE_OK;
}

// Plan.AppendAlloc of a fresh alloc of the task group (structs.go:10707-10714)
int oracle_commit(oracle_stack* s, uint32_t tgi, int32_t row) {
    if (!s->have_job || tgi >= s->job.tgs.size() || row < 0 || row >= (int32_t)s->state.nodes.size()) {
        s->err = "bad commit"; return PE_EINVAL;
    }
    const OTaskGroup& tg = s->tg(tgi);
    Ask ask = tg_ask(tg, s->bin_pack.oversub);
    OAlloc a;
    a.id = s->ctx.next_alloc_id++;
    a.node_row = row; a.ns = s->job.ns; a.job_id = s->job.id; a.tg = tg.name;
    a.terminal = false; a.priority = s->job.priority;
    a.cpu = ask.cpu; a.mem = ask.mem; a.disk = ask.disk;
    tg_net_contrib(tg, &a.mbits, &a.dyn_ports);
    if (row == s->offer_row) {
        a.devs = s->offers;
        a.cores = s->offer_cores;
        a.cpu = s->offer_cpu;
        a.ports = s->offer_ports;
        a.dev = s->offer_net_dev;
    } else {   // commit without a Select of this node: assign on the proposed state
        const ONode& n = s->state.nodes[(size_t)row];
        {   // AssignNetwork's device: the first AvailNetworks entry with the bandwidth
            std::map<std::string, int32_t> used, avail;
            for (auto& nw : n.nets) if (!nw.device.empty()) avail[nw.device] = nw.mbits;
            for (const OAlloc* p : s->ctx.ProposedAllocs(row)) if (!p->terminal && p->mbits) used[p->dev] += p->mbits;
            int32_t ask_mbits = 0;
            for (auto& t : tg.tasks) if (t.has_network) ask_mbits += t.net_mbits;
            for (auto& nw : n.nets)
                if (!nw.device.empty() && used[nw.device] + ask_mbits <= avail[nw.device]) { a.dev = nw.device; break; }
        }
        DevAlloc dev(&n);
        dev.AddAllocs(s->ctx.ProposedAllocs(row));
        for (auto& t : tg.tasks)
            for (auto& r : t.devices) {
                int g; double m; std::string err;
                if (!dev.Assign(s->ctx.caches, r, &g, &m, &err)) continue;
                dev.AddReserved(g, (int64_t)r.count);
                a.devs.push_back({g, (int)r.count});
            }
        // reserved cores: the lowest free ones of the node, as BinPack picks them
        int64_t need = 0;
        for (auto& t : tg.tasks) need += t.cores > 0 ? t.cores : 0;
        if (need > 0) {
            std::set<uint16_t> allocated;
            for (const OAlloc* p : s->ctx.ProposedAllocs(row)) allocated.insert(p->cores.begin(), p->cores.end());
            for (uint16_t c : std::set<uint16_t>(n.rcores.begin(), n.rcores.end()))
                if (!allocated.count(c) && (int64_t)a.cores.size() < need) a.cores.push_back(c);
            a.cpu = tg_ask(tg, s->bin_pack.oversub, n.total_cores ? n.cpu / (int64_t)n.total_cores : 0).cpu;
        }
    }
    s->offer_row = -1;
    s->ctx.plan.node_allocation[row].push_back(a);
    return PE_OK;
}

// Plan.AppendPreemptedAlloc for each preempted alloc (generic_sched.go:794-816)
int oracle_commit_preempt(oracle_stack* s, uint32_t tgi, int32_t row, const uint32_t* preempted, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        if (preempted[i] >= s->state.allocs.size()) { s->err = "bad preempted alloc"; return PE_EINVAL; }
        const OAlloc& a = s->state.allocs[preempted[i]];
        s->ctx.plan.node_preemptions[a.node_row].push_back(a);
    }
    return oracle_commit(s, tgi, row);
}

// Plan.AppendStoppedAlloc (structs.go:10628-10660): NodeUpdate[node] += alloc
int oracle_plan_stop(oracle_stack* s, const uint32_t* allocs, uint32_t n) {
    for (uint32_t i = 0; i < n; i++)
        if (allocs[i] >= s->state.allocs.size()) { s->err = "alloc index out of range"; return PE_EINVAL; }
    for (uint32_t i = 0; i < n; i++) {
        const OAlloc& a = s->state.allocs[allocs[i]];
        s->ctx.plan.node_update[a.node_row].push_back(a);
    }
    return PE_OK;
}

// Plan.PopUpdate (structs.go:10691-10702): the node's last entry, when it is this alloc
int oracle_plan_pop_update(oracle_stack* s, uint32_t alloc) {
    if (alloc >= s->state.allocs.size()) { s->err = "alloc index out of range"; return PE_EINVAL; }
    const OAlloc& a = s->state.allocs[alloc];
    auto it = s->ctx.plan.node_update.find(a.node_row);
    if (it == s->ctx.plan.node_update.end() || it->second.empty() || it->second.back().id != a.id) return PE_OK;
    it->second.pop_back();
    if (it->second.empty()) s->ctx.plan.node_update.erase(it);
    return PE_OK;
}

int oracle_place(oracle_stack* s, uint32_t tgi, uint32_t count, pe_ranked_node* out, uint32_t* placed) {
    uint32_t p = 0;
    s->pre_overflow.clear();
    for (uint32_t i = 0; i < count; i++) {
        pe_select_options opts; std::memset(&opts, 0, sizeof(opts));
        int rc = select_rec(s, tgi, &opts, &out[i], i);
        if (rc != PE_OK) return rc;
        if (out[i].row < 0 && s->cfg.preempt && s->cfg.stack_kind == PE_STACK_GENERIC) {
            opts.preempt = 1;   // selectNextOption (generic_sched.go:786-790)
            rc = select_rec(s, tgi, &opts, &out[i], i);
            if (rc != PE_OK) return rc;
        }
        if (out[i].row < 0) break;   // failedTGAllocs: the rest of the tg is coalesced
        oracle_commit_preempt(s, tgi, out[i].row, full_preempted(s, i, out[i]), out[i].n_preempted);
        p++;
    }
    if (placed) *placed = p;
    return PE_OK;
}

int oracle_system_place(oracle_stack* s, uint32_t tgi, double* out_score, uint8_t* out_status,
                        uint32_t* placed) {
    std::vector<const ONode*> all = s->base_nodes;
    uint32_t p = 0;
    for (size_t i = 0; i < all.size(); i++) {
        s->source.SetNodes(std::vector<const ONode*>{all[i]});
        pe_ranked_node r;
        s->pre_overflow.clear();
        int rc = select_rec(s, tgi, nullptr, &r, 0);
        if (rc != PE_OK) return rc;
        if (r.row < 0) {
            out_score[i] = NAN;
            out_status[i] = s->ctx.metrics.filtered > 0 ? 1 : 2;
            continue;
        }
        out_score[i] = r.final_score; out_status[i] = 0;
        oracle_commit_preempt(s, tgi, r.row, full_preempted(s, 0, r), r.n_preempted);
        p++;
    }
    s->source.SetNodes(all);
    if (placed) *placed = p;
    return PE_OK;
}

// One Select of task group `tgi` with every visited row's outcome traced:
// status_by_row[row] = 0 option (score_by_row = FinalScore), 1 filtered,
// 2 exhausted, 255 not visited. Test hook for the sharded full-pass protocol.
int oracle_full_pass(oracle_stack* s, uint32_t tgi, uint8_t* status_by_row, double* score_by_row,
                     pe_ranked_node* out) {
    const size_t n = s->state.nodes.size();
    for (size_t i = 0; i < n; i++) { status_by_row[i] = 255; score_by_row[i] = 0.0; }
    g_trace_status = status_by_row;
    g_trace_score = score_by_row;
    pe_select_options opts;
    std::memset(&opts, 0, sizeof(opts));
    const int rc = oracle_select(s, tgi, &opts, out);
    g_trace_status = nullptr;
    g_trace_score = nullptr;
    return rc;
}

double oracle_go_pow(double x, double y) { return gomath::pow(x, y); }
double oracle_go_exp(double x) { return gomath::exp(x); }
double oracle_go_log(double x) { return gomath::log(x); }

double oracle_score_fit(int algo, int64_t cpu, int64_t mem, int64_t rcpu, int64_t rmem, int64_t ucpu, int64_t umem) {
    ONode n; n.cpu = cpu; n.mem = mem; n.rcpu = rcpu; n.rmem = rmem;
    return BinPackIterator::score_fit(algo == PE_ALGO_SPREAD, n, ucpu, umem);
}

int oracle_check_constraint(const char* op, const char* l, int ls, const char* r, int rs) {
    orasem::Caches c;
    Val lv, rv;
    lv.is_nil = ls == 0; if (ls) lv.s = l ? l : "";
    rv.is_nil = rs == 0; if (rs) rv.s = r ? r : "";
    return orasem::check_constraint(c, op, lv, rv, ls == 1, rs == 1) ? 1 : 0;
}

int oracle_limit_iter(const double* scores, int n, int limit, double threshold, int max_skip,
                      int* out_order, int* winner, int* pulled) {
    std::vector<RankedNode> nodes((size_t)n);
    StaticRankIterator src;
    for (int i = 0; i < n; i++) { nodes[i].node = nullptr; nodes[i].final_score = scores[i]; src.nodes.push_back(&nodes[i]); }
    LimitIterator lim; lim.source = &src; lim.limit = limit; lim.threshold = threshold; lim.max_skip = max_skip;
    int k = 0;
    std::vector<RankedNode*> emitted;
    for (RankedNode* o = lim.Next(); o; o = lim.Next()) { out_order[k++] = (int)(o - nodes.data()); emitted.push_back(o); }
    RankedNode* mx = nullptr;
    for (RankedNode* o : emitted) if (!mx || o->final_score > mx->final_score) mx = o;
    *winner = mx ? (int)(mx - nodes.data()) : -1;
    *pulled = src.pulled;
    return k;
}

}  // extern "C"

// ---- the iterator state a fallback GenericStack shares with the engine -----
// (test mirror of what the cgo shim reads and writes on the Go chain: the
// StaticIterator cursor, the LimitIterator limit, SpreadIterator.SetTaskGroup
// and the EvalEligibility maps of the shared EvalContext)

static uint32_t str_id(const State& st, const std::string& v) {
    for (uint32_t i = 0; i < st.strs.size(); i++)
        if (st.strs[i] == v) return i;
    return PE_NONE;
}

extern "C" int oracle_get_eligibility(oracle_stack* s, uint32_t changed_only, pe_class_feas* out, uint32_t cap,
                                      uint32_t* n, uint32_t* flags) {
    (void)changed_only;   // the oracle always reports the whole memo
    std::vector<pe_class_feas> ents;
    auto status = [](int f) { return f == kEligible ? (uint32_t)PE_CLASS_ELIGIBLE : (uint32_t)PE_CLASS_INELIGIBLE; };
    for (auto& kv : s->ctx.elig.job)
        if (kv.second == kEligible || kv.second == kIneligible)
            ents.push_back(pe_class_feas{PE_NONE, str_id(s->state, kv.first), status(kv.second)});
    for (auto& tg : s->ctx.elig.tgs)
        for (auto& kv : tg.second)
            if (kv.second == kEligible || kv.second == kIneligible)
                ents.push_back(pe_class_feas{str_id(s->state, tg.first), str_id(s->state, kv.first), status(kv.second)});
    *n = (uint32_t)ents.size();
    if (out) std::memcpy(out, ents.data(), sizeof(pe_class_feas) * std::min<size_t>(cap, ents.size()));
    if (flags) {   // HasEscaped (context.go:237-251)
        bool esc = s->ctx.elig.job_escaped;
        for (auto& kv : s->ctx.elig.tg_escaped) esc = esc || kv.second;
        *flags = esc ? PE_ELIG_ESCAPED : 0u;
    }
    return PE_OK;
}

extern "C" int oracle_put_eligibility(oracle_stack* s, const pe_class_feas* in, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        const std::string cls = S(s->state, in[i].computed_class);
        const bool e = in[i].status == PE_CLASS_ELIGIBLE;
        if (in[i].task_group == PE_NONE) s->ctx.elig.SetJobEligibility(e, cls);
        else s->ctx.elig.SetTaskGroupEligibility(e, S(s->state, in[i].task_group), cls);
    }
    return PE_OK;
}

extern "C" int oracle_get_cursor(const oracle_stack* s, uint32_t* offset, uint32_t* limit) {
    const int m = (int)s->source.nodes.size();
    if (offset) *offset = m ? (uint32_t)(s->source.offset % m) : 0u;
    if (limit) *limit = (uint32_t)s->limit.limit;
    return PE_OK;
}

extern "C" int oracle_set_cursor(oracle_stack* s, uint32_t tgi, uint32_t offset, uint32_t limit) {
    s->source.offset = (int)offset;
    s->limit.limit = (int)limit;
    if (tgi != PE_NONE && s->cfg.stack_kind == PE_STACK_GENERIC) {
        if (!s->have_job || tgi >= s->job.tgs.size()) { s->err = "bad task group"; return PE_EINVAL; }
        s->spread.SetTaskGroup(&s->tg(tgi));
    }
    return PE_OK;
}

/* AllocMetric maps of the last Select (ClassFiltered, ConstraintFiltered,
 * ClassExhausted, DimensionExhausted) as text; returns the bytes needed. */
extern "C" size_t oracle_last_metrics(const oracle_stack* s, char* buf, size_t cap) {
    const std::string t = s->ctx.metrics.Text();
    if (buf && cap) {
        const size_t k = std::min(cap - 1, t.size());
        std::memcpy(buf, t.data(), k);
        buf[k] = 0;
    }
    return t.size() + 1;
}
