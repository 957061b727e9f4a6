// Device records of the plan applier fit check (include/nomad_pe.h, pe_planner_*).
//
// evaluateNodePlan (nomad/plan_apply.go:611-674) → AllocsFit(checkDevices=true)
// (nomad/structs/funcs.go:148-211) per plan node. Everything AllocsFit decides
// besides the resource sums is a set question over small keyed multisets:
//   cores:   a core held by two counted allocs (funcs.go:166-175) or a held core
//            outside the node's available set when that set is non-empty
//            (ComparableResources.Superset, structs.go:3896-3898);
//   ports:   an (IP, port) marked twice in the NetworkIndex bitmaps
//            (network.go:196-233), node-reserved ports included (SetNode);
//   devices: a healthy node instance held twice (DeviceAccounter.AddAllocs,
//            devices.go:62-100; unknown / unhealthy instances are ignored).
// Each is order independent, so the kernel stages every key of a plan node in
// one buffer (LDS, or global scratch for very large nodes) and answers all
// three with one pairwise pass over it.
#pragma once
#include <stdint.h>

namespace pa {

constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kBigRow = 0x80000000u;   // plan row column: the node is k_plan_eval_big's

// key = kind << 60 | value
enum : uint32_t {
    K_CORE_USED = 0,   // value: core id
    K_CORE_AVAIL = 1,  // node available core
    K_PORT_USED = 2,   // value: ip id << 16 | port
    K_PORT_NODE = 3,   // node-reserved (ip, port) after SetNode (deduplicated)
    K_DEV_USED = 4,    // value: instance id << 24 | device tuple id
    K_DEV_AVAIL = 5,   // healthy node instance
};
constexpr uint64_t kValMask = (1ull << 60) - 1;

__host__ __device__ inline uint64_t make_key(uint32_t kind, uint64_t v) { return (uint64_t)kind << 60 | (v & kValMask); }

struct alignas(16) NodeRec {      // 64 B, one per snapshot node
    int64_t cpu, mem, disk;       // NodeResources − ReservedResources (funcs.go:180-181)
    uint64_t core_mask;           // available cores with id < 64 (ids >= 64 are K_CORE_AVAIL keys)
    uint32_t key_off, n_keys;     // static keys: cores >= 64, reserved ports, healthy instances
    uint32_t alloc_off, alloc_cnt;// contiguous snapshot allocs of this node in the pool
    uint32_t alloc_keys;          // Σ keys of those allocs (sizes the scratch fallback)
    uint8_t ready, eligible, setnode_collide, has_cores;
    uint32_t ext_head;            // first chunk of allocs appended by commits (kNone: none)
    uint32_t _pad;
};
static_assert(sizeof(NodeRec) == 64, "NodeRec is 64 bytes");

// Allocs appended to a node by pe_planner_commit since the last compaction:
// pool[off, off + cnt), chained newest first.
struct alignas(16) Chunk {
    uint32_t off, cnt, next, _pad;
};

struct alignas(16) AllocRec {     // 32 B, snapshot pool entry or plan alloc
    int64_t cpu, mem, disk;
    uint32_t key_off;
    uint16_t n_keys;
    uint8_t terminal;
    uint8_t bad_port;             // a port outside [0, 65536): AddReserved* returns collide
};
static_assert(sizeof(AllocRec) == 32, "AllocRec is 32 bytes");

// A plan alloc (16 B): its keys and its resources, an index into the plan's
// table of distinct (cpu, memory, disk) triples (the allocs of one task group
// share one). Plan nodes travel as three u32 columns: snapshot row (kNone:
// unknown; | kBigRow when the node's key bound passes the LDS budget),
// place_off[n + 1] (the caller's own column) and, when the plan removes live
// allocs, rm_off[n + 1] into the sorted removal lists.
struct alignas(16) PlanAllocRec {
    uint32_t key_off;
    uint16_t n_keys;
    uint8_t terminal;
    uint8_t bad_port;
    uint32_t res;
    uint32_t _pad;
};
static_assert(sizeof(PlanAllocRec) == 16, "PlanAllocRec is 16 bytes");

struct PlanRes {
    int64_t cpu, mem, disk;
};
static_assert(sizeof(PlanRes) == 24, "PlanRes is 24 bytes");

struct BigNode {                  // a plan node past the LDS budget (k_plan_eval_big)
    uint32_t p;                   // plan node index
    uint32_t scratch_off;         // its global key scratch
};

// k_plan_eval<G>: a group of G lanes per plan node (64/G nodes per wavefront),
// keys staged in a per-node LDS buffer of lds_keys(G) (16 KiB per workgroup);
// plan nodes whose key bound (node keys + snapshot alloc keys + plan alloc
// keys, the same sum on host and device) exceeds it go to k_plan_eval_big (one
// wavefront each, global scratch). The host picks G (pe_planner, PE_PLAN_GROUP).
constexpr int kWaves = 4;                               // waves per workgroup
__host__ __device__ constexpr int nodes_per_block(int g) { return kWaves * (64 / g); }
__host__ __device__ constexpr uint32_t lds_keys(int g) { return 2048u / (uint32_t)(kWaves * (64 / g)); }
constexpr uint64_t kHole = ~0ull;                       // staged slot of a masked core (kind 15)

struct PlanArgs {
    const NodeRec* nodes;
    const Chunk* chunks;
    const AllocRec* pool;            // snapshot allocs, grouped by node
    const uint64_t* node_keys;
    const uint64_t* pool_keys;
    const uint32_t* prow;            // plan node -> snapshot row (kNone: unknown node)
    const uint32_t* poff;            // [n_plan + 1] plan allocs of each plan node
    const uint32_t* rmoff;           // [n_plan + 1] removals of each plan node (null: none)
    uint32_t n_plan;
    const uint32_t* rm;              // removed pool indices, sorted per plan node
    const PlanAllocRec* pallocs;     // plan allocs
    const PlanRes* pres;             // their distinct resource triples
    const uint64_t* pkeys;
    uint64_t* scratch;
    const BigNode* big;              // plan nodes past the LDS budget
    uint32_t n_big;
    uint8_t* reason;
};

}  // namespace pa
