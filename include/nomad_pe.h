/*
 * nomad_pe.h — C ABI of the MI355X placement engine for Nomad's scheduler hot path.
 *
 * The engine replaces the placement stack behind `scheduler.Stack`
 * (reference: scheduler/stack.go:23-32 — SetNodes / SetJob / Select) for the
 * GenericStack (stack.go:41-179, 336-431) and SystemStack (stack.go:181-333).
 * The Go callers (GenericScheduler.computePlacements, generic_sched.go:472-652;
 * SystemScheduler.computePlacements, scheduler_system.go:283-425) stay
 * unchanged; a cgo shim flattens structs.Node / structs.Job
 * into the POD tables below and calls these entry points.
 *
 * Conventions
 *  - Plain pointers and sizes only; every pointer is borrowed for the duration
 *    of the call (cgo pointer rules) and copied by the engine.
 *  - Strings are interned by the caller: one table per state snapshot
 *    (pe_strtab), every string field is a uint32 id into it; equal strings must
 *    share one id. PE_NONE marks "absent" where a field is optional.
 *  - Every function returns 0 on success or a negative PE_E* code; the message
 *    is available from pe_last_error(handle). "No feasible node" is NOT an
 *    error: Select writes row = -1, exactly like a nil *RankedNode.
 *  - A handle is used by one thread at a time (one Stack per eval worker,
 *    nomad/worker.go:244-274). Handles are independent.
 */
#ifndef NOMAD_PE_H
#define NOMAD_PE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PE_ABI_VERSION 9u
#define PE_NONE 0xFFFFFFFFu
#define PE_MAX_SCORES 8
#define PE_MAX_PREEMPT 16   /* PreemptedAllocs carried inline per RankedNode (the
                               full list of a longer one: pe_preempted_of) */
#define PE_MAX_DEVICE_REQ 4 /* device requests of a task group on the device path */
#define PE_MAX_DEVICES 8    /* GPUs one handle drives (pe_config.device_ids) */

/* ---- status codes ------------------------------------------------------ */
#define PE_OK 0
#define PE_EINVAL (-1)       /* malformed input */
#define PE_ESTATE (-2)       /* call order violated (e.g. Select before SetJob) */
#define PE_EHIP (-3)         /* HIP runtime failure */
#define PE_EUNSUPPORTED (-4) /* feature not on the device path (CSI, cores, ...):
                                the shim falls back to the Go chain for this Select */
#define PE_ENOMEM (-5)
#define PE_EINTERNAL (-6)    /* an engine invariant failed on the device (a kernel bounds guard tripped);
                                the call is abandoned, the handle must be reset (pe_set_state) */

/* ---- interned strings -------------------------------------------------- */
typedef struct pe_strtab {
    const char* bytes;        /* concatenated bytes */
    const uint32_t* offsets;  /* count+1 entries; string i = bytes[offsets[i], offsets[i+1]) */
    uint32_t count;
} pe_strtab;

/* ---- typed device attribute (plugins/shared/structs/attribute.go:39-61) -- */
#define PE_ATTR_INT 1
#define PE_ATTR_FLOAT 2
#define PE_ATTR_STRING 3
#define PE_ATTR_BOOL 4
typedef struct pe_attr {
    uint32_t kind;    /* PE_ATTR_* */
    uint32_t unit;    /* str id of the unit ("" if none) */
    int64_t i;        /* int / bool value */
    double f;         /* float value */
    uint32_t s;       /* str id for string values */
    uint32_t _pad;
} pe_attr;

/* ---- node table: the structs.Node fields the hot path reads -------------
 * (nomad/structs/structs.go:1812-1914). One row per node of the State
 * snapshot. CSR lists use off[n+1].                                         */
typedef struct pe_node_table {
    uint32_t n;
    const uint32_t* id;              /* Node.ID                     */
    const uint32_t* name;            /* Node.Name                   */
    const uint32_t* datacenter;      /* Node.Datacenter             */
    const uint32_t* node_class;      /* Node.NodeClass              */
    const uint32_t* computed_class;  /* Node.ComputedClass (node_class.go:31) */
    const int64_t* cpu_shares;       /* NodeResources.Cpu.CpuShares */
    const int64_t* memory_mb;        /* NodeResources.Memory.MemoryMB */
    const int64_t* disk_mb;          /* NodeResources.Disk.DiskMB   */
    const int64_t* reserved_cpu;     /* ReservedResources.Cpu.CpuShares */
    const int64_t* reserved_memory_mb;
    const int64_t* reserved_disk_mb;
    /* Attributes / Meta maps */
    const uint32_t* attr_off; const uint32_t* attr_key; const uint32_t* attr_val;
    const uint32_t* meta_off; const uint32_t* meta_key; const uint32_t* meta_val;
    /* Drivers map: flags bit0 Detected, bit1 Healthy, bit2 DriverInfo==nil */
    const uint32_t* drv_off; const uint32_t* drv_name; const uint8_t* drv_flags;
    /* NodeResources.Networks: mode ("" = host), device, MBits */
    const uint32_t* net_off; const uint32_t* net_mode; const uint32_t* net_device;
    const int32_t* net_mbits;
    /* NodeResources.NodeNetworks[*].Addresses[*].Alias (host networks) */
    const uint32_t* alias_off; const uint32_t* alias_name;
    /* node-reserved host ports that fall in the dynamic range [20000,32000) */
    const int32_t* reserved_dyn_ports;
    /* HostVolumes map */
    const uint32_t* hv_off; const uint32_t* hv_name; const uint8_t* hv_read_only;
    /* NodeResources.Devices (device groups) */
    const uint32_t* dev_off;
    const uint32_t* dev_vendor; const uint32_t* dev_type; const uint32_t* dev_name;
    const uint32_t* dev_healthy;     /* healthy instance count */
    const uint32_t* dev_attr_off;    /* CSR over device groups */
    const uint32_t* dev_attr_key; const pe_attr* dev_attr_val;
    /* NodeResources.Cpu.ReservableCpuCores (CSR over nodes) and TotalCpuCores;
       ReservedResources.Cpu.ReservedCpuCores (CSR). NULL: no core sets */
    const uint32_t* core_off; const uint16_t* core_id;
    const uint32_t* total_cores;
    const uint32_t* rsv_core_off; const uint16_t* rsv_core_id;
    /* NodeResources.NodeNetworks[*].Addresses[*] in node order (CSR): Alias,
       Address and its ReservedPorts spec (ParsePortRanges syntax, PE_NONE =
       none); ReservedResources.Networks.ReservedHostPorts per node (PE_NONE =
       none). NULL: no addresses (static port asks then find none) */
    const uint32_t* addr_off; const uint32_t* addr_alias; const uint32_t* addr_ip;
    const uint32_t* addr_rsv_ports;
    const uint32_t* rsv_host_ports;
    /* NodeResources.Networks[*] addresses (str ids, per net_off entry): the IP
       field (PE_NONE = "") and the one address AssignNetwork yields from the
       CIDR (yieldIP, network.go:294-315; PE_NONE when the CIDR does not parse
       or holds more than one address). NULL: unknown (task-level static ports
       are then not on the device path) */
    const uint32_t* net_ip; const uint32_t* net_cidr_ip;
} pe_node_table;

/* ---- existing allocations of the snapshot (state AllocsByNode) ---------- */
typedef struct pe_alloc_table {
    uint32_t count;
    const uint32_t* node_row;        /* row in pe_node_table          */
    const uint32_t* ns;              /* Allocation.Namespace          */
    const uint32_t* job_id;          /* Allocation.JobID              */
    const uint32_t* task_group;      /* Allocation.TaskGroup          */
    const uint8_t* terminal;         /* Allocation.TerminalStatus()   */
    const int32_t* priority;         /* Allocation.Job.Priority       */
    const int64_t* cpu_shares;       /* ComparableResources().Flattened.Cpu.CpuShares */
    const int64_t* memory_mb;        /* ...Flattened.Memory.MemoryMB  */
    const int64_t* disk_mb;          /* ...Shared.DiskMB              */
    const int32_t* net_mbits;        /* bandwidth held on the node's host device */
    const int32_t* dyn_ports;        /* ports held in [20000,32000)  */
    /* device instances held: CSR over allocs, (device group index on its node, count) */
    const uint32_t* dev_off; const uint32_t* dev_group; const uint32_t* dev_count;
    /* TaskGroup.Migrate.MaxParallel of the alloc's job, or NULL = 0 for every
       alloc (Preemptor.SetCandidates, scheduler/preemption.go:141-154) */
    const int32_t* max_parallel;
    /* ComparableResources().Flattened.Cpu.ReservedCores (CSR over allocs), or NULL */
    const uint32_t* core_off; const uint16_t* core_id;
    /* ports the alloc holds (NetworkIndex.AddAllocs: AllocatedPorts HostIP /
       Value, or the pre-0.12 networks' IP and ports), CSR over allocs, or NULL */
    const uint32_t* port_off; const uint32_t* port_ip; const int32_t* port_value;
    /* ComparableResources().Flattened.Networks is non-empty (the alloc takes
       part in PreemptForNetwork, preemption.go:302-331), or NULL: derived as
       net_mbits > 0 || dyn_ports > 0 || the alloc holds ports */
    const uint8_t* has_network;
    /* the Device of the alloc's networks (NetworkResource.Device; string id),
       or PE_NONE / NULL: the node's first host network device. Bandwidth is
       kept per device (NetworkIndex.UsedBandwidth[device], network.go:196-230);
       a Select with Preempt whose PreemptForNetwork candidates sit on two
       devices returns PE_EUNSUPPORTED (the reference ranges over a Go map) */
    const uint32_t* net_device;
} pe_alloc_table;

/* ---- job specification (structs.Job / TaskGroup / Task) ----------------- */
typedef struct pe_constraint { uint32_t ltarget, rtarget, operand; } pe_constraint;
typedef struct pe_affinity { uint32_t ltarget, rtarget, operand; int32_t weight; } pe_affinity;
typedef struct pe_spread_target { uint32_t value; int32_t percent; } pe_spread_target;
typedef struct pe_spread {
    uint32_t attribute; int32_t weight;       /* weight is an int8 in structs.Spread */
    uint32_t target_off, target_count;        /* into pe_job.spread_targets */
} pe_spread;
typedef struct pe_device_request {           /* structs.RequestedDevice */
    uint32_t name; uint32_t _pad; uint64_t count;
    uint32_t constraint_off, constraint_count; /* into pe_job.device_constraints */
    uint32_t affinity_off, affinity_count;     /* into pe_job.device_affinities  */
} pe_device_request;
#define PE_LC_MAIN 0
#define PE_LC_PRESTART 1
#define PE_LC_PRESTART_SIDECAR 2
#define PE_LC_POSTSTOP 3
#define PE_LC_POSTSTART 4   /* not counted by AllocatedResources.Comparable() */
typedef struct pe_task {
    uint32_t name, driver;
    int64_t cpu, memory_mb, memory_max_mb;
    int32_t cores;                            /* Resources.Cores: reserved cores (rank.go:437-466) */
    uint32_t lifecycle;                       /* PE_LC_* */
    int32_t has_network, net_mbits, net_dyn_ports, net_reserved_ports;
    uint32_t constraint_off, constraint_count;
    uint32_t affinity_off, affinity_count;
    uint32_t device_off, device_count;
    uint32_t rport_off;                       /* the task network's ReservedPorts (static ports):
                                                 pe_job.rport_value / rport_label [rport_off,
                                                 rport_off + net_reserved_ports) */
} pe_task;
typedef struct pe_task_group {
    uint32_t name; int32_t count;
    int64_t ephemeral_disk_mb;
    uint32_t constraint_off, constraint_count;
    uint32_t affinity_off, affinity_count;
    uint32_t spread_off, spread_count;
    uint32_t task_off, task_count;
    int32_t has_network; uint32_t net_mode;   /* tg Networks[0] */
    int32_t net_dyn_ports, net_reserved_ports;
    uint32_t net_host_network;                /* host network alias of the ports ("default") */
    uint32_t volume_off, volume_count;        /* host volume requests */
    int32_t has_csi_volumes;                  /* CSI: not on the device path */
    uint32_t rport_off, rport_count;          /* tg network ReservedPorts (static ports): into
                                                 pe_job.rport_value / rport_label */
} pe_task_group;
#define PE_JOB_SERVICE 0
#define PE_JOB_BATCH 1
#define PE_JOB_SYSTEM 2
#define PE_JOB_SYSBATCH 3
typedef struct pe_job {
    uint32_t id, ns, type; int32_t priority;
    uint64_t version;
    uint32_t constraint_off, constraint_count;
    uint32_t affinity_off, affinity_count;
    uint32_t spread_off, spread_count;
    uint32_t tg_count;
    const pe_task_group* task_groups;
    const pe_task* tasks;
    const pe_constraint* constraints;        /* job, tg and task constraints */
    const pe_affinity* affinities;
    const pe_spread* spreads;
    const pe_spread_target* spread_targets;
    const pe_device_request* devices;
    const pe_constraint* device_constraints;
    const pe_affinity* device_affinities;
    const uint32_t* volume_source;           /* host volume requests: source name */
    const uint8_t* volume_read_only;
    const int32_t* rport_value;              /* static ports: Port.Value and Port.Label */
    const uint32_t* rport_label;
} pe_job;

/* ---- stack configuration (SchedulerConfiguration, operator.go:128-210) --- */
#define PE_STACK_GENERIC 0
#define PE_STACK_SYSTEM 1
#define PE_ALGO_BINPACK 0
#define PE_ALGO_SPREAD 1
typedef struct pe_config {
    uint32_t stack_kind;      /* PE_STACK_* */
    uint32_t batch;           /* GenericStack batch flag (limit 2) */
    uint32_t algorithm;       /* PE_ALGO_* */
    uint32_t memory_oversubscription;
    uint32_t preempt;         /* SystemStack: BinPack eviction enabled (stack.go:267-278).
                                 GenericStack: PreemptionConfig.{Service,Batch}SchedulerEnabled:
                                 pe_place retries a nil Select with Preempt=true
                                 (selectNextOption, generic_sched.go:773-792) */
    int32_t device;           /* HIP device ordinal (device_count <= 1) */
    /* One handle over several GPUs of this process (SURVEY.md §8b "device
     * count/ids"): device_ids[0] holds the handle's own state, the others
     * replicas of it; full-pass count loops (pe_place of task groups with
     * affinities / spreads) and pe_system_place split the rows over all of
     * them, exchanging per-placement records with ncclAllGather over
     * communicators from ncclCommInitAll. Ids that all name one GPU run the
     * same split with device copies instead of RCCL (loopback, for tests).
     * 0 or 1: the single `device`. */
    uint32_t device_count;
    int32_t device_ids[PE_MAX_DEVICES];
} pe_config;

typedef struct pe_select_options {              /* SelectOptions, stack.go:34-39 */
    const uint32_t* penalty_rows; uint32_t penalty_count;
    const uint32_t* preferred_rows; uint32_t preferred_count;
    uint32_t preempt;
} pe_select_options;

typedef struct pe_ranked_node {                 /* RankedNode, rank.go:21-36 */
    int32_t row;              /* chosen node row, -1 = nil */
    uint32_t n_scores;
    double final_score;
    double scores[PE_MAX_SCORES];   /* rank order: binpack, device-aff, anti-aff,
                                       penalty, node-aff, spread, preemption */
    /* AllocMetric side outputs (structs.go:9826-10026) */
    uint32_t nodes_evaluated, nodes_filtered, nodes_exhausted;
    uint32_t new_offset;      /* StaticIterator cursor after the Select */
    /* PreemptedAllocs (rank.go:511-513): rows of the pe_alloc_table snapshot;
       n_preempted is the whole count, the first PE_MAX_PREEMPT are inline */
    uint32_t n_preempted;
    uint32_t preempted[PE_MAX_PREEMPT];
    /* TaskResources device offers (rank.go:404-405): per device request of the
       task group (tasks in order), the index of the chosen device group on the node */
    uint32_t n_device_offers;
    uint32_t device_offer_group[PE_MAX_DEVICE_REQ];
    /* Cpu.ReservedCores of the task group's tasks (rank.go:437-466): bit c =
       core c; tasks asking cores take them in task order, lowest ids first */
    uint64_t reserved_cores[4];
} pe_ranked_node;

typedef struct pe_placement {                   /* compact per-placement record (batches) */
    int32_t row;              /* chosen node row, -1 = nil (count loop stopped) */
    uint32_t nodes_evaluated;
    double final_score;
} pe_placement;

/* ---- entry points -------------------------------------------------------- */
typedef struct pe_stack pe_stack;

uint32_t pe_abi_version(void);
/* NewGenericStack (stack.go:336) / NewSystemStack (stack.go:207) */
pe_stack* pe_stack_create(const pe_config* cfg);
void pe_stack_destroy(pe_stack* s);
const char* pe_last_error(const pe_stack* s);
/* State snapshot: nodes + non-terminal allocs (scheduler.State, scheduler.go:66-110).
 * Uploads the node SoA to HBM; stays resident across evals until replaced. */
int pe_set_state(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes,
                 const pe_alloc_table* allocs);
/* Start a new evaluation on the resident snapshot: drop the plan (proposed
 * allocs), the EvalEligibility memo and the job (NewEvalContext, context.go:86).
 * The node SoA stays in HBM; only the dynamic columns are restored. */
/* Apply an allocation delta of the state store to the resident snapshot
 * without reloading the nodes (client-status changes that make allocs
 * terminal, allocs placed by other workers' applied plans; nomad/state
 * UpsertAllocs / UpsertPlanResults). Entry i overwrites snapshot alloc
 * index[i], or is appended when index[i] == PE_NONE (or index == NULL); the
 * appended ones take the next indices in order. `strs` extends the snapshot's
 * string table (same ids for the strings it already had). Equivalent to
 * pe_set_state with the updated table: the plan, the memo and the job are
 * reset (a state change starts a new evaluation). */
int pe_update_allocs(pe_stack* s, const pe_strtab* strs, const pe_alloc_table* allocs, const uint32_t* index);
int pe_reset_plan(pe_stack* s);
/* Node upserts into the resident snapshot (state_store.go UpsertNode and the
 * node_endpoint.go Register / UpdateStatus / UpdateDrain paths, with
 * Node.ComputeClass computed by the caller, node_class.go:31-104): row i of
 * `nodes` replaces snapshot row index[i], or is appended when index is NULL
 * or index[i] == PE_NONE (appended rows take the next row numbers in order).
 * The allocs stay; a node's allocs keep their rows. Like pe_update_allocs it
 * starts a new evaluation context (pe_set_job / pe_set_nodes again). */
int pe_update_nodes(pe_stack* s, const pe_strtab* strs, const pe_node_table* nodes, const uint32_t* index);
/* Stack.SetJob (stack.go:93-115 / 290-299). `strs` extends the table given to
 * pe_set_state (same ids for its first entries, job strings appended). */
int pe_set_job(pe_stack* s, const pe_strtab* strs, const pe_job* job);
/* Stack.SetNodes (stack.go:71-91 / 285-288). `rows` is the node list AFTER the
 * caller's shuffleNodes (util.go:366-372): the engine draws no randomness.
 * Writes the LimitIterator limit to *limit_out (may be NULL). */
int pe_set_nodes(pe_stack* s, const uint32_t* rows, uint32_t n, uint32_t* limit_out);
/* Stack.Select (stack.go:117-179 / 301-333) */
int pe_select(pe_stack* s, uint32_t tg_index, const pe_select_options* opts,
              pe_ranked_node* out);
/* Plan.AppendAlloc (structs.go:10707-10714) of an allocation of task group
 * `tg_index` on node `row`: the proposed state seen by later Selects.
 *
 * Speculation (transparent to the caller): the first plain Select of a task
 * group (no preferred / penalty nodes, no Preempt, metrics off) runs the
 * device count loop for the group's remaining placements and returns its first
 * record; while every pe_commit names the row the previous Select returned,
 * later plain Selects of that group are answered from the loop's records with
 * no device work. Any other call first restores the device state to the
 * committed prefix, so results always equal one-at-a-time Selects.
 * PE_SPECULATE=0 in the environment disables it. */
int pe_commit(pe_stack* s, uint32_t tg_index, int32_t row);
/* Apply queued device work now: the speculative count loop's confirmed
 * placements and the SystemScheduler fast path's queued commits (every entry
 * point that reads the device state does this itself; callers use it to
 * settle the device at a point of their choosing). */
int pe_flush(pe_stack* s);
/* SystemStack fast path counters: out[0] k_system passes over the snapshot
 * that filled the per-row cache, out[1] single-node Selects answered from it. */
int pe_system_spec_stats(const pe_stack* s, uint64_t* out2);
/* GPUs this handle drives (pe_config.device_count; 1 for a single device). */
uint32_t pe_device_count(const pe_stack* s);
/* Multi-GPU: one engine handle per GPU and process, joined by
 * an RCCL communicator (ncclGetUniqueId on one rank, the 128 bytes shared by
 * the caller, ncclCommInitRank on every rank). */
int pe_comm_unique_id(uint8_t* out, size_t cap);
/* The RCCL library the collectives call, bound at first use: the one the
 * process already has mapped (soname librccl.so.1, e.g. torch's), else
 * /opt/rocm/lib/librccl.so.1, followed by " (RCCL major.minor.patch)"; ""
 * when none loads or its major version differs from the rccl.h the engine is
 * built against (the communicator calls then fail with that reason). */
const char* pe_comm_library(void);
int pe_comm_init(pe_stack* s, int nranks, int rank, const uint8_t* id);
/* A caller-provided transport instead of RCCL (ranks on hosts without an
 * RCCL path between them, or the CPU rehearsal of the per-GPU processes):
 * exchange(ctx, send, recv, bytes) is an all-gather in rank order, `bytes`
 * from this rank into recv[rank * bytes], returning 0 on success. It is called
 * from the thread inside pe_place_sharded once per placement, on host buffers
 * (the record crosses PCIe both ways). Replaces any RCCL communicator. */
typedef int (*pe_exchange_fn)(void* ctx, const void* send, void* recv, size_t bytes);
int pe_comm_init_host(pe_stack* s, int nranks, int rank, pe_exchange_fn exchange, void* ctx);
/* The full-pass count loop (task groups with affinities / spreads, limit >=
 * list) sharded over the ranks: every rank holds the whole snapshot, job and
 * SetNodes list and sweeps its rows [row_begin, row_end) into one 80-byte
 * record (the sweep's last workgroup merges the rank's workgroup records);
 * per placement one ncclAllGather of the ranks' records on the engine stream
 * (nranks x 80 B), then every rank resolves and commits the same winner.
 * Every rank receives the same records. Windowed task groups return
 * PE_EUNSUPPORTED (replicas only). */
int pe_place_sharded(pe_stack* s, uint32_t tg_index, uint32_t count, uint32_t row_begin, uint32_t row_end,
                     pe_ranked_node* out, uint32_t* placed);
/* Device time of the all-gather in the last pe_place_sharded (microseconds,
 * mean over every placement; includes waiting for peer ranks). */
double pe_last_exchange_us(const pe_stack* s);
/* The same as out4 = {mean, min, max} microseconds and the placements timed
 * (0 at one rank: no exchange runs). */
int pe_last_exchange_stats(const pe_stack* s, double* out4);
/* Counters of the speculative loop: out[0] runs started, [1] Selects answered
 * from records, [2] rollbacks (the caller deviated), [3] records computed. */
int pe_speculation_stats(const pe_stack* s, uint64_t* out4);
/* Plan.AppendAlloc plus Plan.AppendPreemptedAlloc of each preempted alloc
 * (handlePreemptions, generic_sched.go:794-816): `preempted` are alloc-table
 * rows, as returned in pe_ranked_node.preempted by a Select with Preempt. */
int pe_commit_preempt(pe_stack* s, uint32_t tg_index, int32_t row, const uint32_t* preempted,
                      uint32_t n_preempted);
/* The full PreemptedAllocs of record `record` of the last pe_select (record 0)
 * or pe_place (record k) when it holds more than PE_MAX_PREEMPT (rank.go:511-513
 * has no cap): writes min(cap, n) alloc-table rows, the first PE_MAX_PREEMPT
 * equal to the inline ones, and returns n; PE_ESTATE when that record carries
 * its whole list inline. Valid until the next pe_select / pe_place /
 * pe_system_place. The Go shim calls it when n_preempted > PE_MAX_PREEMPT,
 * before pe_commit_preempt(row, list, n). Replaces reading
 * RankedNode.PreemptedAllocs past the inline array (rank.go:511-513). */
int pe_preempted_of(const pe_stack* s, uint32_t record, uint32_t* out, uint32_t cap);
/* Plan.AppendStoppedAlloc (structs.go:10628-10660) of `n` snapshot allocs
 * (alloc-table rows): each becomes a NodeUpdate entry of its node, and a
 * non-terminal one leaves the proposed state of the node
 * (EvalContext.ProposedAllocs, context.go:120-157: resources, devices, the
 * job's collision counts; the property sets count it as cleared,
 * propertyset.go:159-209). The stops of computeJobAllocs
 * (generic_sched.go:382), of a destructive update's previous alloc (:546), of
 * inplaceUpdate / genericAllocUpdateFn (util.go:749, 1037) and of the
 * SystemScheduler (scheduler_system.go:230-241). Undone by pe_reset_plan. */
int pe_plan_stop(pe_stack* s, const uint32_t* allocs, uint32_t n);
/* Plan.PopUpdate (structs.go:10691-10702): drops the last NodeUpdate entry of
 * the alloc's node when it is this alloc (generic_sched.go:644, util.go:756,
 * 1043); otherwise nothing happens. */
int pe_plan_pop_update(pe_stack* s, uint32_t alloc);
/* Fused count loop of GenericScheduler.computePlacements (generic_sched.go:493-649)
 * for `count` fresh placements of one task group (no preferred / penalty nodes):
 * Select -> AppendAlloc repeated on the device; stops at the first nil option
 * (failedTGAllocs short-circuit, generic_sched.go:519-523).
 * out[count] receives each placement; *placed the number placed. */
int pe_place(pe_stack* s, uint32_t tg_index, uint32_t count, pe_ranked_node* out,
             uint32_t* placed);
/* Concurrent evaluations (NumSchedulers workers, nomad/config.go:468; each
 * worker runs one eval against its snapshot, nomad/worker.go:244-274).
 * pe_stage_orders copies `n_evals` visit orders (each a shuffled SetNodes list
 * of length n, row ids) to HBM. pe_place_batch then runs, for every staged
 * order, an independent evaluation of `count` placements of task group
 * `tg_index` from the stack's current plan (offset 0), exactly as
 * SetNodes(order) + pe_place would, without modifying the stack's plan.
 * out[n_evals * count] (row-major by eval), placed[n_evals]; either may be NULL:
 * the results always land in a stack-owned page-locked buffer first, readable
 * in place through pe_batch_results until the next pe_place_batch. The host
 * preparation (fresh-memo feasibility tables, limit) is reused across calls
 * until a mutating call (set_state / set_job / stage_orders / select / ...). */
int pe_stage_orders(pe_stack* s, const uint32_t* orders, uint32_t n_evals, uint32_t n);
int pe_place_batch(pe_stack* s, uint32_t tg_index, uint32_t count, pe_placement* out,
                   uint32_t* placed);
/* Results of the last pe_place_batch: out[n_evals * count]; status[2 * e] =
 * placements of eval e, status[2 * e + 1] = its final StaticIterator offset. */
int pe_batch_results(const pe_stack* s, const pe_placement** out, const uint32_t** status,
                     uint32_t* n_evals, uint32_t* count);
/* Phases of the last pe_place_batch in ms: [0] host preparation, [1] kernel
 * (HIP events), [2] device-to-host result copy (HIP events), [3] call total. */
void pe_last_phase_ms(const pe_stack* s, double* out4);
/* SystemScheduler.computePlacements (scheduler_system.go:283-425) for one task
 * group over every row of the SetNodes list: one single-node Select per row.
 * out_row_score[n] = FinalScore or NaN when filtered/exhausted;
 * out_status[n] = 0 placed, 1 filtered, 2 exhausted. Commits placed allocs.
 * Both arrays NULL: the results stay in the engine's page-locked staging,
 * read through pe_system_results (no copy into caller memory). */
int pe_system_place(pe_stack* s, uint32_t tg_index, double* out_score,
                    uint8_t* out_status, uint32_t* placed);
/* The last pe_system_place's results in the engine's staging (score[n],
 * status[n], as above), valid until the next pe_system_place on the handle. */
int pe_system_results(const pe_stack* s, const double** score, const uint8_t** status, uint32_t* n);
/* Full-scan Select sharded over GPUs (one process per GPU, each holding the
 * same snapshot, job, SetNodes list and plan). Each rank sweeps
 * the snapshot rows [row_begin, row_end) it owns into a pe_shard_rec: the
 * LimitIterator/MaxScoreIterator state of its rows (max score and its earliest
 * visit ranks, the first three non-positive options, option / filter / exhaust
 * counts), which merges associatively. After one all-gather of the records,
 * every rank calls pe_select_merge with all of them and gets the same Select
 * result (stack.go:117-179 with limit MaxInt32; a full pass leaves the cursor
 * unchanged), then commits it with pe_commit. Needs a full pass (affinities or
 * spreads), a visit list without repeated rows and no distinct_property. */
typedef struct pe_shard_rec { uint8_t bytes[80]; } pe_shard_rec;
int pe_select_shard(pe_stack* s, uint32_t tg_index, uint32_t row_begin, uint32_t row_end, pe_shard_rec* out);
int pe_select_merge(pe_stack* s, uint32_t tg_index, const pe_shard_rec* recs, uint32_t n_recs,
                    pe_ranked_node* out);
/* Milliseconds spent in device kernels by the last pe_place / pe_system_place
 * (HIP events on the engine's stream). */
double pe_last_kernel_ms(const pe_stack* s);
/* Algorithmic HBM bytes per node of the last full-scan sweep Select (73 with
 * the verdict byte, 76 with the folded per-node score word), 0 if none ran. */
uint32_t pe_last_sweep_bytes(const pe_stack* s);
/* Per-kernel device time of the windowed count loop (measurement aid; off by
 * default, or PE_KERNEL_SPLIT=1 in the environment at pe_stack_create): with it
 * on, the chain path records HIP events between its kernels and
 * pe_last_kernel_split writes the last launch's ms4 = {k_base, k_chain, k_emit,
 * k_emit_writeback}; PE_ESTATE when the last pe_place / Select ran no chain. */
int pe_set_kernel_split(pe_stack* s, int on);
int pe_last_kernel_split(const pe_stack* s, double* ms4);
/* AllocMetric maps (structs.go:9826-10026) of Selects: ClassFiltered,
 * ConstraintFiltered, ClassExhausted, DimensionExhausted — what
 * `ctx.Metrics()` holds after GenericStack.Select (FilterNode / ExhaustedNode,
 * structs.go:9907-9937). Off by default; switch on before the first Select of
 * an evaluation (the maps depend on the EvalEligibility memo history).
 * Available for every Select: plain, with preferred nodes, and with Preempt
 * (BinPack with evict per visited row, k_evict_trace). */
int pe_set_metrics(pe_stack* s, int on);
/* The last Select's maps as text lines "KIND\tKEY\tCOUNT\n", KIND one of
 * CF / KF / CE / DE, keys sorted. Writes at most cap bytes (NUL-terminated) and
 * returns the bytes needed, or PE_ESTATE when the last Select has none. */
int64_t pe_last_metrics(const pe_stack* s, char* buf, size_t cap);
/* The same maps in binary form (what the Go shim turns into AllocMetric
 * without parsing text): count entries {kind, key, count} and the
 * ScoreMetaData items in GetItemsReverse order (NormScore descending, Go's
 * heap order for equal scores). A key without PE_METRIC_ENGINE_KEY is a
 * string id of the caller's table (the node classes of ClassFiltered /
 * ClassExhausted); a key with it names an engine string (checker reasons,
 * dimensions: pe_metric_string), stable for the handle's life. The arrays
 * stay valid until the next Select or state call. PE_ESTATE when the last
 * Select has no maps. */
#define PE_METRIC_ENGINE_KEY 0x80000000u
#define PE_METRIC_CLASS_FILTERED 1u       /* AllocMetric.ClassFiltered[key]       */
#define PE_METRIC_CONSTRAINT_FILTERED 2u  /* AllocMetric.ConstraintFiltered[key]  */
#define PE_METRIC_CLASS_EXHAUSTED 3u      /* AllocMetric.ClassExhausted[key]      */
#define PE_METRIC_DIMENSION_EXHAUSTED 4u  /* AllocMetric.DimensionExhausted[key]  */
typedef struct pe_metric_count {
    uint32_t kind;    /* PE_METRIC_* */
    uint32_t key;     /* string id (see above) */
    uint32_t count;
} pe_metric_count;
/* NodeScoreMeta.Scores names (the ScoreNode scorers, in the order they ran) */
#define PE_SCORER_BINPACK 0u
#define PE_SCORER_DEVICES 1u
#define PE_SCORER_JOB_ANTI_AFFINITY 2u
#define PE_SCORER_RESCHEDULE_PENALTY 3u   /* "node-reschedule-penalty" */
#define PE_SCORER_NODE_AFFINITY 4u
#define PE_SCORER_ALLOCATION_SPREAD 5u
#define PE_SCORER_PREEMPTION 6u
typedef struct pe_metric_score {
    int32_t row;                      /* NodeID: the node table row */
    uint32_t n_scores;
    double norm;                      /* NormScore */
    uint8_t scorer[PE_MAX_SCORES];    /* PE_SCORER_* */
    double score[PE_MAX_SCORES];
} pe_metric_score;
int pe_last_metrics_bin(const pe_stack* s, const pe_metric_count** counts, uint32_t* n_counts,
                        const pe_metric_score** scores, uint32_t* n_scores);
/* The text of metric key `key` (an engine string or a caller string id):
 * writes at most cap bytes (NUL-terminated), returns the bytes needed or
 * PE_EINVAL for an unknown key. Scorer names: pe_scorer_name. */
int64_t pe_metric_string(const pe_stack* s, uint32_t key, char* buf, size_t cap);
const char* pe_scorer_name(uint32_t scorer);
/* EvalEligibility (scheduler/context.go:190-356) as the reference chain would
 * hold it after this evaluation's Selects: the job-level and per task group
 * ComputedClassFeasibility entries FeasibilityWrapper.Next writes for every
 * node the chain pulls (feasible.go:1061-1153). createBlockedEval /
 * ReblockEval read GetClasses() and HasEscaped() from it
 * (generic_sched.go:177-181, 193-203); the shim mirrors the entries into
 * ctx.Eligibility() after each Select (changed_only = 1 returns the entries
 * set or changed since the last call that fit in `cap`). *n receives the
 * number of entries; *flags bit PE_ELIG_ESCAPED = HasEscaped(). */
#define PE_CLASS_INELIGIBLE 1   /* EvalComputedClassIneligible */
#define PE_CLASS_ELIGIBLE 2     /* EvalComputedClassEligible */
#define PE_ELIG_ESCAPED 1u
typedef struct pe_class_feas {
    uint32_t task_group;      /* PE_NONE: EvalEligibility.job; else the task group name (str id) */
    uint32_t computed_class;  /* Node.ComputedClass (str id, as in pe_node_table.computed_class) */
    uint32_t status;          /* PE_CLASS_INELIGIBLE / PE_CLASS_ELIGIBLE */
} pe_class_feas;
int pe_get_eligibility(pe_stack* s, uint32_t changed_only, pe_class_feas* out, uint32_t cap, uint32_t* n,
                       uint32_t* flags);
/* After the Go chain answered a Select (PE_EUNSUPPORTED): its ctx.Eligibility()
 * entries become the engine's memo, so later Selects filter and decide classes
 * exactly as the chain would (EvalEligibility is shared by the two stacks). */
int pe_put_eligibility(pe_stack* s, const pe_class_feas* in, uint32_t n);
/* The GenericStack iterator state that persists between Selects:
 * StaticIterator.offset (feasible.go:75-117) and the LimitIterator limit
 * (stack.go:81-90; latched to MaxInt32 by task groups with affinities or
 * spreads, stack.go:165-167). Before the shim's fallback GenericStack answers
 * a PE_EUNSUPPORTED Select it takes both from pe_get_cursor; afterwards
 * pe_set_cursor hands the chain's offset and limit back, with the task group
 * it selected for (its SpreadIterator.SetTaskGroup adds the group's spread
 * weights to sumSpreadWeights, spread.go:232-257), or PE_NONE. */
int pe_get_cursor(const pe_stack* s, uint32_t* offset, uint32_t* limit);
/* ---- zero-crossing served Selects --------------------------------------------
 * GenericScheduler.computePlacements (generic_sched.go:552-627) calls Select
 * once per placement, retries a nil one with Preempt=true when preemption is
 * enabled (selectNextOption, :773-792), and the shim commits each option
 * (Plan.AppendAlloc + AppendPreemptedAlloc, :627, :794-816): two or three cgo
 * crossings per placement. After the first plain Select of a task group the
 * engine already holds the records of the group's count loop (DESIGN.md §12,
 * §25): with preemption enabled, a placement that evicts is two records, the
 * plain Select's nil and the Preempt retry's option (flag PE_SPEC_PREEMPT,
 * its PreemptedAllocs in pre_allocs). This view lets the caller answer those
 * Selects and Commits from host memory and cross into C only when it
 * deviates. One view per handle, used from the handle's thread.
 *
 *   Select(tg, opts) with no preferred / penalty nodes, when v->n_rec > 0,
 *     tg == v->tg_index, v->served == v->confirmed, v->served < v->n_rec and
 *     (v->recs[v->served].flags & PE_SPEC_PREEMPT) is set exactly when
 *     opts.Preempt is:
 *       the result is v->recs[v->served], with PreemptedAllocs
 *       v->pre_allocs[v->pre_off[k] .. v->pre_off[k + 1]) for k = v->served
 *       (none when v->pre_off is NULL); then v->served++, and for a nil
 *       result (row < 0, which no Commit follows) also v->confirmed++;
 *   Commit(tg, row) / CommitPreempt(tg, row, list), when v->served ==
 *     v->confirmed + 1, tg == v->tg_index, row == v->recs[v->served - 1].row
 *     and the list is that record's PreemptedAllocs in its order (empty for
 *     Commit): v->confirmed++;
 *   anything else goes through the entry points below, which first take the
 *     counters over, so the engine state is exactly what the sequential calls
 *     would have produced; they may replace or withdraw the records (v->epoch
 *     changes; v->n_rec 0: nothing to serve).
 * A record the engine returned through pe_select may be confirmed through the
 * view as well. With pe_set_metrics on, the runs still publish records, each
 * with its AllocMetric maps. A served record is the leading part of pe_ranked_node (row ..
 * new_offset) plus the device offers; served Selects never reserve cores.
 * Replaces: the Select / Commit crossings of computePlacements' loop. */
#define PE_SPEC_PREEMPT 1u   /* pe_spec_rec.flags: answers the Select with Preempt=true */
typedef struct pe_spec_rec {
    int32_t row;
    uint32_t n_scores;
    double final_score;
    double scores[PE_MAX_SCORES];
    uint32_t nodes_evaluated, nodes_filtered, nodes_exhausted, new_offset;
    uint32_t n_device_offers;
    uint16_t device_offer_group[PE_MAX_DEVICE_REQ];
    uint32_t flags;               /* PE_SPEC_* */
} pe_spec_rec;
typedef struct pe_spec_view {
    uint32_t epoch;               /* engine: changes whenever recs / n_rec / tg_index change */
    uint32_t tg_index;            /* the task group the records answer */
    uint32_t n_rec;               /* records [0, n_rec) are valid */
    uint32_t pad0;
    const pe_spec_rec* recs;      /* the run's records in Select order */
    uint32_t served;              /* caller and engine: Selects answered from recs */
    uint32_t confirmed;           /* caller and engine: records settled (Commits, nils) */
    const uint32_t* pre_off;      /* [n_rec + 1] or NULL: record k's PreemptedAllocs ... */
    const uint32_t* pre_allocs;   /* ... are pre_allocs[pre_off[k] .. pre_off[k + 1]) (alloc-table rows) */
    /* With pe_set_metrics on: record k's AllocMetric maps, what
     * pe_last_metrics_bin returns after that Select, are
     * mcounts[mcounts_off[k] .. mcounts_off[k + 1]) and
     * mscores[mscores_off[k] .. mscores_off[k + 1]); NULL when the records
     * carry none. */
    const pe_metric_count* mcounts;
    const uint32_t* mcounts_off;
    const pe_metric_score* mscores;
    const uint32_t* mscores_off;
} pe_spec_view;
pe_spec_view* pe_spec_view_get(pe_stack* s);
/* SystemScheduler.computePlacements (scheduler_system.go:283-425) runs, for
 * every node, SetNodes([node]) + Select + (on an option) Plan.AppendAlloc:
 * three crossings per node (scheduler_system.go:289-302). From a task group's
 * third single-node Select the engine answers from a per-row cache filled by
 * one k_system pass; this view exposes that cache so the
 * caller answers the triples from host memory and logs them, and crosses into
 * C only when it deviates. One view per handle, used from its thread.
 *
 *   SetNodes([row]) + Select(tg) with no options, when v->n_rows > 0,
 *     tg == v->tg_index, row < v->n_rows, v->n_log < v->log_cap and
 *     outcome[row] is servable: a finite double is an option on `row` with
 *     that FinalScore (one score, nodes_evaluated 1); a NaN whose low two bits
 *     are 1 (filtered) or 2 (exhausted) is nil with nodes_filtered /
 *     nodes_exhausted 1 -- unless v->preempt and it is exhausted (BinPack with
 *     eviction answers: go to C); low bits 3 (PE_SYS_STALE) mean the row
 *     changed since the pass: go to C. Then v->log[v->n_log++] = row, with
 *     PE_SYS_NIL set for a nil answer;
 *   the Commit of that option: v->log[v->n_log - 1] |= PE_SYS_COMMITTED and
 *     outcome[row] = PE_SYS_STALE (a committed row is not served again);
 *   anything else goes through the entry points, which first take the log
 *     over (the engine state is then exactly what the sequential calls would
 *     have produced); they may withdraw the view (v->epoch changes; v->n_rows 0).
 * Replaces: the SetNodes / Select / Commit crossings of the per-node loop. */
#define PE_SYS_NIL (1u << 31)
#define PE_SYS_COMMITTED (1u << 30)
#define PE_SYS_ROW_MASK 0x3FFFFFFFu
#define PE_SYS_STALE 0x7FF8000000000003ull
typedef struct pe_system_view {
    uint32_t epoch;               /* engine: changes whenever outcome / n_rows / tg_index change */
    uint32_t tg_index;            /* the task group the outcomes answer */
    uint32_t n_rows;              /* 0: nothing to serve */
    uint32_t log_cap;             /* entries log[] can hold */
    uint64_t* outcome;            /* [n_rows] per row (bits of a double) */
    uint32_t* log;                /* [log_cap] served Selects in order, written by the caller */
    uint32_t n_log;               /* caller and engine: entries written / taken over */
    uint32_t preempt;             /* nonzero: exhausted rows go to the engine */
    /* With pe_set_metrics on (NULL otherwise): a served Select's AllocMetric
     * maps (scheduler_system.go:334-337), which the caller assembles from
     * per-row entries as FeasibilityWrapper and BinPack would have filled
     * them (feasible.go:1061-1153):
     *   option: ScoreMetaData = [{NodeID of row, NormScore = the outcome's
     *     FinalScore, Scores = {"binpack": mscore[row]}}];
     *   filtered: ConstraintFiltered[key]++ with key = mkey[row], except when
     *     c = mclass[row] != PE_NONE and mfailed[c] is set: key =
     *     mkey_ineligible ("computed class ineligible"); then mfailed[c] = 1
     *     when c != PE_NONE (the EvalEligibility memo of the row's class);
     *   exhausted: DimensionExhausted[mkey[row]]++;
     *   filtered / exhausted: ClassFiltered / ClassExhausted[mnode_class[row]]++
     *     unless it is PE_NONE (a node without NodeClass).
     * Keys as pe_metric_count.key (pe_metric_string). */
    const uint32_t* mkey;
    const uint32_t* mclass;
    uint8_t* mfailed;             /* caller and engine: per memo class */
    const double* mscore;
    const uint32_t* mnode_class;
    uint32_t mkey_ineligible;
    uint32_t pad1;
} pe_system_view;
pe_system_view* pe_system_view_get(pe_stack* s);
int pe_set_cursor(pe_stack* s, uint32_t tg_index, uint32_t offset, uint32_t limit);
/* Host-side constraint semantics used for pre-resolution (checkConstraint,
 * feasible.go:785-820), exposed for known-answer tests; needs no device.
 * l_state / r_state: 0 nil (unknown ${...} target), 1 found, 2 missing ("", false). */
int pe_check_constraint(const char* op, const char* l, int l_state, const char* r, int r_state);

/* ======================================================================== *
 * Plan applier fit check (leader side).
 *
 * Replaces evaluatePlanPlacements' per-node worker calls
 * (nomad/plan_apply.go:439-582) to evaluateNodePlan (plan_apply.go:611-674) →
 * structs.AllocsFit(node, proposed, nil, checkDevices=true)
 * (nomad/structs/funcs.go:148-211), with NetworkIndex.SetNode/AddAllocs
 * (nomad/structs/network.go:92-193, 196-296) and DeviceAccounter
 * (nomad/structs/devices.go:22-101). The planner handle keeps the state
 * snapshot (nodes and their non-terminal allocations) resident in HBM; one
 * kernel evaluates every node of a plan (one wavefront per plan node) and
 * pe_planner_commit folds an applied plan back into the resident snapshot
 * (the optimistic snapshot.UpsertPlanResults of planApply, plan_apply.go:207).
 * Strings: every call carries its own pe_strtab; the planner interns by
 * content, so ids need not be stable across calls.
 * ======================================================================== */

/* evaluateNodePlan outcome per plan node; the reason strings are the
 * reference's (plan_apply.go:627-633, funcs.go:184-208, structs.go:3891-3905). */
#define PE_PLAN_FIT 0
#define PE_PLAN_NODE_MISSING 1      /* "node does not exist" */
#define PE_PLAN_NODE_NOT_READY 2    /* "node is not ready for placements" */
#define PE_PLAN_NODE_INELIGIBLE 3   /* "node is not eligible" */
#define PE_PLAN_CORES 4             /* "cores" (overlap between allocs, or not a subset of the node's) */
#define PE_PLAN_CPU 5               /* "cpu" */
#define PE_PLAN_MEMORY 6            /* "memory" */
#define PE_PLAN_DISK 7              /* "disk" */
#define PE_PLAN_PORTS 8             /* "reserved port collision" */
#define PE_PLAN_BANDWIDTH 9         /* "bandwidth exceeded": never (Overcommitted is disabled, network.go:79-90) */
#define PE_PLAN_DEVICES 10          /* "device oversubscribed" */

/* Nodes of the snapshot, the fields evaluateNodePlan / AllocsFit read. */
typedef struct pe_plan_node_table {
    uint32_t n;
    const uint8_t* ready;            /* Node.Status == "ready" */
    const uint8_t* eligible;         /* Node.SchedulingEligibility != "ineligible" */
    const int64_t* cpu_shares;       /* NodeResources.Cpu.CpuShares */
    const int64_t* memory_mb;
    const int64_t* disk_mb;
    const int64_t* reserved_cpu;     /* ReservedResources (0 when nil) */
    const int64_t* reserved_memory_mb;
    const int64_t* reserved_disk_mb;
    /* NodeResources.Cpu.ReservableCpuCores minus ReservedResources.Cpu.ReservedCpuCores */
    const uint32_t* core_off; const uint32_t* core_id;
    /* NodeResources.Networks entries with Device != "": their IP (str id) */
    const uint32_t* net_off; const uint32_t* net_ip;
    /* NodeResources.NodeNetworks[*].Addresses[*]: Address and ReservedPorts spec (str ids) */
    const uint32_t* addr_off; const uint32_t* addr_ip; const uint32_t* addr_reserved_ports;
    /* ReservedResources.Networks.ReservedHostPorts spec (str id; "" when unset) */
    const uint32_t* reserved_host_ports;
    /* NodeResources.Devices: groups (vendor, type, name) and their instances */
    const uint32_t* dev_off; const uint32_t* dev_vendor; const uint32_t* dev_type; const uint32_t* dev_name;
    const uint32_t* inst_off;        /* CSR over device groups */
    const uint32_t* inst_id; const uint8_t* inst_healthy;
} pe_plan_node_table;

/* Allocations: the snapshot's (node_row set) or a plan's (node_row ignored).
 * Resources are Allocation.ComparableResources() (structs.go:9656-9688). */
typedef struct pe_plan_alloc_table {
    uint32_t count;
    const uint32_t* node_row;
    const uint8_t* terminal;         /* Allocation.TerminalStatus() */
    const int64_t* cpu_shares;
    const int64_t* memory_mb;
    const int64_t* disk_mb;
    /* Flattened.Cpu.ReservedCores (a set per alloc) */
    const uint32_t* core_off; const uint32_t* core_id;
    /* the ports NetworkIndex.AddAllocs marks (network.go:144-193): the
       AllocatedResources.Shared.Ports (HostIP, Value) when non-empty, else the
       Reserved+Dynamic ports of Shared.Networks and of each task's first network (IP) */
    const uint32_t* port_off; const uint32_t* port_ip; const int64_t* port_value;
    /* one entry per AllocatedDeviceResource.DeviceIDs element of every task */
    const uint32_t* dev_off;
    const uint32_t* dev_vendor; const uint32_t* dev_type; const uint32_t* dev_name; const uint32_t* dev_instance;
} pe_plan_alloc_table;

/* One plan (structs.Plan) as evaluatePlanPlacements sees it, node by node. */
typedef struct pe_plan {
    uint32_t n_nodes;                /* nodeIDList: NodeUpdate keys then NodeAllocation keys */
    const uint32_t* node_row;        /* snapshot row, or PE_NONE when the node does not exist */
    /* snapshot allocs RemoveAllocs drops on that node: NodeUpdate ∪ NodePreemptions ∪
       NodeAllocation IDs (plan_apply.go:650-665), as indices into the snapshot alloc table */
    const uint32_t* remove_off; const uint32_t* remove_alloc;
    /* NodeAllocation[node]: CSR into `allocs` */
    const uint32_t* place_off;
    pe_plan_alloc_table allocs;
} pe_plan;

typedef struct pe_planner pe_planner;
pe_planner* pe_planner_create(int device);
void pe_planner_destroy(pe_planner* p);
const char* pe_planner_last_error(const pe_planner* p);
/* Upload the state snapshot: nodes and allocations (terminal ones are kept
 * as rows but never counted). Replaces any earlier snapshot. */
int pe_planner_set_state(pe_planner* p, const pe_strtab* strs, const pe_plan_node_table* nodes,
                         const pe_plan_alloc_table* allocs);
/* evaluateNodePlan for every plan node on the device: reason[i] = PE_PLAN_*.
 * *n_fit = nodes that fit. The AllAtOnce / partial-commit bookkeeping of
 * evaluatePlanPlacements stays with the caller (it needs only reason[]). */
int pe_planner_evaluate(pe_planner* p, const pe_strtab* strs, const pe_plan* plan, uint8_t* reason,
                        uint32_t* n_fit);
/* Apply the nodes whose reason is PE_PLAN_FIT to the resident snapshot:
 * removed allocs stop counting, placed allocs are appended (ApplyPlanResults).
 * `keep[i]` != 0 selects plan node i (the caller passes the result it applied). */
int pe_planner_commit(pe_planner* p, const pe_strtab* strs, const pe_plan* plan, const uint8_t* keep);
/* Device time of the last evaluate (HIP events around the kernel) and its
 * algorithmic bytes (records and keys read + reasons written), computed when
 * asked against the current snapshot: ask before pe_planner_commit. */
double pe_planner_kernel_ms(const pe_planner* p);
uint64_t pe_planner_last_bytes(const pe_planner* p);
uint32_t pe_planner_snapshot_allocs(const pe_planner* p);

#ifdef __cplusplus
}
#endif
#endif /* NOMAD_PE_H */
