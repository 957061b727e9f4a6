"""ctypes mirror of include/nomad_pe.h (the engine's C ABI).

Kept field-for-field identical to the header; tests/test_abi.py checks the
sizes against offsets the library reports, and that every declared symbol is
exported by nomad_amd/libnomadpe.so.
"""
import ctypes as C

u8p = C.POINTER(C.c_uint8)
# pe_exchange_fn (pe_comm_init_host): all-gather of one record per rank
pe_exchange_fn = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
u32p = C.POINTER(C.c_uint32)
u16p = C.POINTER(C.c_uint16)
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
f64p = C.POINTER(C.c_double)

PE_NONE = 0xFFFFFFFF
PE_MAX_SCORES = 8
PE_MAX_PREEMPT = 16
PE_MAX_DEVICE_REQ = 4
PE_OK, PE_EINVAL, PE_ESTATE, PE_EHIP, PE_EUNSUPPORTED, PE_ENOMEM, PE_EINTERNAL = 0, -1, -2, -3, -4, -5, -6

PE_ATTR_INT, PE_ATTR_FLOAT, PE_ATTR_STRING, PE_ATTR_BOOL = 1, 2, 3, 4
PE_LC_MAIN, PE_LC_PRESTART, PE_LC_PRESTART_SIDECAR, PE_LC_POSTSTOP, PE_LC_POSTSTART = 0, 1, 2, 3, 4
PE_JOB_SERVICE, PE_JOB_BATCH, PE_JOB_SYSTEM, PE_JOB_SYSBATCH = 0, 1, 2, 3
PE_STACK_GENERIC, PE_STACK_SYSTEM = 0, 1
PE_ALGO_BINPACK, PE_ALGO_SPREAD = 0, 1


class pe_strtab(C.Structure):
    _fields_ = [("bytes", C.c_char_p), ("offsets", u32p), ("count", C.c_uint32)]


class pe_attr(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("unit", C.c_uint32), ("i", C.c_int64), ("f", C.c_double),
                ("s", C.c_uint32), ("_pad", C.c_uint32)]


class pe_node_table(C.Structure):
    _fields_ = [
        ("n", C.c_uint32),
        ("id", u32p), ("name", u32p), ("datacenter", u32p), ("node_class", u32p),
        ("computed_class", u32p),
        ("cpu_shares", i64p), ("memory_mb", i64p), ("disk_mb", i64p),
        ("reserved_cpu", i64p), ("reserved_memory_mb", i64p), ("reserved_disk_mb", i64p),
        ("attr_off", u32p), ("attr_key", u32p), ("attr_val", u32p),
        ("meta_off", u32p), ("meta_key", u32p), ("meta_val", u32p),
        ("drv_off", u32p), ("drv_name", u32p), ("drv_flags", u8p),
        ("net_off", u32p), ("net_mode", u32p), ("net_device", u32p), ("net_mbits", i32p),
        ("alias_off", u32p), ("alias_name", u32p),
        ("reserved_dyn_ports", i32p),
        ("hv_off", u32p), ("hv_name", u32p), ("hv_read_only", u8p),
        ("dev_off", u32p), ("dev_vendor", u32p), ("dev_type", u32p), ("dev_name", u32p),
        ("dev_healthy", u32p),
        ("dev_attr_off", u32p), ("dev_attr_key", u32p), ("dev_attr_val", C.POINTER(pe_attr)),
        ("core_off", u32p), ("core_id", u16p), ("total_cores", u32p),
        ("rsv_core_off", u32p), ("rsv_core_id", u16p),
        ("addr_off", u32p), ("addr_alias", u32p), ("addr_ip", u32p), ("addr_rsv_ports", u32p),
        ("rsv_host_ports", u32p),
        ("net_ip", u32p), ("net_cidr_ip", u32p),
    ]


class pe_alloc_table(C.Structure):
    _fields_ = [
        ("count", C.c_uint32),
        ("node_row", u32p), ("ns", u32p), ("job_id", u32p), ("task_group", u32p),
        ("terminal", u8p), ("priority", i32p),
        ("cpu_shares", i64p), ("memory_mb", i64p), ("disk_mb", i64p),
        ("net_mbits", i32p), ("dyn_ports", i32p),
        ("dev_off", u32p), ("dev_group", u32p), ("dev_count", u32p),
        ("max_parallel", i32p),
        ("core_off", u32p), ("core_id", u16p),
        ("port_off", u32p), ("port_ip", u32p), ("port_value", i32p),
        ("has_network", u8p),
        ("net_device", u32p),
    ]


class pe_constraint(C.Structure):
    _fields_ = [("ltarget", C.c_uint32), ("rtarget", C.c_uint32), ("operand", C.c_uint32)]


class pe_affinity(C.Structure):
    _fields_ = [("ltarget", C.c_uint32), ("rtarget", C.c_uint32), ("operand", C.c_uint32),
                ("weight", C.c_int32)]


class pe_spread_target(C.Structure):
    _fields_ = [("value", C.c_uint32), ("percent", C.c_int32)]


class pe_spread(C.Structure):
    _fields_ = [("attribute", C.c_uint32), ("weight", C.c_int32),
                ("target_off", C.c_uint32), ("target_count", C.c_uint32)]


class pe_device_request(C.Structure):
    _fields_ = [("name", C.c_uint32), ("_pad", C.c_uint32), ("count", C.c_uint64),
                ("constraint_off", C.c_uint32), ("constraint_count", C.c_uint32),
                ("affinity_off", C.c_uint32), ("affinity_count", C.c_uint32)]


class pe_task(C.Structure):
    _fields_ = [
        ("name", C.c_uint32), ("driver", C.c_uint32),
        ("cpu", C.c_int64), ("memory_mb", C.c_int64), ("memory_max_mb", C.c_int64),
        ("cores", C.c_int32), ("lifecycle", C.c_uint32),
        ("has_network", C.c_int32), ("net_mbits", C.c_int32), ("net_dyn_ports", C.c_int32),
        ("net_reserved_ports", C.c_int32),
        ("constraint_off", C.c_uint32), ("constraint_count", C.c_uint32),
        ("affinity_off", C.c_uint32), ("affinity_count", C.c_uint32),
        ("device_off", C.c_uint32), ("device_count", C.c_uint32),
        ("rport_off", C.c_uint32),
    ]


class pe_task_group(C.Structure):
    _fields_ = [
        ("name", C.c_uint32), ("count", C.c_int32),
        ("ephemeral_disk_mb", C.c_int64),
        ("constraint_off", C.c_uint32), ("constraint_count", C.c_uint32),
        ("affinity_off", C.c_uint32), ("affinity_count", C.c_uint32),
        ("spread_off", C.c_uint32), ("spread_count", C.c_uint32),
        ("task_off", C.c_uint32), ("task_count", C.c_uint32),
        ("has_network", C.c_int32), ("net_mode", C.c_uint32),
        ("net_dyn_ports", C.c_int32), ("net_reserved_ports", C.c_int32),
        ("net_host_network", C.c_uint32),
        ("volume_off", C.c_uint32), ("volume_count", C.c_uint32),
        ("has_csi_volumes", C.c_int32),
        ("rport_off", C.c_uint32), ("rport_count", C.c_uint32),
    ]


class pe_job(C.Structure):
    _fields_ = [
        ("id", C.c_uint32), ("ns", C.c_uint32), ("type", C.c_uint32), ("priority", C.c_int32),
        ("version", C.c_uint64),
        ("constraint_off", C.c_uint32), ("constraint_count", C.c_uint32),
        ("affinity_off", C.c_uint32), ("affinity_count", C.c_uint32),
        ("spread_off", C.c_uint32), ("spread_count", C.c_uint32),
        ("tg_count", C.c_uint32),
        ("task_groups", C.POINTER(pe_task_group)),
        ("tasks", C.POINTER(pe_task)),
        ("constraints", C.POINTER(pe_constraint)),
        ("affinities", C.POINTER(pe_affinity)),
        ("spreads", C.POINTER(pe_spread)),
        ("spread_targets", C.POINTER(pe_spread_target)),
        ("devices", C.POINTER(pe_device_request)),
        ("device_constraints", C.POINTER(pe_constraint)),
        ("device_affinities", C.POINTER(pe_affinity)),
        ("volume_source", u32p),
        ("volume_read_only", u8p),
        ("rport_value", i32p),
        ("rport_label", u32p),
    ]


class pe_config(C.Structure):
    _fields_ = [("stack_kind", C.c_uint32), ("batch", C.c_uint32), ("algorithm", C.c_uint32),
                ("memory_oversubscription", C.c_uint32), ("preempt", C.c_uint32),
                ("device", C.c_int32), ("device_count", C.c_uint32), ("device_ids", C.c_int32 * 8)]


class pe_select_options(C.Structure):
    _fields_ = [("penalty_rows", u32p), ("penalty_count", C.c_uint32),
                ("preferred_rows", u32p), ("preferred_count", C.c_uint32),
                ("preempt", C.c_uint32)]


class pe_ranked_node(C.Structure):
    _fields_ = [("row", C.c_int32), ("n_scores", C.c_uint32), ("final_score", C.c_double),
                ("scores", C.c_double * PE_MAX_SCORES),
                ("nodes_evaluated", C.c_uint32), ("nodes_filtered", C.c_uint32),
                ("nodes_exhausted", C.c_uint32), ("new_offset", C.c_uint32),
                ("n_preempted", C.c_uint32), ("preempted", C.c_uint32 * PE_MAX_PREEMPT),
                ("n_device_offers", C.c_uint32), ("device_offer_group", C.c_uint32 * PE_MAX_DEVICE_REQ),
                ("reserved_cores", C.c_uint64 * 4)]


class pe_shard_rec(C.Structure):
    _fields_ = [("bytes", C.c_uint8 * 80)]


class pe_placement(C.Structure):
    _fields_ = [("row", C.c_int32), ("nodes_evaluated", C.c_uint32), ("final_score", C.c_double)]


PE_CLASS_INELIGIBLE, PE_CLASS_ELIGIBLE = 1, 2
PE_ELIG_ESCAPED = 1


class pe_class_feas(C.Structure):
    _fields_ = [("task_group", C.c_uint32), ("computed_class", C.c_uint32), ("status", C.c_uint32)]


# Entry points declared in include/nomad_pe.h: (name, restype, argtypes)
def _sigs(prefix, handle):
    H = C.c_void_p
    return [
        (prefix + "set_state", C.c_int, [H, C.POINTER(pe_strtab), C.POINTER(pe_node_table),
                                         C.POINTER(pe_alloc_table)]),
        (prefix + "set_job", C.c_int, [H, C.POINTER(pe_strtab), C.POINTER(pe_job)]),
        (prefix + "reset_plan", C.c_int, [H]),
        (prefix + "set_nodes", C.c_int, [H, u32p, C.c_uint32, u32p]),
        (prefix + "select", C.c_int, [H, C.c_uint32, C.POINTER(pe_select_options),
                                      C.POINTER(pe_ranked_node)]),
        (prefix + "commit", C.c_int, [H, C.c_uint32, C.c_int32]),
        (prefix + "commit_preempt", C.c_int, [H, C.c_uint32, C.c_int32, u32p, C.c_uint32]),
        (prefix + "preempted_of", C.c_int, [H, C.c_uint32, u32p, C.c_uint32]),
        (prefix + "plan_stop", C.c_int, [H, u32p, C.c_uint32]),
        (prefix + "plan_pop_update", C.c_int, [H, C.c_uint32]),
        (prefix + "place", C.c_int, [H, C.c_uint32, C.c_uint32, C.POINTER(pe_ranked_node), u32p]),
        (prefix + "system_place", C.c_int, [H, C.c_uint32, f64p, u8p, u32p]),
        (prefix + "get_eligibility", C.c_int, [H, C.c_uint32, C.POINTER(pe_class_feas), C.c_uint32, u32p, u32p]),
        (prefix + "put_eligibility", C.c_int, [H, C.POINTER(pe_class_feas), C.c_uint32]),
        (prefix + "get_cursor", C.c_int, [H, u32p, u32p]),
        (prefix + "set_cursor", C.c_int, [H, C.c_uint32, C.c_uint32, C.c_uint32]),
    ]


ENGINE_SYMBOLS = [
    "pe_abi_version", "pe_stack_create", "pe_stack_destroy", "pe_last_error", "pe_set_state",
    "pe_reset_plan", "pe_set_job", "pe_set_nodes", "pe_select", "pe_commit", "pe_commit_preempt", "pe_place", "pe_system_place",
    "pe_last_kernel_ms", "pe_stage_orders", "pe_place_batch", "pe_batch_results", "pe_last_phase_ms",
    "pe_check_constraint", "pe_last_sweep_bytes", "pe_select_shard", "pe_select_merge",
    "pe_set_metrics", "pe_last_metrics", "pe_update_allocs", "pe_speculation_stats",
    "pe_plan_stop", "pe_plan_pop_update", "pe_update_nodes", "pe_comm_unique_id", "pe_comm_init", "pe_comm_init_host",
    "pe_place_sharded", "pe_last_exchange_us", "pe_get_eligibility", "pe_put_eligibility", "pe_get_cursor",
    "pe_set_cursor", "pe_flush", "pe_system_spec_stats", "pe_device_count", "pe_set_kernel_split",
    "pe_last_kernel_split", "pe_preempted_of", "pe_spec_view_get", "pe_system_view_get", "pe_comm_library", "pe_last_exchange_stats",
    "pe_last_metrics_bin", "pe_metric_string", "pe_scorer_name", "pe_system_results",
]


class pe_spec_rec(C.Structure):   # nomad_pe.h: a served-Select record
    _fields_ = [("row", C.c_int32), ("n_scores", C.c_uint32), ("final_score", C.c_double),
                ("scores", C.c_double * PE_MAX_SCORES), ("nodes_evaluated", C.c_uint32),
                ("nodes_filtered", C.c_uint32), ("nodes_exhausted", C.c_uint32), ("new_offset", C.c_uint32),
                ("n_device_offers", C.c_uint32), ("device_offer_group", C.c_uint16 * PE_MAX_DEVICE_REQ),
                ("flags", C.c_uint32)]


PE_SPEC_PREEMPT = 1   # pe_spec_rec.flags: answers the Select with Preempt=true


PE_METRIC_CLASS_FILTERED, PE_METRIC_CONSTRAINT_FILTERED, PE_METRIC_CLASS_EXHAUSTED, PE_METRIC_DIMENSION_EXHAUSTED = 1, 2, 3, 4
PE_METRIC_ENGINE_KEY = 0x80000000
SCORER_NAMES = ("binpack", "devices", "job-anti-affinity", "node-reschedule-penalty", "node-affinity",
                "allocation-spread", "preemption")


class pe_metric_count(C.Structure):   # nomad_pe.h: one AllocMetric map entry
    _fields_ = [("kind", C.c_uint32), ("key", C.c_uint32), ("count", C.c_uint32)]


class pe_metric_score(C.Structure):   # nomad_pe.h: one NodeScoreMeta
    _fields_ = [("row", C.c_int32), ("n_scores", C.c_uint32), ("norm", C.c_double),
                ("scorer", C.c_uint8 * PE_MAX_SCORES), ("score", C.c_double * PE_MAX_SCORES)]


class pe_spec_view(C.Structure):
    _fields_ = [("epoch", C.c_uint32), ("tg_index", C.c_uint32), ("n_rec", C.c_uint32), ("pad0", C.c_uint32),
                ("recs", C.POINTER(pe_spec_rec)), ("served", C.c_uint32), ("confirmed", C.c_uint32),
                ("pre_off", C.POINTER(C.c_uint32)), ("pre_allocs", C.POINTER(C.c_uint32)),
                ("mcounts", C.POINTER(pe_metric_count)), ("mcounts_off", C.POINTER(C.c_uint32)),
                ("mscores", C.POINTER(pe_metric_score)), ("mscores_off", C.POINTER(C.c_uint32))]


PE_SYS_NIL = 1 << 31
PE_SYS_COMMITTED = 1 << 30
PE_SYS_ROW_MASK = 0x3FFFFFFF
PE_SYS_STALE = 0x7FF8000000000003


class pe_system_view(C.Structure):   # nomad_pe.h: the served system-Select view
    _fields_ = [("epoch", C.c_uint32), ("tg_index", C.c_uint32), ("n_rows", C.c_uint32), ("log_cap", C.c_uint32),
                ("outcome", C.POINTER(C.c_uint64)), ("log", C.POINTER(C.c_uint32)), ("n_log", C.c_uint32),
                ("preempt", C.c_uint32), ("mkey", C.POINTER(C.c_uint32)), ("mclass", C.POINTER(C.c_uint32)),
                ("mfailed", C.POINTER(C.c_uint8)), ("mscore", C.POINTER(C.c_double)),
                ("mnode_class", C.POINTER(C.c_uint32)), ("mkey_ineligible", C.c_uint32), ("pad1", C.c_uint32)]


def bind(lib, prefix, create_name, destroy_name, error_name):
    """Attach restype/argtypes for the stack API on a loaded CDLL."""
    for name, res, args in _sigs(prefix, None):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    getattr(lib, create_name).restype = C.c_void_p
    getattr(lib, create_name).argtypes = [C.POINTER(pe_config)]
    getattr(lib, destroy_name).restype = None
    getattr(lib, destroy_name).argtypes = [C.c_void_p]
    getattr(lib, error_name).restype = C.c_char_p
    getattr(lib, error_name).argtypes = [C.c_void_p]
    return lib


# ---- plan applier (pe_planner_*) ----------------------------------------------
PE_PLAN_FIT, PE_PLAN_NODE_MISSING, PE_PLAN_NODE_NOT_READY, PE_PLAN_NODE_INELIGIBLE = 0, 1, 2, 3
PE_PLAN_CORES, PE_PLAN_CPU, PE_PLAN_MEMORY, PE_PLAN_DISK = 4, 5, 6, 7
PE_PLAN_PORTS, PE_PLAN_BANDWIDTH, PE_PLAN_DEVICES = 8, 9, 10
# reason strings of evaluateNodePlan / AllocsFit (plan_apply.go:627-633, funcs.go:184-208)
PLAN_REASONS = ["", "node does not exist", "node is not ready for placements", "node is not eligible",
                "cores", "cpu", "memory", "disk", "reserved port collision", "bandwidth exceeded",
                "device oversubscribed"]


class pe_plan_node_table(C.Structure):
    _fields_ = [
        ("n", C.c_uint32), ("ready", u8p), ("eligible", u8p),
        ("cpu_shares", i64p), ("memory_mb", i64p), ("disk_mb", i64p),
        ("reserved_cpu", i64p), ("reserved_memory_mb", i64p), ("reserved_disk_mb", i64p),
        ("core_off", u32p), ("core_id", u32p),
        ("net_off", u32p), ("net_ip", u32p),
        ("addr_off", u32p), ("addr_ip", u32p), ("addr_reserved_ports", u32p),
        ("reserved_host_ports", u32p),
        ("dev_off", u32p), ("dev_vendor", u32p), ("dev_type", u32p), ("dev_name", u32p),
        ("inst_off", u32p), ("inst_id", u32p), ("inst_healthy", u8p),
    ]


class pe_plan_alloc_table(C.Structure):
    _fields_ = [
        ("count", C.c_uint32), ("node_row", u32p), ("terminal", u8p),
        ("cpu_shares", i64p), ("memory_mb", i64p), ("disk_mb", i64p),
        ("core_off", u32p), ("core_id", u32p),
        ("port_off", u32p), ("port_ip", u32p), ("port_value", i64p),
        ("dev_off", u32p), ("dev_vendor", u32p), ("dev_type", u32p), ("dev_name", u32p),
        ("dev_instance", u32p),
    ]


class pe_plan(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32), ("node_row", u32p),
        ("remove_off", u32p), ("remove_alloc", u32p),
        ("place_off", u32p), ("allocs", pe_plan_alloc_table),
    ]


PLANNER_SYMBOLS = [
    "pe_planner_create", "pe_planner_destroy", "pe_planner_last_error", "pe_planner_set_state",
    "pe_planner_evaluate", "pe_planner_commit", "pe_planner_kernel_ms", "pe_planner_last_bytes",
    "pe_planner_snapshot_allocs",
]


def bind_planner(lib):
    """Attach restype/argtypes for the pe_planner_* API on a loaded CDLL."""
    H = C.c_void_p
    sigs = [
        ("pe_planner_create", C.c_void_p, [C.c_int]),
        ("pe_planner_destroy", None, [H]),
        ("pe_planner_last_error", C.c_char_p, [H]),
        ("pe_planner_set_state", C.c_int, [H, C.POINTER(pe_strtab), C.POINTER(pe_plan_node_table),
                                           C.POINTER(pe_plan_alloc_table)]),
        ("pe_planner_evaluate", C.c_int, [H, C.POINTER(pe_strtab), C.POINTER(pe_plan), u8p, u32p]),
        ("pe_planner_commit", C.c_int, [H, C.POINTER(pe_strtab), C.POINTER(pe_plan), u8p]),
        ("pe_planner_kernel_ms", C.c_double, [H]),
        ("pe_planner_last_bytes", C.c_uint64, [H]),
        ("pe_planner_snapshot_allocs", C.c_uint32, [H]),
    ]
    for name, res, args in sigs:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib
