/* ORACLE — test infrastructure only. Never linked or loaded by the product
 * (nomad_amd/libnomadpe.so); only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it.
 *
 * C restatement of the reference placement stack (lazy iterator chain) over
 * the same POD inputs as include/nomad_pe.h. Entry points mirror pe_*. */
#ifndef NOMAD_ORACLE_H
#define NOMAD_ORACLE_H
#include "../include/nomad_pe.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_stack oracle_stack;

oracle_stack* oracle_create(const pe_config* cfg);
void oracle_destroy(oracle_stack* s);
const char* oracle_last_error(const oracle_stack* s);
int oracle_set_state(oracle_stack* s, const pe_strtab* strs, const pe_node_table* nodes,
                     const pe_alloc_table* allocs);
int oracle_reset_plan(oracle_stack* s);
int oracle_set_job(oracle_stack* s, const pe_strtab* strs, const pe_job* job);
int oracle_set_nodes(oracle_stack* s, const uint32_t* rows, uint32_t n, uint32_t* limit_out);
int oracle_select(oracle_stack* s, uint32_t tg_index, const pe_select_options* opts,
                  pe_ranked_node* out);
int oracle_commit(oracle_stack* s, uint32_t tg_index, int32_t row);
int oracle_commit_preempt(oracle_stack* s, uint32_t tg_index, int32_t row, const uint32_t* preempted,
                          uint32_t n_preempted);
int oracle_preempted_of(const oracle_stack* s, uint32_t record, uint32_t* out, uint32_t cap);
int oracle_plan_stop(oracle_stack* s, const uint32_t* allocs, uint32_t n);
int oracle_plan_pop_update(oracle_stack* s, uint32_t alloc);
int oracle_place(oracle_stack* s, uint32_t tg_index, uint32_t count, pe_ranked_node* out,
                 uint32_t* placed);
int oracle_system_place(oracle_stack* s, uint32_t tg_index, double* out_score,
                        uint8_t* out_status, uint32_t* placed);

/* One Select with each visited row's outcome traced (0 option + FinalScore,
 * 1 filtered, 2 exhausted, 255 not visited): test hook of the sharded
 * full-pass protocol. */
int oracle_full_pass(oracle_stack* s, uint32_t tg_index, uint8_t* status_by_row, double* score_by_row,
                     pe_ranked_node* out);

/* Known-answer-test helpers (scalar restatements). */
double oracle_go_pow(double x, double y);
double oracle_go_exp(double x);
double oracle_go_log(double x);
/* funcs.go:237-279: algo 0 binpack / 1 spread; returns the raw fit score in [0,18] */
double oracle_score_fit(int algo, int64_t cpu, int64_t mem, int64_t reserved_cpu,
                        int64_t reserved_mem, int64_t used_cpu, int64_t used_mem);
/* feasible.go:785: l_state/r_state: 0 = nil (unknown target), 1 = found, 2 = ("", false) */
int oracle_check_constraint(const char* op, const char* l, int l_state, const char* r, int r_state);
/* select.go: LimitIterator(limit, threshold, maxSkip) + MaxScoreIterator over a
 * StaticRankIterator of `n` FinalScores. Writes the emitted order (indices) to
 * out_order (capacity n), returns the count; *winner = MaxScore pick (-1 none);
 * *pulled = options pulled from the source. */
int oracle_limit_iter(const double* scores, int n, int limit, double threshold, int max_skip,
                      int* out_order, int* winner, int* pulled);

/* Plan applier fit check (plan_oracle.cpp): pe_planner_* on the CPU. */
typedef struct oracle_planner oracle_planner;
oracle_planner* oracle_planner_create(void);
void oracle_planner_destroy(oracle_planner* p);
int oracle_planner_set_state(oracle_planner* p, const pe_strtab* strs, const pe_plan_node_table* nodes,
                             const pe_plan_alloc_table* allocs);
int oracle_planner_evaluate(oracle_planner* p, const pe_strtab* strs, const pe_plan* plan, uint8_t* reason,
                            uint32_t* n_fit);
int oracle_planner_commit(oracle_planner* p, const pe_strtab* strs, const pe_plan* plan, const uint8_t* keep);

#ifdef __cplusplus
}
#endif
#endif
