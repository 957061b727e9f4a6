#!/bin/bash
# Counters of the C5 count loop kernel (k_ploop, one 256-lane workgroup): what
# makes its per-placement evaluations cold. Separate rocprofv3 --pmc passes
# over tools/c5_prof.py (pe_place of the C5 evaluation, twice), each within
# the per-block slot limits (SQ 8, TCP 4, TCC 4), then a per-placement summary
# by tools/pmc_summary.py. Outputs in gpurun_out/ploop_pmc/.
set -eo pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/ploop_pmc
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
P1="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_DCACHE_HITS SQC_DCACHE_MISSES"
P2="SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY"
P3="SQ_IFETCH SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES"
P4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum"
P5="TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"
P6="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum"
P7="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum TCP_TOTAL_READ_sum TCP_TOTAL_WRITE_sum"
P8="TA_FLAT_READ_WAVEFRONTS_sum TA_FLAT_READ_LDS_WAVEFRONTS_sum"
PASSES=${PLOOP_PASSES:-"1 2 3 4 5 6 7 8"}
i=0
for k in $PASSES; do
  eval P=\$P$k
  i=$k
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o p$i -- \
    python3 "$ROOT/tools/c5_prof.py" > "$OUT/p$i.log" 2>&1
done
cd "$ROOT"
python3 tools/pmc_summary.py k_ploop 1000 "$OUT"/p*/ > "$OUT/ploop_counters.json"
cat "$OUT/ploop_counters.json"
