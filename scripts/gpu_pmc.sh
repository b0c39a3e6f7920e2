#!/bin/bash
# PMC passes over scripts/prof_run.py (each pass its own run; counters only, no tracing).
# usage: [WG_WORKLOAD=ragged] gpu_pmc.sh <tag> [full]  -> gpurun_out/<tag>N/, then scripts/pmc_summary.py <tag>
# (traffic passes only unless "full" is given; "valu" = the instruction-issue pass only)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-pmc}
if [ ! -s gpurun_out/counters_avail.txt ]; then
  timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_avail.txt 2>&1 || echo "counter listing failed"
fi
i=0
sets=("FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE SQ_WAVES")
if [ "$2" = "valu" ]; then sets=("SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" "GRBM_GUI_ACTIVE SQ_WAVES"); fi
if [ "$2" = "full" ]; then sets+=(\
            "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT" \
            "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS" \
            "SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32" \
            "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INST_LEVEL_VMEM"); fi
for ctrs in "${sets[@]}"; do
  i=$((i+1))
  echo "== pass $i: $ctrs"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${tag}$i -o pmc -- python scripts/prof_run.py > gpurun_out/${tag}$i.log 2>&1 || { echo "pass $i failed rc=$?"; tail -5 gpurun_out/${tag}$i.log; exit 1; }
done
python scripts/pmc_summary.py $tag
echo done
