#!/bin/bash
# Dynamic instruction mix of the step kernel per compile-time variant (profiling aid, not product): for every
# ab_session/lib_<v>.so (scripts/variant_ab.py build ...), two rocprofv3 --pmc passes over scripts/prof_run.py (one
# full-batch launch per step), each pass its own run; per-dispatch averages -> gpurun_out/<tag>_<v>_summary.json.
# usage: [WG_WORKLOAD=canonical] gpu_pmc_mix.sh <tag> [variant ...]   (default: every library in ab_session/)
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-mix}; shift
vs=("$@")
if [ ${#vs[@]} -eq 0 ]; then for f in ab_session/lib_*.so; do v=${f#ab_session/lib_}; vs+=("${v%.so}"); done; fi
sets=("SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_ACTIVE_INST_VALU" \
      "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES")
for v in "${vs[@]}"; do
  i=0
  for ctrs in "${sets[@]}"; do
    i=$((i+1))
    echo "== $v pass $i"
    WALKER_HIP_LIB=ab_session/lib_$v.so timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/${tag}_${v}$i -o pmc -- python scripts/prof_run.py > gpurun_out/${tag}_${v}$i.log 2>&1 || { echo "$v pass $i failed rc=$?"; tail -5 gpurun_out/${tag}_${v}$i.log; exit 1; }
  done
  python scripts/pmc_summary.py ${tag}_${v} > /dev/null || exit 1
done
echo done
