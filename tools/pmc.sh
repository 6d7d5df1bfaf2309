#!/bin/bash
# Hardware-counter passes over one frame of a config (one rocprofv3 process per pass; --pmc
# only ever with --kernel-trace, per the pool's rules), then the per-launch summary keyed
# by the code object's hash: profiles/pmc/<config>_<hash>.json (read back by bench.py).
# usage (on the GPU box): CONFIG=C4 bash tools/pmc.sh
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
CONFIG=${CONFIG:-C4}
O=$R/gpurun_out/pmc_$CONFIG
rm -rf $O; mkdir -p $O
ARGS="--config $CONFIG --steps 1 --warmup 0 --no-cpu ${BENCH_ARGS}"
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
    "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
    "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VALU2 SQ_INSTS_BRANCH SQ_INSTS_VSKIPPED SQ_INSTS_VMEM SQ_INSTS_FLAT" \
    "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 $R/bench.py $ARGS > $O/pmc_$i.log 2>&1 || { echo "pass $i ($set) failed"; tail -3 $O/pmc_$i.log; exit 1; }
  echo "pass $i ok: $set"
done
# (PMC_TAG: the summary's name for an overridden size, e.g. final_scene_w1440_s64, bench.py)
python3 $R/tools/pmc_summary.py $O $R/gpurun_out/pmc_out --config ${PMC_TAG:-$CONFIG} --round ${ROUND:-5}
