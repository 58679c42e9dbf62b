#!/bin/bash
# PMC passes for bench.py (one counter group per rocprofv3 run; no trace
# domains combined with --pmc).  Output: gpurun_out/pmc_<R>/<pass>/...
# PASSES selects passes (default: all).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=${ROUND:-r02}
ARGS=${BENCH_ARGS:---steps 6 --warmup 1 --verify-frames 0 --pcie-steps 0 --stats-steps 0}
OUT=gpurun_out/pmc_$R
mkdir -p $OUT
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 240 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o pmc -- python3 bench.py $ARGS > $OUT/$name.json 2> $OUT/$name.err
}
rc=0
for p in ${PASSES:-fetch write sq sq2 tcc valu}; do
  case $p in
    fetch) run fetch FETCH_SIZE ;;
    write) run write WRITE_SIZE ;;
    sq) run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY ;;
    sq2) run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE SQ_BUSY_CYCLES ;;
    tcc) run tcc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum ;;
    valu) run valu SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE ;;
    lds) run lds SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE ;;
  esac
  rc=$?
  [ $rc -ne 0 ] && break
done
python3 tools/pmc_summarize.py $OUT > $OUT/summary.json; cat $OUT/summary.json
exit $rc
