#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, per MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE in separate passes) over one broadcast of a workload.
#   [MSGS=512] bash tools/pmc_passes.sh c4 gpurun_out/pmc_c4 ["GROUP1" "GROUP2" ...]
set -e
WL=${1:-c4}
OUT=${2:-gpurun_out/pmc_$WL}
shift 2 || true
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
if [ $# -gt 0 ]; then GROUPS_=("$@"); else
GROUPS_=("FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ TCC_EA0_WRREQ"
         "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT"
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
         "TCC_HIT TCC_MISS" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS"); fi
mkdir -p "$OUT"
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pass$i" -o p -- \
      python3 tools/round_profile.py "$WL" 1 $MSGS > "$OUT/pass$i.log" 2>&1
  echo "pass $i ($grp) done"
done
