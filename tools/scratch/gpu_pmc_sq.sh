# SQ issue/stall counters of one c4 broadcast (3 passes: SQ cycles, SQ instruction counts,
# TLB / L2) and a per-dispatch report for one kernel.
#   bash tools/gpu_pmc_sq.sh <tag> [kernel-name-substring]
set -o pipefail
tag=${1:-sq}
K=${2:-k_gossip_fused}
bash tools/pmc_passes.sh c4 gpurun_out/pmc_$tag \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
  "TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCC_HIT TCC_MISS" || exit 1
cd tools || exit 1
python3 pmc_sq_report.py ../gpurun_out/pmc_$tag "$K" > ../gpurun_out/pmc_$tag/report_sq.txt || exit 1
python3 pmc_report.py ../gpurun_out/pmc_$tag > ../gpurun_out/pmc_$tag/report.txt || exit 1
cat ../gpurun_out/pmc_$tag/report_sq.txt
