#!/bin/bash
# orient+BRIEF patch-stride A/B (round 5): SQ counters (LDS bank conflicts)
# and serial rocprofv3 averages of the shipped build and the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in base "$@"; do
  if [ $v = base ]; then unset ORBX_LIB_VARIANT; else export ORBX_LIB_VARIANT=$v; fi
  bash tools/pmc_sq.sh gpurun_out/sq_ob_$v --allow-diag > /dev/null || exit 1
  echo "== $v"; grep -A16 "orient_brief" gpurun_out/sq_ob_$v/summary.txt | grep -E "LDS_BANK|LDS_IDX|INSTS_VALU|INSTS_LDS"
done
unset ORBX_LIB_VARIANT
bash tools/variant_serial.sh ob base "$@" | grep -E "==|orient|fast_cells|pyr_band"
