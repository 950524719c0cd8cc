#!/bin/bash
# PMC counters per hot kernel (two passes: SQ/GRBM, then TCC bytes), kernel-trace only —
# never combined with sys/runtime traces. Output: gpurun_out/pmc_{sq,tcc}/.
set -e
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
  -- python3 tools/kernel_zoo.py
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_tcc -o run \
  --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- python3 tools/kernel_zoo.py
