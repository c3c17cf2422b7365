# PMC of the bf16 weight gradient: LDS-DMA loop vs register-staged loop (one counter set per pass)
set -o pipefail
export TMPDIR=/tmp
export PROBE_ORDER=a
for dma in 1 0; do
  SDML_WGRAD_DMA=$dma tools/gpu.sh pmc wgpmc_mfma_$dma "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVES" python tools/probes/wgrad_bias_probe.py || exit 1
  SDML_WGRAD_DMA=$dma tools/gpu.sh pmc wgpmc_lds_$dma "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" python tools/probes/wgrad_bias_probe.py || exit 1
done
