# PMC passes over one split-K dW GEMM (bench_gemm --only dw/s4) and the LDS-DMA
# stream micro (tools/micro/dmapat); out: gpurun_out/dwpmc/
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/dwpmc
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA"
P2="TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCC_HIT TCC_MISS"
P3="TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES TCP_UTCL1_STALL_MULTI_MISS TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/gemm_p$i -o run --output-format csv -- python3 $R/tools/bench_gemm.py --reps 20 --only dw/s4 > $O/gemm_p$i.log 2>&1 || { echo FAIL gemm $i; tail -20 $O/gemm_p$i.log; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc $P -d $O/dma_p$i -o run --output-format csv -- $R/tools/micro/dmapat > $O/dma_p$i.log 2>&1 || { echo FAIL dma $i; tail -20 $O/dma_p$i.log; exit 1; }
done
echo PMC_OK
