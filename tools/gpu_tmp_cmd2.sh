mkdir -p gpurun_out
timeout -k 10 120 python tools/setup_ts.py > gpurun_out/setup_ts_r03.txt 2>&1; tail -12 gpurun_out/setup_ts_r03.txt
bash tools/gpu_pmc_grad.sh g1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA" > gpurun_out/pmc_g1.txt 2>&1; tail -60 gpurun_out/pmc_g1.txt
