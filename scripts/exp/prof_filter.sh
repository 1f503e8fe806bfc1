cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/exp/steady_step.py 1 4 > gpurun_out/steady_step_r6t.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r6t -o run --output-format csv -- python3 scripts/exp/steady_step.py 1 3 > gpurun_out/prof_r6t.log 2>&1 || exit 2
CMD="scripts/exp/steady_step.py 1 2" TAG=ft PASSES="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY;SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_LDS_ADDR_CONFLICT,SQ_INST_LEVEL_LDS,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VALU,SQ_INSTS_VMEM_RD,SQ_INST_LEVEL_VMEM" bash scripts/gpu_pmc_cmd.sh
