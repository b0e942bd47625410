# SQ / LDS counters for the fused multi-relation forward (development helper)
cd "${GRAFT_REPO_ROOT:-.}" && export TMPDIR=/tmp && mkdir -p gpurun_out/pm
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE" "TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  n=$(echo $grp | cut -c1-12 | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pm/$n -o x --output-format csv -- python3 bench.py --graph proteins --relations 8 --steps 2 --warmup 1 > gpurun_out/pm/$n.log 2>&1 || exit $?
done
