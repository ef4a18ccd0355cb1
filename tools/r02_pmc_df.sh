# PMC counters of the deflate kernel on repeat and text (256 MiB, level 2)
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pd1_* gpurun_out/pd2_* gpurun_out/pd3_*
for k in repeat text; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pd1_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 0 > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SMEM -d gpurun_out/pd2_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 0 > /dev/null 2>&1
python tools/pmc_sum.py gpurun_out/pd1_$k k_deflate > gpurun_out/pmcd_$k.json
python tools/pmc_sum.py gpurun_out/pd2_$k k_deflate >> gpurun_out/pmcd_$k.json
done
timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS -d gpurun_out/pd3_repeat --output-format csv -- python3 tools/deflate_once.py repeat 256 2 0 > gpurun_out/pd3.log 2>&1 && python tools/pmc_sum.py gpurun_out/pd3_repeat k_deflate > gpurun_out/pmcd3.json
cat gpurun_out/pmcd_repeat.json gpurun_out/pmcd_text.json gpurun_out/pmcd3.json
