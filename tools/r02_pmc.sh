set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in repeat text; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc1_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU -d gpurun_out/pmc2_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 > /dev/null 2>&1
python tools/pmc_sum.py gpurun_out/pmc1_$k k_deflate > gpurun_out/pmc_$k.json
python tools/pmc_sum.py gpurun_out/pmc2_$k k_deflate >> gpurun_out/pmc_$k.json
done
cat gpurun_out/pmc_repeat.json gpurun_out/pmc_text.json
