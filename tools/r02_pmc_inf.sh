# PMC counters of the inflate kernels (lanes / resolve) on repeat and text, plus phases
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pi1_* gpurun_out/pi2_*
for k in repeat text; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pi1_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 1 > /dev/null 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_SMEM -d gpurun_out/pi2_$k --output-format csv -- python3 tools/deflate_once.py $k 256 2 1 > /dev/null 2>&1
python tools/pmc_sum.py gpurun_out/pi1_$k k_inflate > gpurun_out/pmci_$k.json
python tools/pmc_sum.py gpurun_out/pi2_$k k_inflate >> gpurun_out/pmci_$k.json
done
cat gpurun_out/pmci_repeat.json gpurun_out/pmci_text.json
rm -f gpurun_out/phases.txt
DMX_KINDS=repeat,text timeout -k 10 200 python tools/phases.py gpurun_out/phases.txt > /dev/null 2>&1
cat gpurun_out/phases.txt
