set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc1 --output-format csv -- python3 tests/dev_one.py repeat 256 2 1 > gpurun_out/pmc1.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU -d gpurun_out/pmc2 --output-format csv -- python3 tests/dev_one.py repeat 256 2 1 > gpurun_out/pmc2.txt 2>&1
