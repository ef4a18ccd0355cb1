# A/B: 16 vs 32 segments per wave in the lane decoder
set -e
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed 2 > gpurun_out/ab16.txt 2>&1
DMX_LIB=$PWD/build_ab/libdmx32.so timeout -k 10 200 python -u tools/kernel_times.py 1024 repeat,text,mixed 2 > gpurun_out/ab32.txt 2>&1
cat gpurun_out/ab16.txt gpurun_out/ab32.txt
