# Round-6 GPU check, part E: 64 KiB lanes at 32 segments per wave + split-half resolve, 1 GiB.
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r6e_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6e_prof --output-format csv -- python3 tools/c4_probe.py mixed 1024 > gpurun_out/r6e_probe.txt 2>&1; rc=$?
cat gpurun_out/r6e_probe.txt | grep seg=
python3 tools/kstat_brief.py gpurun_out/r6e_prof/runc/*_kernel_stats.csv | head -8
exit $rc
