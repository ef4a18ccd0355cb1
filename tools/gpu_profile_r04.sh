# Round-4 evidence in one GPU call: rocprofv3 kernel stats of the third-party streams path 5
# takes (with the reference's 1-core inflate beside each), then tools/profile_all.sh (per-corpus
# kernel stats + PMC traffic).  Results under gpurun_out/; `bash tools/profile_all.sh collect r04`
# and the cp lines at the end of this file's usage note copy them into profiles/.
# usage: gpurun -- 'bash tools/gpu_profile_r04.sh'   (FOREIGN=0 / CORPORA=0 skip a part)
set -e
mkdir -p gpurun_out/r04 && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "${FOREIGN:-1}" = 1 ]; then
  for spec in bmp:0:1 text:1024:1 zeros:256:1 zfixed:text:64 single:text:16 mixed:256:6; do
    tag=$(echo $spec | tr ':' '_')
    rm -rf gpurun_out/r04/fs_$tag
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04/fs_$tag --output-format csv -- \
      python3 tools/foreign_probe.py $spec --ref > gpurun_out/r04/fs_$tag.txt 2>&1
    grep -v amdgpu.ids gpurun_out/r04/fs_$tag.txt
  done
fi
if [ "${CORPORA:-1}" = 1 ]; then
  bash tools/profile_all.sh run > gpurun_out/r04/profile_all.log 2>&1 || { tail -20 gpurun_out/r04/profile_all.log; exit 1; }
  tail -12 gpurun_out/r04/profile_all.log
fi
