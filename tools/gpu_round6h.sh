# Round-6 check (developer aid): GPU tests, resolve A/B ($LIBS) and path-5 A/B (base vs ra0).
set -e
mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LIBS="${LIBS:-old prev base}" bash tools/gpu_ab.sh > gpurun_out/ab_rs.log 2>&1
LIBS="base ra0" SPECS="bmp:0:1 text:64:1 mixed:32:6" bash tools/gpu_ab_p5.sh > gpurun_out/ab_p5.log 2>&1
