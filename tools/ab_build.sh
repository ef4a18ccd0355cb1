# A/B aid: build libdmx.so of a git ref into ab/libdmx_<name>.so (run here, not on the GPU box)
# usage: bash tools/ab_build.sh <ref> <name>
set -e
ref=$1; name=$2
rm -rf /tmp/abbuild && mkdir -p /tmp/abbuild
git archive "$ref" deflate.hpp_amd include | tar -x -C /tmp/abbuild
make -C /tmp/abbuild/deflate.hpp_amd -s -j8 > /dev/null
mkdir -p ab && cp /tmp/abbuild/deflate.hpp_amd/lib/libdmx.so ab/libdmx_$name.so
echo built ab/libdmx_$name.so
