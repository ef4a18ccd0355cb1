# A/B aid: build the working tree's libdmx.so with extra -D flags into ab/libdmx_<name>.so
# usage: bash tools/ab_variant.sh <name> "-DFOO=0 -DBAR=1"
set -e
name=$1; flags=$2
rm -rf /tmp/abv_$name && mkdir -p /tmp/abv_$name
cp -r deflate.hpp_amd include /tmp/abv_$name/
rm -rf /tmp/abv_$name/deflate.hpp_amd/build /tmp/abv_$name/deflate.hpp_amd/lib
make -C /tmp/abv_$name/deflate.hpp_amd -s -j8 HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $flags" > /dev/null
mkdir -p ab && cp /tmp/abv_$name/deflate.hpp_amd/lib/libdmx.so ab/libdmx_$name.so
echo built ab/libdmx_$name.so
