# containers/checksums/file streaming tests + libdmx fixtures for the gloo tests
set -e
mkdir -p gpurun_out
timeout -k 10 120 python -u tests/golden/make_dmx_fixtures.py > gpurun_out/fix.log 2>&1 || { cat gpurun_out/fix.log; exit 1; }
mkdir -p gpurun_out/dmx && cp tests/golden/dmx/* gpurun_out/dmx/
timeout -k 10 500 python -u -m pytest tests/test_gpu_containers.py tests/test_gpu_parity.py -k "container or checksum or zlib or gzip or file or dropin" -x -v --timeout 200 --timeout-method thread > gpurun_out/cont_tests.log 2>&1 || { tail -60 gpurun_out/cont_tests.log; exit 1; }
tail -5 gpurun_out/cont_tests.log
