# developer A/B of the workgroup serial decoder's walk parameters (tools/serial_probe.py)
set -e
for cfg in "128 24" "160 24" "192 32" "128 32"; do
  set -- $cfg
  echo "== warm $1 rounds $2"
  DMX_SERIAL_WARM=$1 DMX_SERIAL_ROUNDS=$2 timeout -k 10 200 python -u tools/serial_probe.py 2>&1 | grep -E "MB/s"
done
