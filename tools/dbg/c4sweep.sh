set -u
for cfg in "65536 2" "32768 0.5" "16384 0.25" "8192 0"; do
  set -- $cfg
  echo "== min $1 share $2"
  SDZ_SPLIT_DEBUG=1 SDZ_SPLIT_MIN=$1 SDZ_SPLIT_SHARE=$2 timeout -k 10 200 python3 tools/run_configs.py --config c4 --scale 8 2>&1 | grep -E "sdz split|inflate:|kernel_ms" | cut -c1-240 || exit 1
done
