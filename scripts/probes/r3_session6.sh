set -o pipefail
echo "== market"; TILES=47,42,52 timeout -k 10 120 python scripts/probes/dist_tiled_probe.py || exit 1
echo "== 1M shard"; SHAPE=10000,125000,2048 TILES=47,42 timeout -k 10 180 python scripts/probes/dist_tiled_probe.py || exit 1
