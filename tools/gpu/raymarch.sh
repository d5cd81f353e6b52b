# ray-march kernel alone (bench.ray_march: 4 M random rays) and the LOS table build
set -o pipefail
timeout -k 10 120 python -c "
import bench, json
print(json.dumps(bench.ray_march()))
" || exit 1
