bash tools/gpu/round_check.sh || exit 1
bash tools/gpu/skip_ab.sh "--workload config4" 0 256 1048576 65536 1049088 || exit 2
bash tools/gpu/skip_ab.sh "--spawns melee" 0 256 1048576 65536 || exit 3
