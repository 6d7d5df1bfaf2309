set -o pipefail
TAG=r02_d PMC=1 STAMPS=1 bash tools/gpu_round.sh || exit 1
bash tools/bench_configs.sh r02_d_configs || exit 1
