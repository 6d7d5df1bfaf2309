set -o pipefail
TAG=${TAG:-r02_e} PMC=1 STAMPS=1 bash tools/gpu_round.sh || exit 1
bash tools/bench_configs.sh ${TAG:-r02_e}_configs || exit 1
