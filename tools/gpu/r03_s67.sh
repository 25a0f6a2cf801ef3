set -o pipefail
bash tools/gpu/r03_s7.sh || exit 1
bash tools/gpu/r03_s6.sh || exit 1
