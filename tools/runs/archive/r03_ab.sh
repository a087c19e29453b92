set -o pipefail
bash tools/r03_b.sh || exit 1
bash tools/r03_a.sh || exit 1
